# concat-deltas (deferred floor) time-tile A/B: probe builds SBK_DT_TILE = 16 / 32 / 128 against the product's 64
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
( for r in 1 2 3; do for lib in speechbrain_amd/libsbk.so gpurun_probe_DT16.so gpurun_probe_DT32.so gpurun_probe_DT128.so; do echo -n "$lib "; SBK_PROBE_LIB=$lib timeout -k 10 120 python scripts/dt_time.py 2>/dev/null || exit $?; done; done ) > gpurun_out/r05bk_dt_ab.log 2>&1
rc=$?; cat gpurun_out/r05bk_dt_ab.log; exit $rc
