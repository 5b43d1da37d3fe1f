# SpecAugment slab width with the 256-row windows: probe builds SBK_RL_JMAX = 4 / 1 (and 4 with 128-row windows) against the product's 2
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
( for r in 1 2 3; do timeout -k 10 300 python scripts/sa_time.py speechbrain_amd/libsbk.so gpurun_probe_J4.so gpurun_probe_J1.so gpurun_probe_W128J4.so || exit $?; done ) > gpurun_out/r05bn_sa_j_ab.log 2>&1
rc=$?; cat gpurun_out/r05bn_sa_j_ab.log; exit $rc
