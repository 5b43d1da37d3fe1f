# SpecAugment roll4 window size A/B (probe builds window / ring sizes against the product 512 / 1024)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
( for r in 1 2 3; do timeout -k 10 300 python scripts/sa_time.py speechbrain_amd/libsbk.so gpurun_probe_W256R1024.so gpurun_probe_W128R1024.so gpurun_probe_W256R512.so gpurun_probe_W128R512.so || exit $?; done ) > gpurun_out/r05bh_sa_wr_ab.log 2>&1
rc=$?; cat gpurun_out/r05bh_sa_wr_ab.log; exit $rc
