# 256x256 GEMM: correctness + shape sweep
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 300 python scripts/g256_bench.py > gpurun_out/r05b_g256.log 2>&1
rc=$?
cat gpurun_out/r05b_g256.log | tail -60
exit $rc
