# 256x256 GEMM bf16 + MXFP8 sweep
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 300 python scripts/g256_bench.py > gpurun_out/r05c_g256.log 2>&1 && \
timeout -k 10 300 python scripts/mx256_bench.py > gpurun_out/r05c_mx256.log 2>&1
rc=$?
grep -E "BAD|TF/s" gpurun_out/r05c_g256.log
cat gpurun_out/r05c_mx256.log
exit $rc
