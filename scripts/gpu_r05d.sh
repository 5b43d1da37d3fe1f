# 256x256 GEMMs wired into config 5: w2v / gemm GPU tests, C5 bench both precisions, C3 bench, C5 kernel stats
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_wav2vec.py tests/test_gpu_gemm_tn.py tests/test_gpu_xattn.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05d_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > gpurun_out/r05d_bench_c5_mx.log 2>&1 && \
timeout -k 10 300 python bench.py --config c5 --precision bf16 --no-cpu-baseline > gpurun_out/r05d_bench_c5_bf16.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05d_bench_c3.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05d_prof_c5 -o run -- python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r05d_prof_c5.log 2>&1
rc=$?
tail -3 gpurun_out/r05d_tests.log
tail -1 gpurun_out/r05d_bench_c5_mx.log | cut -c1-600
tail -1 gpurun_out/r05d_bench_c5_bf16.log | cut -c1-600
tail -1 gpurun_out/r05d_bench_c3.log | cut -c1-300
exit $rc
