# fast GELU epilogue (C5), C3 fp32 precision bench line, streaming deltas (C2)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm256.py tests/test_gpu_features.py tests/test_gpu_wav2vec.py -q --timeout 300 --timeout-method thread > gpurun_out/r05f_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r05f_tests.log
# a plain test failure (rc 1) does not stop the benches; a timeout / crash does
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > gpurun_out/r05f_bench_c2.log 2>&1 && \
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > gpurun_out/r05f_bench_c5_mx.log 2>&1 && \
timeout -k 10 300 python bench.py --config c5 --precision bf16 --no-cpu-baseline > gpurun_out/r05f_bench_c5_bf16.log 2>&1 && \
timeout -k 10 300 python bench.py --precision fp32 --no-cpu-baseline > gpurun_out/r05f_bench_c3_fp32.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05f_prof_c3_fp32 -o run -- python bench.py --precision fp32 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r05f_prof_c3_fp32.log 2>&1
rc2=$?
tail -1 gpurun_out/r05f_bench_c2.log | cut -c1-1200
tail -1 gpurun_out/r05f_bench_c5_mx.log | cut -c1-200
tail -1 gpurun_out/r05f_bench_c5_bf16.log | cut -c1-200
tail -1 gpurun_out/r05f_bench_c3_fp32.log
exit $rc2
