# frontend2 (scalar row offsets, rsqrt): the parity tests that run it + C3 bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_encoder.py tests/test_gpu_bench_parity.py tests/test_gpu_amp.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05ae_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05ae_bench_c3.log 2>&1
rc=$?; tail -1 gpurun_out/r05ae_tests.log; tail -1 gpurun_out/r05ae_bench_c3.log | cut -c1-250; exit $rc
