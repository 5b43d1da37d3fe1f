# frontend2 K-split block 2: parity tests that run it, product timing, probe timeline, C3 bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_encoder.py tests/test_gpu_bench_parity.py tests/test_gpu_amp.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05w_tests.log 2>&1 && \
timeout -k 10 120 python scripts/fe_probe.py > gpurun_out/r05w_fe.log 2>&1 && \
SBK_PROBE_TL=1 SBK_PROBE_LIB=gpurun_probe_FETL.so timeout -k 10 120 python scripts/fe_probe.py > gpurun_out/r05w_fe_tl.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05w_bench_c3.log 2>&1
rc=$?; tail -2 gpurun_out/r05w_tests.log; cat gpurun_out/r05w_fe.log gpurun_out/r05w_fe_tl.log | grep -v amdgpu.ids; tail -1 gpurun_out/r05w_bench_c3.log | cut -c1-300; exit $rc
