# frontend2 block-2 software pipelining: parity tests, timing, probe timeline, SQ counters
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_encoder.py tests/test_gpu_bench_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05ab_tests.log 2>&1 && \
timeout -k 10 120 python scripts/fe_probe.py > gpurun_out/r05ab_fe.log 2>&1 && \
SBK_PROBE_TL=1 SBK_PROBE_LIB=gpurun_probe_FETL.so timeout -k 10 120 python scripts/fe_probe.py > gpurun_out/r05ab_fe_tl.log 2>&1
rc=$?; tail -1 gpurun_out/r05ab_tests.log; cat gpurun_out/r05ab_fe.log gpurun_out/r05ab_fe_tl.log | grep -v amdgpu.ids; exit $rc
