# frontend2 one-pass LN stats, per-utterance floor: parity tests, timing, probe timeline, SQ counters
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_encoder.py tests/test_gpu_bench_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05aa_tests.log 2>&1 && \
timeout -k 10 120 python scripts/fe_probe.py > gpurun_out/r05aa_fe.log 2>&1 && \
SBK_PROBE_TL=1 SBK_PROBE_LIB=gpurun_probe_FETL.so timeout -k 10 120 python scripts/fe_probe.py > gpurun_out/r05aa_fe_tl.log 2>&1 && \
bash scripts/fe_pmc.sh
rc=$?; tail -1 gpurun_out/r05aa_tests.log; cat gpurun_out/r05aa_fe.log gpurun_out/r05aa_fe_tl.log | grep -v amdgpu.ids; exit $rc
