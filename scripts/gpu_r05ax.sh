# frontend2 with the 16-lane A-fragment swizzle: A/B vs the previous commit, then the parity tests that run it
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
bash scripts/fe_ab.sh r05ax_fe_aswz_ab.log gpurun_probe_HEADFE.so > /dev/null && \
timeout -k 10 500 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_encoder.py tests/test_gpu_bench_parity.py tests/test_gpu_amp.py tests/test_gpu_dropin.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r05ax_tests.log 2>&1
rc=$?; cat gpurun_out/r05ax_fe_aswz_ab.log; grep -E "FAILED|passed|failed" gpurun_out/r05ax_tests.log | tail -5; exit $rc
