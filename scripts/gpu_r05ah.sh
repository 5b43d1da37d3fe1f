# frontend2, block 2 beside the previous tile's epilogue: A/B vs the previous commit, then the parity tests that run it (no -x)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
bash scripts/fe_ab.sh r05ah_fe_overlap_ab.log gpurun_probe_HEADFE.so > /dev/null && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_encoder.py tests/test_gpu_bench_parity.py tests/test_gpu_amp.py tests/test_gpu_dropin.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r05ah_tests.log 2>&1
rc=$?; cat gpurun_out/r05ah_fe_overlap_ab.log; grep -E "FAILED|passed|failed" gpurun_out/r05ah_tests.log | tail -8; exit $rc
