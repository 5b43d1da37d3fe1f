# attention with lazy softmax rescaling: A/B vs the previous commit (alternating, 3 rounds), then the attention /
# encoder / bench parity tests
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && : > gpurun_out/r05au_att_ab.log && \
for r in 1 2 3; do for lib in speechbrain_amd/libsbk.so gpurun_probe_HEADAT.so; do echo -n "$lib: " >> gpurun_out/r05au_att_ab.log; SBK_PROBE_LIB=$lib timeout -k 10 120 python scripts/att_time.py 2>/dev/null | tail -1 >> gpurun_out/r05au_att_ab.log || exit $?; done; done && \
timeout -k 10 500 python -u -m pytest tests/test_gpu_encoder.py tests/test_gpu_bench_parity.py tests/test_gpu_mha_general.py tests/test_gpu_xattn.py tests/test_gpu_wav2vec.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r05au_tests.log 2>&1
rc=$?; cat gpurun_out/r05au_att_ab.log; grep -E "FAILED|passed|failed" gpurun_out/r05au_tests.log | tail -5; exit $rc
