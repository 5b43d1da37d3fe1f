# Round-4 check: new parity tests, stream probe, chain A/B, bench (never the product).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_recipe.py \
  tests/test_gpu_train.py::test_layernorm_wide_rows tests/test_gpu_features.py::test_fbank_misaligned_view \
  tests/test_gpu_gemm_tn.py::test_wgrad_bf16_strided_operands tests/test_gpu_ddp.py > gpurun_out/r04a_tests.log 2>&1 && \
timeout -k 10 150 python -u scripts/stream_probe.py > gpurun_out/stream_probe3.log 2>&1 && \
timeout -k 10 200 python scripts/chain_time.py speechbrain_amd/libsbk.so gpurun_probe_CONTIG.so > gpurun_out/chain_time.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r04a_bench.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r04a_tests.log | tail -8
cat gpurun_out/stream_probe3.log gpurun_out/chain_time.log 2>/dev/null
tail -1 gpurun_out/r04a_bench.log 2>/dev/null | cut -c1-300
exit $rc
