# Image-stream FFN kernel + in-place SpecAugment: parity + timing (never the product).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_encoder.py \
  -k "ffn or chain or image or encoder" > gpurun_out/r04d_tests.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_augment.py > gpurun_out/r04d_aug.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu tests/test_gpu_bench_parity.py > gpurun_out/r04d_parity.log 2>&1 && \
timeout -k 10 200 python scripts/chain_time.py speechbrain_amd/libsbk.so > gpurun_out/r04d_chain.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r04d_bench.log 2>&1 && \
timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 5 > gpurun_out/r04d_bench_c2.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r04d_tests.log gpurun_out/r04d_aug.log gpurun_out/r04d_parity.log | tail -8
cat gpurun_out/r04d_chain.log 2>/dev/null
tail -1 gpurun_out/r04d_bench.log 2>/dev/null | cut -c1-300
tail -1 gpurun_out/r04d_bench_c2.log 2>/dev/null | cut -c1-1500
exit $rc
