# FFN kernel checks + timing on the GPU box (never the product).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_encoder.py -k "ffn" > gpurun_out/ffn_tests.log 2>&1 && \
timeout -k 10 120 python scripts/kbench.py ffn > gpurun_out/ffn_kbench.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_bench_parity.py > gpurun_out/ffn_parity.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/ffn_bench.log 2>&1; rc=$?; tail -3 gpurun_out/ffn_tests.log; cat gpurun_out/ffn_kbench.log; tail -3 gpurun_out/ffn_parity.log; tail -1 gpurun_out/ffn_bench.log | cut -c1-400; exit $rc
