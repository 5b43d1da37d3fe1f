# config-4 training step, fused vs materialised transducer head (GPU box)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_thead.py > gpurun_out/thead_tests.log 2>&1 && tail -1 gpurun_out/thead_tests.log && \
timeout -k 10 400 python bench_train.py --steps 5 --warmup 2 > gpurun_out/c4_fused.log 2>&1 && tail -1 gpurun_out/c4_fused.log | cut -c1-700 && \
timeout -k 10 400 python bench_train.py --steps 5 --warmup 2 --head materialised > gpurun_out/c4_mat.log 2>&1; rc=$?; tail -1 gpurun_out/c4_mat.log | cut -c1-300; exit $rc
