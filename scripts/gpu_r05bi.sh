# SpecAugment with 256-row windows: augment GPU tests (in-place / copy / scalar routes vs the oracle), C2 line
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_augment.py tests/test_gpu_features.py tests/test_gpu_bench_parity.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r05bi_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > gpurun_out/r05bi_bench_c2.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" gpurun_out/r05bi_tests.log | tail -3; tail -1 gpurun_out/r05bi_bench_c2.log | cut -c1-300; exit $rc
