# Round-end check of the rebuilt library: smoke, the feature / augment / bench-parity GPU tests, the default bench.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04ab_smoke.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_augment.py tests/test_gpu_features.py tests/test_gpu_bench_parity.py > gpurun_out/r04ab_tests.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/r04ab_bench_c3.log 2>&1
rc=$?
tail -2 gpurun_out/r04ab_smoke.log
tail -1 gpurun_out/r04ab_tests.log
tail -1 gpurun_out/r04ab_bench_c3.log | cut -c1-250
exit $rc
