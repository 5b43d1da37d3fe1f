# Round-5 baseline on a fresh box: GPU suite, smoke, C3 bench, C3 kernel stats.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_xattn.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r05a_xattn.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05a_gpu_tests.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05a_smoke.log 2>&1 && \
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r05a_bench_c3.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05a_prof_c3 -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r05a_prof_c3.log 2>&1
rc=$?
tail -5 gpurun_out/r05a_xattn.log
tail -2 gpurun_out/r05a_gpu_tests.log
tail -2 gpurun_out/r05a_smoke.log
tail -1 gpurun_out/r05a_bench_c3.log | cut -c1-300
exit $rc
