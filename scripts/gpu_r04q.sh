# Final tree check after the fast-path version bump: the whole GPU suite, smoke, the default bench.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04q_gpu_tests.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04q_smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/r04q_bench_c3.log 2>&1 && \
bash scripts/gpu_r04r.sh
rc=$?
tail -2 gpurun_out/r04q_gpu_tests.log
tail -2 gpurun_out/r04q_smoke.log
tail -1 gpurun_out/r04q_bench_c3.log | cut -c1-300
exit $rc
