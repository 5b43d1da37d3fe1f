# Eager fast path for the sbk custom ops (no dispatcher outside tracing) + C2 host fixes: the whole GPU suite,
# smoke, C2 / C3 benches, C3 kernel stats.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04j_gpu_tests.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04j_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --config c2 > gpurun_out/r04j_bench_c2.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r04j_bench_c3.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04j_prof_c3 -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04j_prof_c3.log 2>&1 && \
bash scripts/gpu_r04k.sh
rc=$?
tail -3 gpurun_out/r04j_gpu_tests.log
tail -2 gpurun_out/r04j_smoke.log
tail -1 gpurun_out/r04j_bench_c2.log | cut -c1-300
tail -1 gpurun_out/r04j_bench_c3.log | cut -c1-300
exit $rc
