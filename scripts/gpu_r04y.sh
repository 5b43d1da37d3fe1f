# Round-4 final tree (per-trip mel chunk counts on): Fbank time, the GPU suite, smoke, C3 and C2 bench, C3 kernel stats.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 200 python scripts/fe_time.py > gpurun_out/r04y_fe_time.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04y_gpu_tests.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04y_smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/r04y_bench_c3.log 2>&1 && \
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > gpurun_out/r04y_bench_c2.log 2>&1 && \
timeout -k 10 300 python scripts/c2_host.py > gpurun_out/r04y_c2_host.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04y_prof_c3 -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04y_prof_c3.log 2>&1
rc=$?
cat gpurun_out/r04y_fe_time.log
tail -2 gpurun_out/r04y_gpu_tests.log
tail -2 gpurun_out/r04y_smoke.log
tail -1 gpurun_out/r04y_bench_c3.log | cut -c1-300
tail -1 gpurun_out/r04y_bench_c2.log | cut -c1-400
head -3 gpurun_out/r04y_c2_host.log
exit $rc
