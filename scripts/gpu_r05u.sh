# Persistent frontend2: parity tests that run it (features, encoder, bench parity, AMP), C3 bench, C3 kernel stats.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_encoder.py tests/test_gpu_bench_parity.py tests/test_gpu_amp.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05u_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05u_bench_c3.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05u_prof_c3 -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r05u_prof_c3.log 2>&1
rc=$?
tail -3 gpurun_out/r05u_tests.log
tail -1 gpurun_out/r05u_bench_c3.log | cut -c1-400
f=$(find gpurun_out/r05u_prof_c3 -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && grep -i "frontend2" "$f" | cut -c1-200
exit $rc
