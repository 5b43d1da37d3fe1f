# Round-5 final check (bank-model layouts, batched Fbank table stage, 256-row SpecAugment windows): the whole GPU suite, smoke, C3 (with its CPU baseline), C2, C5, rocprofv3 kernel
# stats of C3 and the HBM traffic passes of the C3 step.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05bj_gpu_tests.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05bj_smoke.log 2>&1 && \
timeout -k 10 500 python bench.py > gpurun_out/r05bj_bench_c3.log 2>&1 && \
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > gpurun_out/r05bj_bench_c2.log 2>&1 && \
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > gpurun_out/r05bj_bench_c5.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05bj_prof_c3 -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r05bj_prof_c3.log 2>&1 && \
bash scripts/pmc_traffic.sh r05bj_pmc_c3
rc=$?
tail -2 gpurun_out/r05bj_gpu_tests.log
tail -2 gpurun_out/r05bj_smoke.log
tail -1 gpurun_out/r05bj_bench_c3.log | cut -c1-600
tail -1 gpurun_out/r05bj_bench_c2.log | cut -c1-300
tail -1 gpurun_out/r05bj_bench_c5.log | cut -c1-300
exit $rc
