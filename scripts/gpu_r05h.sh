# SpecAugment in place by time chunks: parity (every route), the C2 bench; then the r05g A/B + timelines
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_augment.py tests/test_augment_draws.py > gpurun_out/r05h_aug.log 2>&1 && \
timeout -k 10 120 python scripts/sa_time.py > gpurun_out/r05h_sa_time.log 2>&1 && \
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > gpurun_out/r05h_bench_c2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05h_prof_c2 -o run -- python bench.py --config c2 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r05h_prof_c2.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r05h_aug.log | tail -5
cat gpurun_out/r05h_sa_time.log
tail -1 gpurun_out/r05h_bench_c2.log | cut -c1-1500
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_r05g.sh
