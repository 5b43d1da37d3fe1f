# Round-6 baseline on one box: the new tests, the full GPU suite, config-3 bench
# (default, d_model 144), and a rocprof stats pass of the default bench.
set -u
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_variants.py tests/test_gpu_doctests.py > gpurun_out/r06d_new.log 2>&1
rc=$?; echo "new tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r06d_bench_c3.log 2>&1 || exit $?
tail -1 gpurun_out/r06d_bench_c3.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --d-model 144 > gpurun_out/r06d_bench_c3_d144.log 2>&1 || exit $?
tail -1 gpurun_out/r06d_bench_c3_d144.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06d_prof_d144 -o prof -- python3 bench.py --no-cpu-baseline --d-model 144 --steps 10 > gpurun_out/r06d_prof_d144.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu --deselect tests/test_gpu_variants.py --deselect tests/test_gpu_doctests.py > gpurun_out/r06d_all.log 2>&1
echo "all rc=$?"
