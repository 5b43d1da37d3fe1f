# Round 6: targeted GPU tests, then the config-3 bench at d 256 and d 144 and
# the full GPU suite.  Tag: $1 (log prefix).
set -u
cd /root/repo
T=${1:-r06x}
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_variants.py tests/test_gpu_doctests.py tests/test_gpu_bench_parity.py > gpurun_out/${T}_new.log 2>&1
rc=$?; echo "targeted tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench_c3.log 2>&1 || exit $?
tail -1 gpurun_out/${T}_bench_c3.log | cut -c1-400
timeout -k 10 300 python -u bench.py --no-cpu-baseline --d-model 144 > gpurun_out/${T}_bench_c3_d144.log 2>&1 || exit $?
tail -1 gpurun_out/${T}_bench_c3_d144.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_d144 -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --d-model 144 --steps 10 > gpurun_out/${T}_prof_d144.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu --deselect tests/test_gpu_variants.py --deselect tests/test_gpu_doctests.py --deselect tests/test_gpu_bench_parity.py > gpurun_out/${T}_all.log 2>&1
echo "all rc=$?"
tail -1 gpurun_out/${T}_all.log
