# Round 6 final check: full GPU suite, smoke, config-3 / d=144 / c2 / c5
# benches, rocprof kernel stats of the config-3 bench, FETCH/WRITE_SIZE
# passes of it.  Stops at the first failing step.
set -u
cd /root/repo
T=${1:-r06z}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -5 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $O/bench_c3.log 2>&1 || exit $?
tail -1 $O/bench_c3.log | cut -c1-200
timeout -k 10 300 python -u bench.py --no-cpu-baseline --d-model 144 > $O/bench_c3_d144.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --config c2 > $O/bench_c2.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --config c5 > $O/bench_c5.log 2>&1 || exit $?
bash scripts/profile.sh $T/prof --steps 20 --warmup 5 || exit $?
bash scripts/pmc_traffic.sh $T/pmc_c3 || exit $?
echo done
