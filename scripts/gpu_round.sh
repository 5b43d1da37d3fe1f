#!/bin/bash
# GPU box, round verification: full -m gpu suite, smoke, config-3 and config-2
# benches, rocprofv3 kernel stats of the config-3 bench, FETCH/WRITE_SIZE
# passes of the config-2 bench.  Stops at the first failing step.
# usage: scripts/gpu_round.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r03c}
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$O/bench_default.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 5 > "$O/bench_c2.log" 2>&1 || exit $?
bash scripts/profile.sh "$TAG/prof" --steps 20 --warmup 5 || exit $?
bash scripts/pmc_traffic.sh "$TAG/pmc_c2" --config c2 || exit $?
exit 0
