#!/bin/bash
# HBM traffic per launch of the bench's kernels: two rocprofv3 counter passes
# (FETCH_SIZE, then WRITE_SIZE; they cannot share a pass), kernel trace only.
# usage: scripts/pmc_traffic.sh <tag> [bench args]  -> gpurun_out/<tag>_{fetch,write}/k_counter_collection.csv
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc_traffic}
shift
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  D="$R/gpurun_out/${TAG}_$(echo $C | cut -d_ -f1 | tr A-Z a-z)"
  mkdir -p "$D"
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d "$D" -o k --output-format csv \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-graph --no-cpu-baseline "$@" > "$D/log.txt" 2>&1 || exit $?
done
