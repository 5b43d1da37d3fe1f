#!/bin/bash
# rocprofv3 kernel-trace + stats of the bench (N=1); summaries land in gpurun_out/prof.
# usage: scripts/profile.sh [tag] [bench args...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-prof}; shift
mkdir -p "$R/gpurun_out/$TAG"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$TAG" -o run --output-format csv \
  -- python3 "$R/bench.py" --no-cpu-baseline "$@" > "$R/gpurun_out/$TAG/bench_stdout.log" 2>&1
rc=$?
echo "rocprof rc=$rc" >> "$R/gpurun_out/$TAG/bench_stdout.log"
exit $rc
