#!/bin/bash
# rocprofv3 kernel-trace + stats of bench_train (N=1); summaries in gpurun_out/<tag>.
# usage: scripts/profile_train.sh [tag] [bench_train args...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-prof_train}; shift
mkdir -p "$R/gpurun_out/$TAG"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$TAG" -o run --output-format csv \
  -- python3 "$R/bench_train.py" "$@" > "$R/gpurun_out/$TAG/bench_stdout.log" 2>&1
rc=$?
echo "rocprof rc=$rc" >> "$R/gpurun_out/$TAG/bench_stdout.log"
exit $rc
