#!/bin/bash
# config-5 bench (MXFP8 and bf16) + rocprofv3 kernel stats of the MXFP8 run
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/c5prof
timeout -k 10 400 python bench.py --config c5 --steps 5 --warmup 2 > gpurun_out/c5_mx.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --config c5 --precision bf16 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/c5_bf16.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/c5prof" -o run --output-format csv \
  -- python3 "$R/bench.py" --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-graph > "$R/gpurun_out/c5prof/stdout.log" 2>&1
