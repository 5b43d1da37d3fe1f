#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/mxpmc"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAVES -d "$R/gpurun_out/mxpmc" -o p1 --output-format csv -- python3 "$R/scripts/mx_one.py" > "$R/gpurun_out/mxpmc/p1.log" 2>&1
