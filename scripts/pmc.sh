#!/bin/bash
# usage: scripts/pmc.sh <tag> <kbench-mode> "<counters>"
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; MODE=$2; CTRS=$3
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --pmc $CTRS --kernel-trace -d $R/gpurun_out/$TAG -o k --output-format csv -- python3 $R/scripts/kbench.py $MODE > $R/gpurun_out/$TAG/log.txt 2>&1
