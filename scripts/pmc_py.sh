#!/bin/bash
# usage: scripts/pmc_py.sh <tag> "<counters>" <script.py> [args...]
# One rocprofv3 counter pass (kernel trace only) over a Python probe script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; CTRS=$2; shift 2
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --pmc $CTRS --kernel-trace -d $R/gpurun_out/$TAG -o k --output-format csv -- python3 "$R/$@" > $R/gpurun_out/$TAG/log.txt 2>&1
