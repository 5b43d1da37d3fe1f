#!/bin/bash
# GPU-box check: parity tests, then (only if no crash) the bench.
# usage: scripts/gpu_check.sh [pytest-args...]
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x "$@" > gpurun_out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1
rc2=$?
echo "bench rc=$rc2" >> gpurun_out/bench.log
exit $rc2
