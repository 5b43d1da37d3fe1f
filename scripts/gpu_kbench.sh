#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_encoder.py -m gpu -q -x > gpurun_out/pytest_enc.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_enc.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python scripts/kbench.py all > gpurun_out/kbench.log 2>&1
