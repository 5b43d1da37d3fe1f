#!/bin/bash
# GPU box: feature parity tests, then per-launch Fbank time of the product library against probe builds
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fe_pytest.log 2>&1 || exit $?
timeout -k 10 200 python scripts/fe_time.py speechbrain_amd/libsbk.so gpurun_probe_*.so > gpurun_out/fe_ab.log 2>&1
