#!/bin/bash
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/feat_tests.log 2>&1
