#!/bin/bash
# GPU box: GEMM tile sweep of the config-3 shapes, then the round verification.
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 240 python scripts/gemm_shapes_sweep.py > gpurun_out/gemm_shapes.log 2>&1 || exit $?
bash scripts/gpu_round.sh ${1:-r03d}
