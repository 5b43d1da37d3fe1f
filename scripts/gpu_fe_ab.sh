#!/bin/bash
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 200 python scripts/fe_time.py speechbrain_amd/libsbk.so gpurun_probe_*.so > gpurun_out/fe_ab.log 2>&1
