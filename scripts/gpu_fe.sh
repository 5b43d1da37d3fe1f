#!/bin/bash
# GPU box: feature-kernel parity tests, A/B kernel timing, then the C2 and C3 benches.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_bench_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/fe_pytest.log 2>&1 || exit $?
timeout -k 10 200 python scripts/fe_time.py speechbrain_amd/libsbk.so gpurun_probe_*.so > gpurun_out/fe_ab.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 5 > gpurun_out/fe_c2.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/fe_c3.log 2>&1 || exit $?
[ -f gpurun_probe_TL.so ] && SBK_PROBE_LIB=gpurun_probe_TL.so timeout -k 10 120 python scripts/rf_tl.py > gpurun_out/rf_tl.log 2>&1
exit 0
