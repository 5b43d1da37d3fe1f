# Round 6: preamble overlap (key padding mask + linear_pos GEMM on a side
# stream beside the src Linear) and the padded src Linear at d = 144:
# targeted GPU tests, then same-box A/B of SBK_AB_OVERLAP at d = 256 and 144.
set -u
cd /root/repo
T=${1:-r06o}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bench_parity.py tests/test_gpu_encoder.py tests/test_gpu_variants.py tests/test_gpu_doctests.py tests/test_gpu_trace.py tests/test_gpu_recipe.py > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/${T}_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/r06_ab_env.sh ${T}_ab SBK_AB_OVERLAP 0 1 || exit $?
bash scripts/r06_ab_env.sh ${T}_ab144 SBK_AB_OVERLAP 0 1 "--d-model 144" || exit $?
