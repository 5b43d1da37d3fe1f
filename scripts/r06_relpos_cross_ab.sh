set -u
cd /root/repo
cp ab/libsbk_B.so speechbrain_amd/libsbk.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_xattn.py tests/test_gpu_mha_general.py tests/test_gpu_variants.py tests/test_gpu_doctests.py tests/test_gpu_recipe.py > gpurun_out/r06ab_tests.log 2>&1 || { tail -30 gpurun_out/r06ab_tests.log; exit 1; }
tail -1 gpurun_out/r06ab_tests.log
for v in A B A B; do cp ab/libsbk_$v.so speechbrain_amd/libsbk.so; echo "== $v"; timeout -k 10 120 python -u scripts/relpos_cross_timing.py 2>&1 | grep -v amdgpu.ids; done
cp ab/libsbk_B.so speechbrain_amd/libsbk.so
