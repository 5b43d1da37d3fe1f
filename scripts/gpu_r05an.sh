# Fbank with the next block's span issued before the stores: feature parity tests, then per-launch Fbank time
# of the product library against the previous commit's build (alternating, 3 rounds)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_recipe.py tests/test_gpu_bench_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05an_tests.log 2>&1 && \
for r in 1 2 3; do timeout -k 10 200 python scripts/fe_time.py speechbrain_amd/libsbk.so gpurun_probe_HEADFB.so >> gpurun_out/r05an_fb_ab.log 2>&1 || exit $?; done
rc=$?; tail -1 gpurun_out/r05an_tests.log; grep -v amdgpu gpurun_out/r05an_fb_ab.log | tail -12; exit $rc
