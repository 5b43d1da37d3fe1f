# fused head: tests + timing for the product build and a probe build
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_thead.py > gpurun_out/thead_tests.log 2>&1 && tail -1 gpurun_out/thead_tests.log && \
timeout -k 10 300 python scripts/thead_bench.py > gpurun_out/thead_bench.log 2>&1 && grep -v amdgpu.ids gpurun_out/thead_bench.log && \
SBK_PROBE_LIB=gpurun_probe_BN128.so timeout -k 10 400 python -u scripts/probe_pytest.py -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_thead.py > gpurun_out/thead_tests128.log 2>&1 && tail -1 gpurun_out/thead_tests128.log && \
SBK_PROBE_LIB=gpurun_probe_BN128.so timeout -k 10 300 python scripts/thead_bench.py > gpurun_out/thead_bench128.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/thead_bench128.log; exit $rc
