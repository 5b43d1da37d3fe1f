# fused transducer head tests on the GPU box
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_thead.py > gpurun_out/thead_tests.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|error|err |peak|assert" gpurun_out/thead_tests.log | head -60; tail -3 gpurun_out/thead_tests.log; exit $rc
