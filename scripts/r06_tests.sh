set -u
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_variants.py tests/test_gpu_doctests.py > gpurun_out/r06c_new.log 2>&1
rc=$?
echo "new tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu --deselect tests/test_gpu_variants.py --deselect tests/test_gpu_doctests.py > gpurun_out/r06c_all.log 2>&1
echo "all rc=$?"
