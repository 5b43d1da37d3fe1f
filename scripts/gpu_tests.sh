#!/bin/bash
# GPU box: full -m gpu suite, then the bench (N=1), each under its own limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
rc2=$?
echo "bench rc=$rc2" >> gpurun_out/bench.log
[ $rc -eq 0 ] && exit $rc2
exit $rc
