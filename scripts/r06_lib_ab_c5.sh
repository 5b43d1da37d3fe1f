# Same-box A/B of two builds of libsbk.so (ab/libsbk_A.so, ab/libsbk_B.so) on
# the config-5 bench: targeted GPU tests on B, then alternating benches.
# usage: bash scripts/r06_lib_ab_c5.sh <tag> [test files...]
set -u
cd /root/repo
T=$1; shift
cp ab/libsbk_B.so speechbrain_amd/libsbk.so
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread "$@" > gpurun_out/${T}_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/${T}_tests.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
for i in 1 2 3; do
  for v in A B; do
    cp ab/libsbk_$v.so speechbrain_amd/libsbk.so
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --config c5 > gpurun_out/${T}_${v}_$i.log 2>&1 || exit $?
    python - gpurun_out/${T}_${v}_$i.log $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], "ms/step", d["ms_per_step"], "mx_gemm avg us", r["avg_launch_us"], "frac", r["frac"])
PY
  done
done
cp ab/libsbk_B.so speechbrain_amd/libsbk.so
