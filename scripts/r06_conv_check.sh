# conv-module change: its tests, then 3 bench runs (conv / chain / attention averages)
set -u
cd /root/repo
T=$1
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_encoder.py tests/test_gpu_bench_parity.py tests/test_gpu_doctests.py -k "conv or bench or Conv or conformer" > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/${T}_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench_$i.log 2>&1 || exit $?
  python - gpurun_out/${T}_bench_$i.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
oth = {o["kernel"].split(" (")[0][:26]: o["avg_launch_us"] for o in r.get("other_kernels", [])}
print("ms", d["ms_per_step"], "chain", r["avg_launch_us"], oth)
PY
done
