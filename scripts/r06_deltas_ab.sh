# Same-box sweep of the concat-deltas tile height and store order (ab/libsbk_{A,T32,T128,C,C32}.so:
# 64 rows (HEAD), 32, 128; C: row-contiguous stores at 64 / 32 rows) on the config-2 bench, alternating.
set -u
cd /root/repo
for i in 1 2; do
  for v in A T16 T24; do
    cp ab/libsbk_$v.so speechbrain_amd/libsbk.so
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --config c2 > gpurun_out/r06ai_${v}_$i.log 2>&1 || exit $?
    python - gpurun_out/r06ai_${v}_$i.log $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
oth = {o["kernel"].split(" (")[0][:24]: (o["us"], o["frac"]) for o in r.get("other_kernels", [])}
print(sys.argv[2], "ms", d["ms_per_step"], "fbank", r["avg_launch_us"], oth)
PY
  done
done
cp ab/libsbk_A.so speechbrain_amd/libsbk.so
