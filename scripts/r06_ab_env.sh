# Same-box A/B of an environment switch on the config-3 bench (alternating
# runs): $1 tag, $2 variable, $3 value A, $4 value B, [$5 extra bench args]
set -u
cd /root/repo
T=$1; V=$2; A=$3; Bv=$4; X=${5:-}
for i in 1 2 3; do
  for val in $A $Bv; do
    env $V=$val timeout -k 10 300 python -u bench.py --no-cpu-baseline $X > gpurun_out/${T}_${val}_$i.log 2>&1 || exit $?
    python - gpurun_out/${T}_${val}_$i.log $V=$val <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
oth = {o["kernel"].split(" (")[0][:28]: o["avg_launch_us"] for o in r.get("other_kernels", [])}
print(sys.argv[2], "ms", d["ms_per_step"], "chain", r["avg_launch_us"], oth)
PY
  done
done
