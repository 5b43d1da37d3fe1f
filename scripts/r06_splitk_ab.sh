# Same-box A/B of the MXFP8 split-K tail (gemm256.hip split_tail) on the
# config-5 bench: A = workspace withheld (whole tiles), B = default.  GPU
# tests of the 256-tile GEMMs and the wav2vec2 path first.
# usage: bash scripts/r06_splitk_ab.sh <tag>
set -u
cd /root/repo
T=$1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm256.py \
  tests/test_gpu_wav2vec.py > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/${T}_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2 3; do
  for v in A B; do
    timeout -k 10 300 python -u - $v > gpurun_out/${T}_${v}_$i.log 2>&1 <<'PY' || exit $?
import runpy, sys
if sys.argv[1] == "A":
    import speechbrain_amd._w2v as w
    w._ws_floats = lambda *a: 0
sys.argv = ["bench.py", "--no-cpu-baseline", "--config", "c5"]
runpy.run_path("bench.py", run_name="__main__")
PY
    python - gpurun_out/${T}_${v}_$i.log $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], "ms", d["ms_per_step"], "mx_gemm avg us", r["avg_launch_us"], "frac", r["frac"])
PY
  done
done
