# conv module: depthwise conv on v_dot2c_f32_bf16, LN1 frames interleaved: parity, timeline, C3 bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_encoder.py tests/test_gpu_bench_parity.py > gpurun_out/r05j_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r05j_tests.log
[ $rc -ne 0 ] && exit $rc
CM_PRE=1 SBK_PROBE_LIB=gpurun_probe_CMTL.so timeout -k 10 120 python -u scripts/cm_tl.py > gpurun_out/r05j_cm_tl.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05j_bench_c3.log 2>&1
rc=$?
cat gpurun_out/r05j_cm_tl.log
tail -1 gpurun_out/r05j_bench_c3.log | cut -c1-400
python - <<'PY'
import json
for l in open('gpurun_out/r05j_bench_c3.log'):
    if l.startswith('{'):
        d=json.loads(l)
        for k in d['roofline'].get('other_kernels',[]): print(k.get('kernel'), k.get('avg_launch_us'))
PY
exit $rc
