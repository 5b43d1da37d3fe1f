# Fbank table stage with batched loads: feature parity tests, same-box A/B against the previous commit, the C2 and C3 lines
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_bench_parity.py tests/test_gpu_encoder.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r05bc_tests.log 2>&1 && \
( for r in 1 2 3; do for lib in speechbrain_amd/libsbk.so gpurun_probe_HEADFB.so; do echo -n "$lib "; SBK_PROBE_LIB=$lib timeout -k 10 120 python scripts/spec_probe.py 32 2>/dev/null || exit $?; done; done ) > gpurun_out/r05bc_ab.log 2>&1 && \
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > gpurun_out/r05bc_bench_c2.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05bc_bench_c3.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" gpurun_out/r05bc_tests.log | tail -3; cat gpurun_out/r05bc_ab.log; tail -1 gpurun_out/r05bc_bench_c2.log | cut -c1-200; tail -1 gpurun_out/r05bc_bench_c3.log | cut -c1-260; exit $rc
