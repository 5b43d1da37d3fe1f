# attention 32-query variant: A/B + encoder tests + C3 bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 200 python scripts/att_ab.py > gpurun_out/r05e_att_ab.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_encoder.py tests/test_gpu_bench_parity.py tests/test_gpu_dropin.py tests/test_gpu_wav2vec.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05e_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05e_bench_c3.log 2>&1
rc=$?
cat gpurun_out/r05e_att_ab.log
tail -3 gpurun_out/r05e_tests.log
tail -1 gpurun_out/r05e_bench_c3.log | cut -c1-300
exit $rc
