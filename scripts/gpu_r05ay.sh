# conv module + layer chain with the measured ds_read_b128 / ds_write_b64 lane-group bank model:
# parity tests, same-box A/B against the previous commit's kernels, LDS conflict counters
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_encoder.py tests/test_gpu_bench_parity.py tests/test_gpu_amp.py tests/test_gpu_dropin.py tests/test_gpu_trace.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r05ay_tests.log 2>&1 && \
( for r in 1 2 3; do timeout -k 10 300 python scripts/chain_time.py speechbrain_amd/libsbk.so gpurun_probe_HEADCF.so || exit $?; timeout -k 10 300 python scripts/conv_time.py speechbrain_amd/libsbk.so gpurun_probe_HEADCF.so || exit $?; done ) > gpurun_out/r05ay_ab.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d gpurun_out/r05ay_pmc_conv -o run -- python3 scripts/conv_time.py --one > gpurun_out/r05ay_pmc_conv.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d gpurun_out/r05ay_pmc_chain -o run -- python3 scripts/chain_time.py --one > gpurun_out/r05ay_pmc_chain.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r05ay_bench.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" gpurun_out/r05ay_tests.log | tail -5; cat gpurun_out/r05ay_ab.log; tail -1 gpurun_out/r05ay_bench.log; exit $rc
