# FFN chain: LN exchange with one barrier per pass, activation under MFMAs (probe) — A/B + timeline (never the product) + parity.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_encoder.py tests/test_gpu_bench_parity.py tests/test_gpu_augment.py > gpurun_out/r04g_tests.log 2>&1 && \
timeout -k 10 400 python scripts/chain_time.py gpurun_probe_img.so speechbrain_amd/libsbk.so gpurun_probe_ACTPIPE.so gpurun_probe_NODMA.so gpurun_probe_NOACT.so gpurun_probe_NOLN.so gpurun_probe_NOMFMA.so gpurun_probe_img.so speechbrain_amd/libsbk.so gpurun_probe_ACTPIPE.so > gpurun_out/r04g_chain_time.log 2>&1 && \
SBK_PROBE_LIB=gpurun_probe_TL.so timeout -k 10 120 python scripts/ffn_chain_tl.py > gpurun_out/r04g_chain_tl.log 2>&1
rc=$?
cat gpurun_out/r04g_chain_time.log
grep -E "passed|failed|FAILED|Error" gpurun_out/r04g_tests.log | tail -4
exit $rc
