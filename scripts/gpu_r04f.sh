# FFN chain phase-removal probes on the weight-image kernel (never the product) + encoder parity.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_encoder.py tests/test_gpu_bench_parity.py > gpurun_out/r04f_enc.log 2>&1 && \
timeout -k 10 400 python scripts/chain_time.py gpurun_probe_base.so speechbrain_amd/libsbk.so gpurun_probe_NODMA.so gpurun_probe_NOACT.so gpurun_probe_NOLN.so gpurun_probe_NOMFMA.so speechbrain_amd/libsbk.so > gpurun_out/r04f_chain_time.log 2>&1
rc=$?
cat gpurun_out/r04f_chain_time.log
grep -E "passed|failed|FAILED|Error" gpurun_out/r04f_enc.log | tail -4
exit $rc
