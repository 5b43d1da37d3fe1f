# FFN chain: MFMAs pinned to their step (sched_barrier) A/B, activation-under-MFMA probe, and the paired-workgroup
# seam probe (one 48-KB partial exchange between blockIdx and blockIdx^8) — probes never the product; + parity.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 400 python scripts/chain_time.py gpurun_probe_img.so speechbrain_amd/libsbk.so gpurun_probe_ACTPIPE.so gpurun_probe_PAIRX.so gpurun_probe_img.so speechbrain_amd/libsbk.so gpurun_probe_ACTPIPE.so gpurun_probe_PAIRX.so > gpurun_out/r04h_chain_time.log 2>&1 && \
SBK_PROBE_LIB=gpurun_probe_TL.so timeout -k 10 120 python scripts/ffn_chain_tl.py > gpurun_out/r04h_chain_tl.log 2>&1 && \
SBK_PROBE_LIB=gpurun_probe_PAIRXTL.so timeout -k 10 120 python scripts/ffn_chain_tl.py > gpurun_out/r04h_pairx_tl.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_encoder.py tests/test_gpu_bench_parity.py > gpurun_out/r04h_tests.log 2>&1
rc=$?
cat gpurun_out/r04h_chain_time.log
grep -E "passed|failed|FAILED|Error" gpurun_out/r04h_tests.log | tail -4
exit $rc
