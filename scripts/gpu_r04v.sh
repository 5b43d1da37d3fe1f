# FFN chain: LDS row pad 8 (probe, never the product) against 16 — SQ counters showed 23 % of LDS cycles in bank conflicts.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 300 python scripts/chain_time.py speechbrain_amd/libsbk.so gpurun_probe_PAD8.so speechbrain_amd/libsbk.so gpurun_probe_PAD8.so > gpurun_out/r04v_chain_pad.log 2>&1
rc=$?
cat gpurun_out/r04v_chain_pad.log
exit $rc
