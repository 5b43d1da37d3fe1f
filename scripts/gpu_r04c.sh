# Chain-kernel lean-DMA probe (never the product).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python scripts/chain_time.py speechbrain_amd/libsbk.so gpurun_probe_SIMPLEDMA.so gpurun_probe_NODMA.so \
  speechbrain_amd/libsbk.so gpurun_probe_SIMPLEDMA.so > gpurun_out/chain_probes2.log 2>&1
rc=$?
cat gpurun_out/chain_probes2.log
exit $rc
