# FFN chain prologue probes (never the product): the first two tiles issued ahead of the x rows (TFIRST), the x rows
# loaded once with the residual layout read back through an LDS staging image (XONCE), both (XT).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 400 python scripts/chain_time.py speechbrain_amd/libsbk.so gpurun_probe_TFIRST.so gpurun_probe_XONCE.so gpurun_probe_XT.so speechbrain_amd/libsbk.so gpurun_probe_TFIRST.so gpurun_probe_XONCE.so gpurun_probe_XT.so > gpurun_out/r04k_chain_time.log 2>&1
rc=$?
cat gpurun_out/r04k_chain_time.log
exit $rc
