# SQ counters of the fused conv module (two passes) and the final tree's C2 HBM traffic passes.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
bash scripts/conv_pmc.sh && \
bash scripts/pmc_traffic.sh r04z_pmc_c2 --config c2
rc=$?
tail -3 gpurun_out/conv_pmc/p1.log
exit $rc
