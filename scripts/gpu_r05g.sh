# chain vs GEMM-FFN A/B; fresh s_memtime timelines of the three C3 layer kernels (probe builds, never the product)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 240 python -u scripts/chain_gemm_ab.py > gpurun_out/r05g_chain_gemm_ab.log 2>&1 && \
CM_PRE=1 SBK_PROBE_LIB=gpurun_probe_CMTL.so timeout -k 10 120 python -u scripts/cm_tl.py > gpurun_out/r05g_cm_tl.log 2>&1 && \
SBK_PROBE_LIB=gpurun_probe_FFTL.so timeout -k 10 120 python -u scripts/ffn_chain_tl.py > gpurun_out/r05g_chain_tl.log 2>&1 && \
SBK_PROBE_LIB=gpurun_probe_ATTL.so timeout -k 10 120 python -u scripts/att_dma_tl.py > gpurun_out/r05g_att_tl.log 2>&1
rc=$?
cat gpurun_out/r05g_chain_gemm_ab.log gpurun_out/r05g_cm_tl.log
exit $rc
