# augment parity on the roll route (new long / narrow / bilinear cases); then the r05g timelines
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_augment.py > gpurun_out/r05i_aug.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r05i_aug.log | tail -5
[ $rc -ne 0 ] && exit $rc
CM_PRE=1 SBK_PROBE_LIB=gpurun_probe_CMTL.so timeout -k 10 120 python -u scripts/cm_tl.py > gpurun_out/r05g_cm_tl.log 2>&1 && \
SBK_PROBE_LIB=gpurun_probe_FFTL.so timeout -k 10 120 python -u scripts/ffn_chain_tl.py > gpurun_out/r05g_chain_tl.log 2>&1 && \
SBK_PROBE_LIB=gpurun_probe_ATTL.so timeout -k 10 120 python -u scripts/att_dma_tl.py > gpurun_out/r05g_att_tl.log 2>&1 && \
SBK_PROBE_LIB=gpurun_probe_RFTL.so timeout -k 10 120 python -u scripts/rf_tl.py > gpurun_out/r05g_rf_tl.log 2>&1
rc=$?
cat gpurun_out/r05g_cm_tl.log
exit $rc
