# Fbank span prefetch into a second frame-region buffer (probe SBK_RF_PF=1, two workgroups per CU):
# bitwise output check against the product, same-box A/B, then the timeline probe of the product
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 120 python scripts/fb_out.py gpurun_out/fb_prod.npy && \
SBK_PROBE_LIB=gpurun_probe_PF.so timeout -k 10 120 python scripts/fb_out.py gpurun_out/fb_pf.npy && \
python -c "import numpy as np; a=np.load('gpurun_out/fb_prod.npy'); b=np.load('gpurun_out/fb_pf.npy'); print('bitwise equal:', a.shape, bool((a.view(np.uint32)==b.view(np.uint32)).all()))" && \
( for r in 1 2 3; do for lib in speechbrain_amd/libsbk.so gpurun_probe_PF.so; do echo -n "$lib "; SBK_PROBE_LIB=$lib timeout -k 10 120 python scripts/spec_probe.py 32 2>/dev/null || exit $?; done; done ) > gpurun_out/r05bf_pf_ab.log 2>&1 && \
SBK_PROBE_LIB=gpurun_probe_TL.so timeout -k 10 120 python scripts/rf_tl.py > gpurun_out/r05bf_fbank_timeline.log 2>&1
rc=$?; cat gpurun_out/r05bf_pf_ab.log; tail -12 gpurun_out/r05bf_fbank_timeline.log; exit $rc
