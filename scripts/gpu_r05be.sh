# Fbank (register-FFT) timeline after the batched table stage (probe build, never the product)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
SBK_PROBE_LIB=gpurun_probe_TL.so timeout -k 10 120 python scripts/rf_tl.py > gpurun_out/r05be_fbank_timeline.log 2>&1
rc=$?; cat gpurun_out/r05be_fbank_timeline.log; exit $rc
