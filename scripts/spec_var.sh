cd $GRAFT_REPO_ROOT && for v in "" NOFFT NOMEL BOTH; do if [ -n "$v" ]; then export SBK_PROBE_LIB=gpurun_probe_$v.so; fi; echo "== $v"; timeout -k 10 120 python -c "
import os,sys,torch
sys.path.insert(0,'.')
import speechbrain_amd._lib as L
if os.environ.get('SBK_PROBE_LIB'): L.LIB_PATH=os.path.abspath(os.environ['SBK_PROBE_LIB'])
from speechbrain_amd.lobes.features import Fbank
from scripts.kbench import timeit
fb=Fbank(n_mels=80).cuda(); wav=torch.randn(32,240000,device='cuda')*0.1
print('fbank %.1f us' % timeit(lambda: fb(wav), reps=20), flush=True)
" || exit 1; done
