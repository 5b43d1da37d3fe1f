# SpecAugment in place at J = 2 with 16-B fixup stores: per-call time and parity; then the round-4 final tree
# (scripts/gpu_r04final.sh).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 200 python scripts/sa_time.py speechbrain_amd/libsbk.so speechbrain_amd/libsbk.so > gpurun_out/r04p_sa_time.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_augment.py > gpurun_out/r04p_aug.log 2>&1 && \
cat gpurun_out/r04p_sa_time.log && bash scripts/gpu_r04final.sh
