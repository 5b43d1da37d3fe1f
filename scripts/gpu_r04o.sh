# SpecAugment in place: slab width A/B (J = 4 product, 2, 1 probes; never the product), parity, C2 stats.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 300 python scripts/sa_time.py speechbrain_amd/libsbk.so gpurun_probe_RJ2.so gpurun_probe_RJ1.so speechbrain_amd/libsbk.so gpurun_probe_RJ2.so gpurun_probe_RJ1.so > gpurun_out/r04o_sa_time.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_augment.py > gpurun_out/r04o_aug.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04o_prof_c2 -o run -- python bench.py --config c2 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04o_prof_c2.log 2>&1
rc=$?
cat gpurun_out/r04o_sa_time.log
grep -E "passed|failed|FAILED|Error" gpurun_out/r04o_aug.log | tail -3
exit $rc
