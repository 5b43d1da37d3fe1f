# SpecAugment fixup4 with the partial sums loaded eight at a time: per-call time, parity, C2 kernel stats.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 200 python scripts/sa_time.py speechbrain_amd/libsbk.so speechbrain_amd/libsbk.so > gpurun_out/r04u_sa_time.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_augment.py > gpurun_out/r04u_aug.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04u_prof_c2 -o run -- python bench.py --config c2 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04u_prof_c2.log 2>&1 && \
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > gpurun_out/r04u_bench_c2.log 2>&1
rc=$?
cat gpurun_out/r04u_sa_time.log
tail -2 gpurun_out/r04u_aug.log
tail -1 gpurun_out/r04u_bench_c2.log | cut -c1-300
exit $rc
