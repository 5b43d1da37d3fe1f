# Final-tree C2 evidence: kernel stats and the HBM traffic passes of the config-2 step (SpecAugment at J = 2).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04t_prof_c2 -o run -- python bench.py --config c2 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04t_prof_c2.log 2>&1 && \
bash scripts/pmc_traffic.sh r04t_pmc_c2 --config c2 && \
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > gpurun_out/r04t_bench_c2.log 2>&1
rc=$?
tail -1 gpurun_out/r04t_bench_c2.log | cut -c1-300
exit $rc
