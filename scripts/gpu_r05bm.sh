# the C2 and C5 lines with the merged traffic table
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > gpurun_out/r05bm_bench_c2.log 2>&1 && \
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > gpurun_out/r05bm_bench_c5.log 2>&1
rc=$?; tail -1 gpurun_out/r05bm_bench_c2.log | cut -c1-250; tail -1 gpurun_out/r05bm_bench_c5.log | cut -c1-250; exit $rc
