# Round-5 closing evidence: config-5 kernel stats (MXFP8 step), SQ counters of the attention and conv-module kernels
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05av_c5prof && export TMPDIR=/tmp && \
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r05av_c5prof" -o run --output-format csv \
  -- python3 "$R/bench.py" --config c5 --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/r05av_c5prof/stdout.log" 2>&1) && \
bash scripts/att_pmc.sh && bash scripts/conv_pmc.sh && \
python3 scripts/pmc_summary.py relpos_flash_dma gpurun_out/att_pmc/p1/run_counter_collection.csv gpurun_out/att_pmc/p2/run_counter_collection.csv > gpurun_out/r05av_att_sq.txt && \
python3 scripts/pmc_summary.py conv_module gpurun_out/conv_pmc/p1/run_counter_collection.csv gpurun_out/conv_pmc/p2/run_counter_collection.csv > gpurun_out/r05av_conv_sq.txt
rc=$?; cat gpurun_out/r05av_att_sq.txt gpurun_out/r05av_conv_sq.txt; head -6 gpurun_out/r05av_c5prof/run_kernel_stats.csv | cut -c1-150; exit $rc
