# LDS counters of every kernel of the config-3 step (bench.py), after the bank-model layouts
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS -d gpurun_out/r05az_pmc -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r05az_pmc.log 2>&1
rc=$?; tail -3 gpurun_out/r05az_pmc.log; exit $rc
