#!/bin/bash
# SQ counters of the fused front-end (fe_probe.py launches) (two passes; summaries in gpurun_out/fe_pmc)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/fe_pmc"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES \
  -d "$R/gpurun_out/fe_pmc/p1" -o run --output-format csv -- python3 "$R/scripts/fe_probe.py" > "$R/gpurun_out/fe_pmc/p1.log" 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
  -d "$R/gpurun_out/fe_pmc/p2" -o run --output-format csv -- python3 "$R/scripts/fe_probe.py" > "$R/gpurun_out/fe_pmc/p2.log" 2>&1
