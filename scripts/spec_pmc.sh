#!/bin/bash
# SQ counters of the spectrum kernels (spec_probe at B = 32; two passes;
# summaries in gpurun_out/spec_pmc).  Probe tooling, not the product.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/spec_pmc"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  -d "$R/gpurun_out/spec_pmc/p1" -o run --output-format csv -- python3 "$R/scripts/spec_probe.py" 32 > "$R/gpurun_out/spec_pmc/p1.log" 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE \
  -d "$R/gpurun_out/spec_pmc/p2" -o run --output-format csv -- python3 "$R/scripts/spec_probe.py" 32 > "$R/gpurun_out/spec_pmc/p2.log" 2>&1
