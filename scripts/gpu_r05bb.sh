# Fbank spectrum kernel: frame-region stride A/B (product 106 vs 124 / 108 float2, from the LDS bank model) + LDS counters
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
( for r in 1 2 3; do for lib in speechbrain_amd/libsbk.so gpurun_probe_FS124.so gpurun_probe_FS108.so; do echo -n "$lib "; SBK_PROBE_LIB=$lib timeout -k 10 120 python scripts/spec_probe.py 32 || exit $?; done; done ) > gpurun_out/r05bb_fs_ab.log 2>&1 && \
SBK_PROBE_LIB=gpurun_probe_FS124.so timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d gpurun_out/r05bb_pmc_fs124 -o run -- python3 scripts/spec_probe.py 32 > gpurun_out/r05bb_pmc.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d gpurun_out/r05bb_pmc_fs106 -o run -- python3 scripts/spec_probe.py 32 >> gpurun_out/r05bb_pmc.log 2>&1
rc=$?; cat gpurun_out/r05bb_fs_ab.log; exit $rc
