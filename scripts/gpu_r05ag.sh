# frontend2 with the next tile staged by the idle waves: parity tests, A/B vs the previous commit, timeline, HBM traffic
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_encoder.py tests/test_gpu_bench_parity.py tests/test_gpu_amp.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05ag_tests.log 2>&1 && \
bash scripts/fe_ab.sh r05ag_fe_stage_ab.log gpurun_probe_HEADFE.so > /dev/null && \
SBK_PROBE_TL=1 SBK_PROBE_LIB=gpurun_probe_FETL.so timeout -k 10 120 python scripts/fe_probe.py > gpurun_out/r05ag_fe_tl.log 2>&1 && \
mkdir -p gpurun_out/r05ag_fe_write && cd /tmp && \
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r05ag_fe_write -o k --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/fe_probe.py > $GRAFT_REPO_ROOT/gpurun_out/r05ag_fe_write/log.txt 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; tail -1 gpurun_out/r05ag_tests.log; cat gpurun_out/r05ag_fe_stage_ab.log; grep -v amdgpu gpurun_out/r05ag_fe_tl.log | head -14; exit $rc
