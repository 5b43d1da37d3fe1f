# frontend2 (persistent) timeline: product timing + probe-build s_memtime marks of workgroup 100
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 120 python scripts/fe_probe.py > gpurun_out/r05v_fe.log 2>&1 && \
SBK_PROBE_TL=1 SBK_PROBE_LIB=gpurun_probe_FETL.so timeout -k 10 120 python scripts/fe_probe.py > gpurun_out/r05v_fe_tl.log 2>&1
rc=$?; cat gpurun_out/r05v_fe.log gpurun_out/r05v_fe_tl.log | grep -v amdgpu.ids; exit $rc
