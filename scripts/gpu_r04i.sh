# MFMAs pinned to their K-step (sched_barrier) in the FFN chain and the conv module: A/B against the previous build
# (gpurun_probe_img.so); the bench step as 1 / 2 / 4 utterance groups on their own streams; parity; kernel stats.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 300 python scripts/chain_time.py gpurun_probe_img.so speechbrain_amd/libsbk.so gpurun_probe_img.so speechbrain_amd/libsbk.so > gpurun_out/r04i_chain_time.log 2>&1 && \
SBK_PROBE_LIB=gpurun_probe_img.so timeout -k 10 120 python scripts/kbench.py convmod > gpurun_out/r04i_conv_ab.log 2>&1 && \
timeout -k 10 120 python scripts/kbench.py convmod >> gpurun_out/r04i_conv_ab.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bench_parity.py tests/test_gpu_encoder.py > gpurun_out/r04i_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r04i_bench_s1.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --streams 2 > gpurun_out/r04i_bench_s2.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --streams 4 > gpurun_out/r04i_bench_s4.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04i_prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --streams 2 > gpurun_out/r04i_prof.log 2>&1
rc=$?
cat gpurun_out/r04i_chain_time.log gpurun_out/r04i_conv_ab.log
grep -E "passed|failed|FAILED|Error|B=32" gpurun_out/r04i_tests.log | tail -5
for f in s1 s2 s4; do tail -1 gpurun_out/r04i_bench_$f.log | cut -c1-200; done
exit $rc
