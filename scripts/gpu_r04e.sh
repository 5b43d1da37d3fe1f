# SpecAugment (copy path + device cell count): parity, C2 bench and per-kernel stats (never the product).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_augment.py > gpurun_out/r04e_aug.log 2>&1 && \
timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 5 > gpurun_out/r04e_bench_c2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04e_prof_c2 -o run -- python bench.py --config c2 --steps 10 --warmup 3 > gpurun_out/r04e_prof_c2.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_encoder.py tests/test_gpu_bench_parity.py > gpurun_out/r04e_enc.log 2>&1 && \
timeout -k 10 300 python scripts/chain_time.py gpurun_probe_base.so speechbrain_amd/libsbk.so gpurun_probe_base.so speechbrain_amd/libsbk.so > gpurun_out/r04e_chain_time.log 2>&1 && \
SBK_PROBE_LIB=gpurun_probe_TL.so timeout -k 10 120 python scripts/ffn_chain_tl.py > gpurun_out/r04e_chain_tl.log 2>&1
rc=$?
cat gpurun_out/r04e_chain_time.log
grep -E "passed|failed|FAILED|Error" gpurun_out/r04e_aug.log gpurun_out/r04e_enc.log | tail -6
tail -1 gpurun_out/r04e_bench_c2.log 2>/dev/null | cut -c1-1200
find gpurun_out/r04e_prof_c2 -name "*kernel_stats.csv" | head -2
exit $rc
