# SpecAugment in place (roll4 + fixup4): parity on every route, the C2 bench, its kernel stats and PMC traffic;
# conv module XCD-aware tile remap probe (never the product) A/B.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_augment.py > gpurun_out/r04m_aug.log 2>&1 && \
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > gpurun_out/r04m_bench_c2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04m_prof_c2 -o run -- python bench.py --config c2 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04m_prof_c2.log 2>&1 && \
bash scripts/pmc_traffic.sh r04m_pmc_c2 --config c2 && \
timeout -k 10 300 python scripts/conv_time.py speechbrain_amd/libsbk.so gpurun_probe_CMXCD.so speechbrain_amd/libsbk.so gpurun_probe_CMXCD.so > gpurun_out/r04m_conv_xcd.log 2>&1
rc=$?
cat gpurun_out/r04m_conv_xcd.log
grep -E "passed|failed|FAILED|Error" gpurun_out/r04m_aug.log | tail -4
tail -1 gpurun_out/r04m_bench_c2.log | cut -c1-900
exit $rc
