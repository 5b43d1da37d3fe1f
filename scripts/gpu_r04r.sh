# MXFP8 GEMM: the next-next stage's LDS-DMA issued after the stage's MFMAs — A/B against the previous build
# (gpurun_probe_mxbase.so, never the product), config-5 parity, the config-5 bench.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
SBK_PROBE_LIB=gpurun_probe_mxbase.so timeout -k 10 300 python scripts/c5_kbench.py > gpurun_out/r04r_c5k_base.log 2>&1 && \
timeout -k 10 300 python scripts/c5_kbench.py > gpurun_out/r04r_c5k_new.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_wav2vec.py > gpurun_out/r04r_w2v_tests.log 2>&1 && \
timeout -k 10 400 python bench.py --config c5 --no-cpu-baseline > gpurun_out/r04r_bench_c5.log 2>&1
rc=$?
paste gpurun_out/r04r_c5k_base.log gpurun_out/r04r_c5k_new.log | cut -c1-150
tail -2 gpurun_out/r04r_w2v_tests.log
tail -1 gpurun_out/r04r_bench_c5.log | cut -c1-300
exit $rc
