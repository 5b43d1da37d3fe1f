# HBM traffic of the config-2 kernels after the round-5 feature changes (FETCH_SIZE / WRITE_SIZE passes), then the C2 and C5 lines
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
bash scripts/pmc_traffic.sh r05bl_pmc_c2 --config c2 && \
cd $GRAFT_REPO_ROOT && python3 scripts/traffic_json.py gpurun_out/r05bl_pmc_c2_fetch/k_counter_collection.csv gpurun_out/r05bl_pmc_c2_write/k_counter_collection.csv gpurun_out/r05bl_c2_traffic.json
rc=$?; exit $rc
