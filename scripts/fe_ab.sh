# frontend2 A/B on one box: the product library against probe builds, alternating, 3 rounds
# usage: scripts/fe_ab.sh <out-log> <probe.so>...
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
out=$1; shift
: > gpurun_out/$out
for r in 1 2 3; do
  for lib in speechbrain_amd/libsbk.so "$@"; do
    echo -n "$lib: " >> gpurun_out/$out
    SBK_PROBE_LIB=$lib timeout -k 10 120 python scripts/fe_probe.py 2>/dev/null | grep fused >> gpurun_out/$out || exit $?
  done
done
cat gpurun_out/$out
