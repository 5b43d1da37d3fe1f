#!/bin/bash
# rocprofv3 kernel stats of the spectrum probe for probe builds of features.hip
# usage: scripts/spec_prof.sh V1 V2 ...   (V = probe name; "base" = the product lib)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  D="$R/gpurun_out/spec_$v"; mkdir -p "$D"
  if [ "$v" = base ]; then unset SBK_PROBE_LIB; else export SBK_PROBE_LIB="$R/gpurun_probe_$v.so"; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$D" -o run --output-format csv \
    -- python3 "$R/scripts/spec_probe.py" 32 > "$D/log.txt" 2>&1 || exit $?
done
