#!/bin/bash
# Build probe variants of libsbk.so with one source compiled under -DSBK_PROBE_<V>
# (phase-removal experiments; never the product).  Output: gpurun_probe_<V>.so
# usage: scripts/probe_build.sh <source.hip> V1 V2 ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
SRC=$1; shift
B=$(basename "$SRC" .hip)
mkdir -p /tmp/probe
for v in "$@"; do
  # V may be NAME (-> -DSBK_PROBE_NAME) or NAME=DEF1,DEF2 (-> -DDEF1 -DDEF2, output gpurun_probe_NAME.so)
  if [[ "$v" == *=* ]]; then DEFS=$(echo "${v#*=}" | sed 's/,/ -D/g; s/^/-D/'); v=${v%%=*}; else DEFS="-DSBK_PROBE_$v"; fi
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -fPIC -fvisibility=hidden \
    -mllvm -amdgpu-mfma-vgpr-form -I"$R/speechbrain_amd/csrc" -I"$(dirname "$SRC")" $DEFS -c "$SRC" -o /tmp/probe/${B}_$v.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$R/gpurun_probe_$v.so" /tmp/probe/${B}_$v.o \
    $(ls "$R"/speechbrain_amd/csrc/build/*.o | grep -v "/$B.o")
done
