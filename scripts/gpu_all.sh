#!/bin/bash
# tests -> bench -> rocprof profile, stopping at the first crash-class failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
scripts/gpu_check.sh "$@"
rc=$?
if [ $rc -ne 0 ]; then exit $rc; fi
scripts/profile.sh prof --steps 5 --warmup 2
