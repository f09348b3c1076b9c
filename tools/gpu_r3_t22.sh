#!/bin/bash
# round 3: final part a (suite, smoke, default bench) and the early-store A/B in one call
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
tools/final_r3a.sh
rc=$?
[ $rc -ge 124 ] && exit $rc
tools/gpu_r3_t21.sh
