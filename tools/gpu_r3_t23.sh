#!/bin/bash
# round 3: final evidence a (suite, smoke, default bench) on the final tree, then b + c (rocprof, PMC)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
tools/final_r3a.sh
rc=$?
[ $rc -ge 124 ] && exit $rc
tools/final_r3bc.sh
