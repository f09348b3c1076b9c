#!/bin/bash
# round-3 evidence, parts b + c: rocprof kernel stats of the graph-replayed launches, then the PMC passes
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
tools/final_r3b.sh
rc=$?
[ $rc -ge 124 ] && exit $rc
tools/pmc_r3.sh > gpurun_out/pmc_r3.log 2>&1
rc2=$?
tail -n 5 gpurun_out/pmc_r3.log
[ $rc2 -ne 0 ] && exit $rc2
exit $rc
