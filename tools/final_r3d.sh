#!/bin/bash
# round-3 final tree evidence (after the sinc exp map): smoke, the default bench line, rocprof stats of
# the graph-replayed hover launches in both precisions
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
mkdir -p gpurun_out
PROF="rocprofv3 --kernel-trace --stats --output-format csv"
B="python3 $R/bench.py --graph-only --no-cpu-baseline --no-configs --no-sweep"
T=(
  "r3_smoke|200|cd $R && python -c 'import __graft_entry__ as g; g.smoke()'"
  "r3_bench|900|cd $R && python bench.py"
  "prof_r3_c2_fp64|200|cd /tmp && export TMPDIR=/tmp && $PROF -d $R/gpurun_out/prof_r3_c2_fp64 -o k -- $B --precision fp64"
  "prof_r3_c2_fp32|200|cd /tmp && export TMPDIR=/tmp && $PROF -d $R/gpurun_out/prof_r3_c2_fp32 -o k -- $B --precision fp32"
)
exec "$R/tools/gpu_steps.sh" "${T[@]}"
