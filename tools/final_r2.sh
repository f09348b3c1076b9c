#!/bin/bash
# round-2 evidence: smoke, the driver's default bench line, rocprof kernel stats per benched config
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
mkdir -p gpurun_out
PROF="rocprofv3 --kernel-trace --stats --output-format csv"
T=(
  "smoke_r2|200|cd $R && python -c 'import __graft_entry__ as g; g.smoke()'"
  "bench_r2|500|cd $R && python bench.py"
  "prof_r2_c2|200|cd /tmp && export TMPDIR=/tmp && $PROF -d $R/gpurun_out/prof_r2_c2 -o k -- python3 $R/bench.py --no-configs --no-sweep --no-cpu-baseline"
  "prof_r2_c4|200|cd /tmp && export TMPDIR=/tmp && $PROF -d $R/gpurun_out/prof_r2_c4 -o k -- python3 $R/bench.py --task race --level level3 --drones 4 --envs 4096 --physics PYB_DW --racemode COMPETE --steps 200 --warmup 20 --no-cpu-baseline"
  "prof_r2_c3|200|cd /tmp && export TMPDIR=/tmp && $PROF -d $R/gpurun_out/prof_r2_c3 -o k -- python3 $R/bench.py --task race --level level0 --drones 2 --envs 2048 --steps 200 --warmup 20 --no-cpu-baseline"
  "prof_r2_c3p|200|cd /tmp && export TMPDIR=/tmp && $PROF -d $R/gpurun_out/prof_r2_c3p -o k -- python3 $R/bench.py --task race --level level0 --drones 2 --envs 2048 --steps 200 --warmup 20 --no-cpu-baseline --policy example"
)
exec "$R/tools/gpu_steps.sh" "${T[@]}"
