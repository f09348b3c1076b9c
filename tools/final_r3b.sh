#!/bin/bash
# round-3 evidence, part b: rocprof kernel stats of the graph-replayed launches of every benched
# config (bench.py --graph-only: no eager event-timed launches after the timed region)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
mkdir -p gpurun_out
PROF="rocprofv3 --kernel-trace --stats --output-format csv"
B="python3 $R/bench.py --graph-only --no-cpu-baseline"
RACE4="--task race --level level3 --drones 4 --envs 4096 --physics PYB_DW --racemode COMPETE --steps 200 --warmup 20"
RACE3="--task race --level level0 --drones 2 --envs 2048 --steps 200 --warmup 20"
T=()
for P in fp64 fp32; do
  T+=("prof_r3_c2_$P|200|cd /tmp && export TMPDIR=/tmp && $PROF -d $R/gpurun_out/prof_r3_c2_$P -o k -- $B --no-configs --no-sweep --precision $P")
  T+=("prof_r3_c4_$P|200|cd /tmp && export TMPDIR=/tmp && $PROF -d $R/gpurun_out/prof_r3_c4_$P -o k -- $B $RACE4 --precision $P")
  T+=("prof_r3_c3_$P|200|cd /tmp && export TMPDIR=/tmp && $PROF -d $R/gpurun_out/prof_r3_c3_$P -o k -- $B $RACE3 --precision $P")
  T+=("prof_r3_c3p_$P|200|cd /tmp && export TMPDIR=/tmp && $PROF -d $R/gpurun_out/prof_r3_c3p_$P -o k -- $B $RACE3 --precision $P --policy example")
done
exec "$R/tools/gpu_steps.sh" "${T[@]}"
