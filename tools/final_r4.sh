#!/bin/bash
# Round-4 evidence on one GPU box, each step under its own time limit (tools/gpu_steps.sh):
#   A: GPU suite, smoke, the default bench line (K = 2000) and the driver's form (K = 20)
#   B: rocprofv3 kernel-trace stats of the graph-replayed launches per benched workload
# usage: tools/final_r4.sh A|B
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
PROF="cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv"
B="python3 $R/bench.py --no-cpu-baseline --no-configs --graph-only"
RACE3="--task race --level level0 --drones 2 --envs 2048 --physics PYB --racemode COMPARE --steps 1000 --warmup 50"
RACE4="--task race --level level3 --drones 4 --envs 4096 --physics PYB_DW --racemode COMPETE --steps 1000 --warmup 50"
A=(
  "r4_pytest_gpu|700|cd $R && python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread"
  "r4_smoke|200|cd $R && python -c 'import __graft_entry__ as g; g.smoke()'"
  "r4_bench|400|cd $R && python bench.py > gpurun_out/r4_bench.json"
  "r4_bench_k20|300|cd $R && python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_bench_k20.json"
)
P=(
  "r4_prof_c2_fp64|200|$PROF -d $R/gpurun_out/r4_prof_c2_fp64 -o k -- $B --steps 2000"
  "r4_prof_c2_fp32|200|$PROF -d $R/gpurun_out/r4_prof_c2_fp32 -o k -- $B --steps 2000 --precision fp32"
  "r4_prof_c4_fp64|200|$PROF -d $R/gpurun_out/r4_prof_c4_fp64 -o k -- $B $RACE4"
  "r4_prof_c4_fp32|200|$PROF -d $R/gpurun_out/r4_prof_c4_fp32 -o k -- $B $RACE4 --precision fp32"
  "r4_prof_c3_fp64|200|$PROF -d $R/gpurun_out/r4_prof_c3_fp64 -o k -- $B $RACE3"
  "r4_prof_c3p_fp64|200|$PROF -d $R/gpurun_out/r4_prof_c3p_fp64 -o k -- $B $RACE3 --policy example"
  "r4_prof_c3p_fp32|200|$PROF -d $R/gpurun_out/r4_prof_c3p_fp32 -o k -- $B $RACE3 --policy example --precision fp32"
)
case "$1" in
  A) exec "$R/tools/gpu_steps.sh" "${A[@]}" ;;
  B) exec "$R/tools/gpu_steps.sh" "${P[@]}" ;;
  *) echo "usage: $0 A|B"; exit 2 ;;
esac
