#!/bin/bash
# One parameterised runner for every GPU-box job of this repo (run it through gpurun).  Each step
# runs under its own time limit; a step that crashes, aborts, faults or times out (exit >= 124) ends
# the run, an ordinary failure (exit 1) is recorded and the next step still runs.  Outputs go to
# gpurun_out/TAG/; commit the summaries you keep under profiles/.
#
#   tools/gpu.sh check TAG             the driver's bench form (K = 20) + the focused parity tests
#   tools/gpu.sh evidence TAG          GPU suite, smoke, default bench line (K = 2000), driver form (K = 20)
#   tools/gpu.sh prof TAG              rocprofv3 kernel-trace stats of the graph-replayed launches per workload
#   tools/gpu.sh pmc TAG [alg fp64 fp32]   PMC passes: HBM traffic + VALU counters (tools/pmc_summary.py folds them)
#   tools/gpu.sh fold TAG              (CPU side, after the pmc run merged back) fold the passes into
#                                      profiles/pmc_traffic.json and profiles/pmc_valu.json
#   tools/gpu.sh mix TAG LEVEL DRONES PHYSICS MODE E PRECISION   instruction-mix / activity passes of one race config
#   tools/gpu.sh phases TAG [LIB]      race phase profile (timing build, e.g. gym_pybullet_adrp_amd/libadrp_devt.so)
#   BENCH_ARGS="..." tools/gpu.sh ab TAG ROUNDS ARM [ARM ...]
#                                      A/B/n: bench.py once per arm, interleaved; an arm is a library path,
#                                      optionally followed by ,VAR=value switches
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
CMD="$1"; TAG="${2:-run}"; shift 2
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
PROF="cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv"
NB="python3 $R/bench.py --no-cpu-baseline --no-configs --graph-only"
RACE3="--task race --level level0 --drones 2 --envs 2048 --physics PYB --racemode COMPARE --steps 1000 --warmup 50"
RACE4="--task race --level level3 --drones 4 --envs 4096 --physics PYB_DW --racemode COMPETE --steps 1000 --warmup 50"

steps() {   # "name|seconds|command" ...
  local status=0
  for spec in "$@"; do
    local name="${spec%%|*}" rest="${spec#*|}"
    local secs="${rest%%|*}" cmd="${rest#*|}"
    echo "=== [$name] ($secs s): $cmd"
    timeout -k 10 "$secs" bash -c "$cmd" > "$O/$name.log" 2>&1
    local rc=$?
    echo "=== [$name] exit $rc"; tail -n 15 "$O/$name.log"
    [ $rc -ne 0 ] && status=$rc
    if [ $rc -ge 124 ]; then echo "stopping: step $name ended with $rc"; return $rc; fi
  done
  return $status
}

pmc() {     # name counters cmd...   (one counter group per rocprofv3 run, its own hard limit)
  local n="$1" c="$2"; shift 2
  echo "=== $n"
  (cd /tmp && TMPDIR=/tmp timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d "$O/$n" -o p -- "$@") > "$O/$n.log" 2>&1
  local rc=$?
  echo "=== $n exit $rc"
  return $rc
}

case "$CMD" in
  check)
    steps "bench_k20|420|python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.json" \
          "tests|500|python -u -m pytest -x -v --timeout 200 --timeout-method thread -s ${TESTS:-tests -m gpu}" ;;
  evidence)
    steps "pytest_gpu|900|python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
          "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
          "bench|420|python bench.py > $O/bench.json" \
          "bench_k20|420|python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.json" ;;
  prof)
    steps "prof_c2_fp64|200|$PROF -d $O/prof_c2_fp64 -o k -- $NB --steps 2000" \
          "prof_c2_fp32|200|$PROF -d $O/prof_c2_fp32 -o k -- $NB --steps 2000 --precision fp32" \
          "prof_c4_fp64|200|$PROF -d $O/prof_c4_fp64 -o k -- $NB $RACE4" \
          "prof_c4_fp32|200|$PROF -d $O/prof_c4_fp32 -o k -- $NB $RACE4 --precision fp32" \
          "prof_c3_fp64|200|$PROF -d $O/prof_c3_fp64 -o k -- $NB $RACE3" \
          "prof_c3_fp32|200|$PROF -d $O/prof_c3_fp32 -o k -- $NB $RACE3 --precision fp32" \
          "prof_c3p_fp64|200|$PROF -d $O/prof_c3p_fp64 -o k -- $NB $RACE3 --policy example" \
          "prof_c3p_fp32|200|$PROF -d $O/prof_c3p_fp32 -o k -- $NB $RACE3 --policy example --precision fp32" ;;
  pmc)
    FL="SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU"
    BU="SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
    for P in ${@:-alg fp64 fp32}; do
      if [ "$P" = alg ]; then   # the flop model: the one-lane fp32 kernel (read at handle creation)
        for W in "r3 level0 2 PYB COMPARE 2048" "r4 level3 4 PYB_DW COMPETE 4096" "r4g level3 4 PYB_GND_DRAG_DW COMPETE 4096"; do
          set -- $W
          ADRP_RACE_QUAD=0 pmc "${1}_alg_fp32" "$FL" python3 "$R/tools/pmc_race_steps.py" $2 $3 $4 $5 $6 40 "$R" fp32 || exit $?
        done
        continue
      fi
      H="python3 $R/tools/pmc_steps.py 4096 60 $P $R"
      R3="python3 $R/tools/pmc_race_steps.py level0 2 PYB COMPARE 2048 40 $R $P"
      R4="python3 $R/tools/pmc_race_steps.py level3 4 PYB_DW COMPETE 4096 40 $R $P"
      R4G="python3 $R/tools/pmc_race_steps.py level3 4 PYB_GND_DRAG_DW COMPETE 4096 40 $R $P"
      pmc h_f_$P FETCH_SIZE $H && pmc h_w_$P WRITE_SIZE $H && \
      pmc r3_f_$P FETCH_SIZE $R3 && pmc r3_w_$P WRITE_SIZE $R3 && \
      pmc r4_f_$P FETCH_SIZE $R4 && pmc r4_w_$P WRITE_SIZE $R4 && \
      pmc r4g_f_$P FETCH_SIZE $R4G && pmc r4g_w_$P WRITE_SIZE $R4G && \
      pmc r3_fl_$P "$FL" $R3 && pmc r3_bu_$P "$BU" $R3 && \
      pmc r4_fl_$P "$FL" $R4 && pmc r4_bu_$P "$BU" $R4 && \
      pmc r4g_fl_$P "$FL" $R4G && pmc r4g_bu_$P "$BU" $R4G && \
      pmc h_fl_$P "$FL" $H && pmc h_bu_$P "$BU" $H || exit $?
    done ;;
  fold)
    S="python3 $R/tools/pmc_summary.py"
    set -e
    for W in "r3 race_level0_2_PYB_fp32_2048 4096" "r4 race_level3_4_PYB_DW_fp32_4096 16384" \
             "r4g race_level3_4_PYB_GND_DRAG_DW_fp32_4096 16384"; do
      set -- $W
      [ -d "$O/${1}_alg_fp32" ] && $S --alg "$R/profiles/pmc_valu.json" "$2" "$O/${1}_alg_fp32" "$3"
    done
    for P in fp64 fp32; do
      [ -d "$O/h_f_$P" ] || continue
      $S "$R/profiles/pmc_traffic.json" \
        "PYB_${P}_4096" "$O/h_f_$P" "$O/h_w_$P" \
        "race_level0_2_PYB_${P}_2048" "$O/r3_f_$P" "$O/r3_w_$P" \
        "race_level3_4_PYB_DW_${P}_4096" "$O/r4_f_$P" "$O/r4_w_$P" \
        "race_level3_4_PYB_GND_DRAG_DW_${P}_4096" "$O/r4g_f_$P" "$O/r4g_w_$P"
      $S --valu "$R/profiles/pmc_valu.json" \
        "PYB_${P}_4096" "$O/h_fl_$P" "$O/h_bu_$P" \
        "race_level0_2_PYB_${P}_2048" "$O/r3_fl_$P" "$O/r3_bu_$P" \
        "race_level3_4_PYB_DW_${P}_4096" "$O/r4_fl_$P" "$O/r4_bu_$P" \
        "race_level3_4_PYB_GND_DRAG_DW_${P}_4096" "$O/r4g_fl_$P" "$O/r4g_bu_$P"
    done ;;
  mix)
    M="python3 $R/tools/pmc_race_steps.py $1 $2 $3 $4 $5 40 $R $6"
    pmc a "SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT" $M && \
    pmc b "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32" $M && \
    pmc c "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 SQ_WAIT_INST_LDS SQ_INSTS_VSKIPPED" $M && \
    pmc d "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INST_CYCLES_SALU SQ_INST_CYCLES_SMEM" $M ;;
  phases)
    L="${1:-gym_pybullet_adrp_amd/libadrp_devt.so}"
    steps "phases_c3|200|ADRP_LIB=$L python tools/race_phases.py level0 2 PYB COMPARE 2048" \
          "phases_c3p|200|ADRP_LIB=$L RACE_POLICY=example python tools/race_phases.py level0 2 PYB COMPARE 2048" \
          "phases_c4|200|ADRP_LIB=$L python tools/race_phases.py level3 4 PYB_DW COMPETE 4096" ;;
  ab)
    ROUNDS="$1"; shift
    for r in $(seq 1 "$ROUNDS"); do
      for ARM in "$@"; do
        IFS=',' read -r -a parts <<< "$ARM"
        envs=("ADRP_LIB=${parts[0]}" "${parts[@]:1}")
        # shellcheck disable=SC2086
        env "${envs[@]}" timeout -k 10 150 python bench.py --no-cpu-baseline --no-configs $BENCH_ARGS > "$O/ab_last.log" 2>&1 \
          || { tail -5 "$O/ab_last.log"; exit 1; }
        python3 - "$ARM" "$O/ab_last.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
r = d["roofline"]
print(f"{sys.argv[1]:60s} kernel_us {r['kernel_us']:8.3f} eager {r.get('eager_dispatch_us', float('nan')):8.3f} "
      f"step_us {d['ms_per_step'] * 1e3:8.3f} value {d['value']:.4e}", flush=True)
PY
        python3 - "$ARM" "$O/ab_last.log" >> "$O/ab_results.txt" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(sys.argv[1], d["roofline"]["kernel_us"], d["ms_per_step"] * 1e3)
PY
      done
    done ;;
  *) sed -n 2,17p "$0"; exit 2 ;;
esac
