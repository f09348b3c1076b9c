#!/bin/bash
# Round-4 PMC passes of the benched step kernels, one counter group per rocprofv3 run (each under its
# own time limit): HBM traffic (FETCH_SIZE, WRITE_SIZE) and the VALU counters, for hover config 2,
# race configs 3 / 4 and config 4 with PYB_GND_DRAG_DW, both precisions; plus the FLOPS pass of the
# one-lane fp32 kernel on PYB_GND_DRAG_DW (the flop model of that workload).
# Summaries: tools/pmc_summary.py (profiles/pmc_traffic.json, profiles/pmc_valu.json).
# usage: tools/pmc_r4.sh [fp64|fp32|alg ...]   (default: alg fp64 fp32)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/pmc_r4"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
FL="SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU"
BU="SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
run() {  # name counters cmd...
  local n="$1" c="$2"; shift 2
  echo "=== $n"
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d "$O/$n" -o p -- "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "=== $n exit $rc"
  [ $rc -eq 0 ] || exit $rc
}
for P in ${@:-alg fp64 fp32}; do
  if [ "$P" = alg ]; then
    # ADRP_RACE_QUAD=0 is read by the library at handle creation (not an exec hop)
    export ADRP_RACE_QUAD=0
    run r4g_alg_fp32 "$FL" python3 $R/tools/pmc_race_steps.py level3 4 PYB_GND_DRAG_DW COMPETE 4096 40 $R fp32 || exit $?
    unset ADRP_RACE_QUAD
    continue
  fi
  H="python3 $R/tools/pmc_steps.py 4096 60 $P $R"
  R3="python3 $R/tools/pmc_race_steps.py level0 2 PYB COMPARE 2048 40 $R $P"
  R4="python3 $R/tools/pmc_race_steps.py level3 4 PYB_DW COMPETE 4096 40 $R $P"
  R4G="python3 $R/tools/pmc_race_steps.py level3 4 PYB_GND_DRAG_DW COMPETE 4096 40 $R $P"
  run h_f_$P FETCH_SIZE $H && run h_w_$P WRITE_SIZE $H && \
  run r3_f_$P FETCH_SIZE $R3 && run r3_w_$P WRITE_SIZE $R3 && \
  run r4_f_$P FETCH_SIZE $R4 && run r4_w_$P WRITE_SIZE $R4 && \
  run r4g_f_$P FETCH_SIZE $R4G && run r4g_w_$P WRITE_SIZE $R4G && \
  run r3_fl_$P "$FL" $R3 && run r3_bu_$P "$BU" $R3 && \
  run r4_fl_$P "$FL" $R4 && run r4_bu_$P "$BU" $R4 && \
  run r4g_fl_$P "$FL" $R4G && run r4g_bu_$P "$BU" $R4G && \
  run h_fl_$P "$FL" $H && run h_bu_$P "$BU" $H || exit $?
done
