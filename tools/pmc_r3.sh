#!/bin/bash
# Round-3 PMC passes of the benched step kernels at both precisions, one counter group per rocprofv3
# run (each under its own time limit): HBM traffic (FETCH_SIZE, WRITE_SIZE; tools/fetch_calib for the
# gfx950 correction) and the VALU counters, for hover config 2 and race configs 3 / 4.
# Summaries: tools/pmc_summary.py (profiles/pmc_traffic.json, profiles/pmc_valu.json).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/pmc_r3"
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
for P in fp64 fp32; do
  H="python3 $R/tools/pmc_steps.py 4096 60 $P $R"
  R3="python3 $R/tools/pmc_race_steps.py level0 2 PYB COMPARE 2048 40 $R $P"
  R4="python3 $R/tools/pmc_race_steps.py level3 4 PYB_DW COMPETE 4096 40 $R $P"
  run h_f_$P FETCH_SIZE $H && run h_w_$P WRITE_SIZE $H && \
  run r3_f_$P FETCH_SIZE $R3 && run r3_w_$P WRITE_SIZE $R3 && \
  run r4_f_$P FETCH_SIZE $R4 && run r4_w_$P WRITE_SIZE $R4 && \
  run r3_fl_$P "$FL" $R3 && run r3_bu_$P "$BU" $R3 && \
  run r4_fl_$P "$FL" $R4 && run r4_bu_$P "$BU" $R4 && \
  run h_fl_$P "$FL" $H && run h_bu_$P "$BU" $H || exit $?
done
