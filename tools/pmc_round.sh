#!/bin/bash
# PMC passes of the benched step kernels, one counter group per rocprofv3 run (each under its own
# time limit): HBM traffic (FETCH_SIZE, WRITE_SIZE) and the VALU roofline (FLOPS, instruction mix,
# busy cycles) for hover config 2 and race configs 3 / 4.  Summaries: tools/pmc_summary.py.
# usage: tools/pmc_round.sh TAG
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r2}"
O="$R/gpurun_out/pmc_$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
FL="SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU"
BU="SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
H="python3 $R/tools/pmc_steps.py 4096 60 fp32 $R"
R3="python3 $R/tools/pmc_race_steps.py level0 2 PYB COMPARE 2048 40 $R"
R4="python3 $R/tools/pmc_race_steps.py level3 4 PYB_DW COMPETE 4096 40 $R"
run() {  # name counters cmd...
  local n="$1" c="$2"; shift 2
  echo "=== $n"
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d "$O/$n" -o p -- "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "=== $n exit $rc"
  [ $rc -eq 0 ] || exit $rc
}
run hf FETCH_SIZE $H && run hw WRITE_SIZE $H && \
run r3f FETCH_SIZE $R3 && run r3w WRITE_SIZE $R3 && \
run r4f FETCH_SIZE $R4 && run r4w WRITE_SIZE $R4 && \
run r3fl "$FL" $R3 && run r3bu "$BU" $R3 && \
run r4fl "$FL" $R4 && run r4bu "$BU" $R4 && \
run hfl "$FL" $H && run hbu "$BU" $H
