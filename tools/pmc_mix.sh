#!/bin/bash
# Instruction-mix / activity PMC passes of one race config (one counter group per rocprofv3 run,
# each under its own time limit): where the wave cycles of the step kernel go.
# usage: tools/pmc_mix.sh TAG LEVEL DRONES PHYSICS MODE E PRECISION
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
O="$R/gpurun_out/pmc_$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/tools/pmc_race_steps.py $1 $2 $3 $4 $5 40 $R $6"
A="SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT"
B="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32"
C="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 SQ_WAIT_INST_LDS SQ_INSTS_VSKIPPED"
D="SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INST_CYCLES_SALU SQ_INST_CYCLES_SMEM"
run() {
  local n="$1" c="$2"
  echo "=== $n"
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d "$O/$n" -o p -- $CMD > "$O/$n.log" 2>&1
  local rc=$?
  echo "=== $n exit $rc"
  [ $rc -eq 0 ] || exit $rc
}
run a "$A" && run b "$B" && run c "$C" && run d "$D"
