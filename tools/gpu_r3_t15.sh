#!/bin/bash
# round 3: hybrid contact GJK (fp32, fp64 rerun of undecided queries): suite, phases, reset cost;
# in-loop vs pre-drawn sub-step draws (ADRP_RACE_PREDRAW)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
exec tools/gpu_steps.sh \
  "r3_suite4|600|python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests" \
  "r3_ph4_c4|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devt.so python tools/race_phases.py level3 4 PYB_DW COMPETE 4096" \
  "r3_ph4_c3p|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devt.so RACE_POLICY=example python tools/race_phases.py level0 2 PYB COMPARE 2048" \
  "r3_ph4_c4_nopre|200|ADRP_RACE_PREDRAW=0 ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devt.so python tools/race_phases.py level3 4 PYB_DW COMPETE 4096" \
  "r3_reset_ab4|300|python tools/reset_ab.py level3 4 PYB_DW COMPETE 4096 fp32 && ADRP_RACE_PREDRAW=0 python tools/reset_ab.py level3 4 PYB_DW COMPETE 4096 fp32 && python tools/reset_ab.py level3 4 PYB_DW COMPETE 4096 fp64 && ADRP_RACE_PREDRAW=0 python tools/reset_ab.py level3 4 PYB_DW COMPETE 4096 fp64"
