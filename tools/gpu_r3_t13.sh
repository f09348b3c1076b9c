#!/bin/bash
# round 3: capped-GJK dump (pre-stall stats build); full GPU suite on the GJK stall exit + precomputed
# nominal attitudes; phases and the auto-reset cost on the new kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
exec tools/gpu_steps.sh \
  "r3_cap2_c3p|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devg.so RACE_POLICY=example python tools/gjk_capped.py level0 2 PYB COMPARE 2048 300" \
  "r3_suite2|600|python -u -m pytest -m gpu -v -x --timeout 300 --timeout-method thread tests" \
  "r3_ph2_c4|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devt.so python tools/race_phases.py level3 4 PYB_DW COMPETE 4096" \
  "r3_ph2_c3p|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devt.so RACE_POLICY=example python tools/race_phases.py level0 2 PYB COMPARE 2048" \
  "r3_reset_ab2|200|python tools/reset_ab.py level3 4 PYB_DW COMPETE 4096 fp32 && python tools/reset_ab.py level3 4 PYB_DW COMPETE 4096 fp64"
