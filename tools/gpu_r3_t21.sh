#!/bin/bash
# round 3: drone body stored right after the sub-step loop (ab1) vs at the end (ab0); obs-phase split
# with the early store under the actor
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
L=gym_pybullet_adrp_amd
ab() {  # lib
  echo "ADRP_LIB=$L/$1 AB_ONLY=autoreset python tools/reset_ab.py level3 4 PYB_DW COMPETE 4096 fp32 && ADRP_LIB=$L/$1 AB_ONLY=autoreset python tools/reset_ab.py level3 4 PYB_DW COMPETE 4096 fp64 && ADRP_LIB=$L/$1 AB_ONLY=autoreset RACE_POLICY=example python tools/reset_ab.py level0 2 PYB COMPARE 2048 fp32 && ADRP_LIB=$L/$1 AB_ONLY=autoreset python tools/reset_ab.py level0 2 PYB COMPARE 2048 fp32"
}
exec tools/gpu_steps.sh \
  "r3_es_0|400|$(ab libadrp_ab0.so)" \
  "r3_es_1|400|$(ab libadrp_ab1.so)" \
  "r3_es_0b|400|$(ab libadrp_ab0.so)" \
  "r3_es_1b|400|$(ab libadrp_ab1.so)" \
  "r3_obs2_c3p|200|ADRP_LIB=$L/libadrp_devo.so RACE_POLICY=example python tools/race_phases.py level0 2 PYB COMPARE 2048"
