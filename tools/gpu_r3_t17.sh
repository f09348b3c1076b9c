#!/bin/bash
# round 3: compiled-in cf2x physical constants in the quad kernel (ab1) vs runtime constants (ab0),
# both with the out-of-line fp64 contact GJK
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
L=gym_pybullet_adrp_amd
ab() {  # lib
  echo "ADRP_LIB=$L/$1 AB_ONLY=autoreset python tools/reset_ab.py level3 4 PYB_DW COMPETE 4096 fp32 && ADRP_LIB=$L/$1 AB_ONLY=autoreset python tools/reset_ab.py level0 2 PYB COMPARE 2048 fp32 && ADRP_LIB=$L/$1 AB_ONLY=autoreset RACE_POLICY=example python tools/reset_ab.py level0 2 PYB COMPARE 2048 fp32 && ADRP_LIB=$L/$1 AB_ONLY=autoreset python tools/reset_ab.py level3 4 PYB_DW COMPETE 4096 fp64"
}
exec tools/gpu_steps.sh \
  "r3_ab_0|400|$(ab libadrp_ab0.so)" \
  "r3_ab_1|400|$(ab libadrp_ab1.so)" \
  "r3_ab_0b|400|$(ab libadrp_ab0.so)" \
  "r3_ab_1b|400|$(ab libadrp_ab1.so)"
