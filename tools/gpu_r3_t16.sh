#!/bin/bash
# round 3: library A/B on the benched race configs (kernel event times, auto-reset on):
# dev (baseline) vs devs (SLP vectorisation) vs devn (out-of-line fp64 contact GJK)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
L=gym_pybullet_adrp_amd
ab() {  # lib
  echo "ADRP_LIB=$L/$1 AB_ONLY=autoreset python tools/reset_ab.py level3 4 PYB_DW COMPETE 4096 fp32 && ADRP_LIB=$L/$1 AB_ONLY=autoreset python tools/reset_ab.py level0 2 PYB COMPARE 2048 fp32 && ADRP_LIB=$L/$1 AB_ONLY=autoreset RACE_POLICY=example python tools/reset_ab.py level0 2 PYB COMPARE 2048 fp32"
}
exec tools/gpu_steps.sh \
  "r3_ab_dev|300|$(ab libadrp_dev.so)" \
  "r3_ab_devs|300|$(ab libadrp_devs.so)" \
  "r3_ab_devn|300|$(ab libadrp_devn.so)" \
  "r3_ab_dev2|300|$(ab libadrp_dev.so)"
