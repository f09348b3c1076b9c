#!/bin/bash
# round 3: downwash partner positions by DPP row broadcasts (ab1) vs ds_bpermute (ab0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
L=gym_pybullet_adrp_amd
ab() {  # lib
  echo "ADRP_LIB=$L/$1 AB_ONLY=autoreset python tools/reset_ab.py level3 4 PYB_DW COMPETE 4096 fp32 && ADRP_LIB=$L/$1 AB_ONLY=autoreset python tools/reset_ab.py level3 4 PYB_DW COMPETE 4096 fp64"
}
exec tools/gpu_steps.sh \
  "r3_dw_0|300|$(ab libadrp_ab0.so)" \
  "r3_dw_1|300|$(ab libadrp_ab1.so)" \
  "r3_dw_0b|300|$(ab libadrp_ab0.so)" \
  "r3_dw_1b|300|$(ab libadrp_ab1.so)" \
  "r3_dw_test|300|ADRP_LIB=$L/libadrp_ab1.so python -u -m pytest -m gpu -v --timeout 250 --timeout-method thread tests/test_race_gpu.py -k 'quad_matches and PYB_DW'"
