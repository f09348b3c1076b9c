#!/bin/bash
# round 3: suite on the fp64 compiled-in constants + per-group commander bounds; GJK iterations of
# the slowest workgroup under the actor; kernel times of the final libadrp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
exec tools/gpu_steps.sh \
  "r3_suite5|600|python -u -m pytest -m gpu -v -s --timeout 300 --timeout-method thread tests" \
  "r3_gjkw_c3p|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devg.so RACE_POLICY=example python tools/race_phases.py level0 2 PYB COMPARE 2048" \
  "r3_kt|400|AB_ONLY=autoreset python tools/reset_ab.py level3 4 PYB_DW COMPETE 4096 fp32 && AB_ONLY=autoreset python tools/reset_ab.py level3 4 PYB_DW COMPETE 4096 fp64 && AB_ONLY=autoreset RACE_POLICY=example python tools/reset_ab.py level0 2 PYB COMPARE 2048 fp32 && AB_ONLY=autoreset RACE_POLICY=example python tools/reset_ab.py level0 2 PYB COMPARE 2048 fp64"
