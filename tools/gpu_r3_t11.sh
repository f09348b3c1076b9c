#!/bin/bash
# round 3: capped GJK queries under the actor (fp32 / fp64) and random targets (config 4); hardcoded
# teacher forcing re-run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
exec tools/gpu_steps.sh \
  "r3_cap_c3p|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devg.so RACE_POLICY=example python tools/gjk_capped.py level0 2 PYB COMPARE 2048 300" \
  "r3_cap_c3p64|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devg.so RACE_POLICY=example RACE_PRECISION=fp64 python tools/gjk_capped.py level0 2 PYB COMPARE 2048 300" \
  "r3_cap_c4|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devg.so python tools/gjk_capped.py level3 4 PYB_DW COMPETE 4096 300" \
  "r3_cmd4|400|python -u -m pytest -m gpu -v -s --timeout 250 --timeout-method thread tests/test_commander_gpu.py tests/test_race_gpu.py -k 'hardcoded or reset or quad_matches or enable_commands'"
