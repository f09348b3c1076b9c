#!/bin/bash
# round 3: capped GJK contact queries under the actor (pre-stall GJK-stats build), fp32, two seeds' worth
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
exec tools/gpu_steps.sh \
  "r3_cap2_c3p|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devg.so RACE_POLICY=example python tools/gjk_capped.py level0 2 PYB COMPARE 2048 300"
