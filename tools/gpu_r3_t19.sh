#!/bin/bash
# round 3: obs-phase split (bounds / GJK pool / row / compete rows) under the actor and in config 4;
# hardcoded / commander tests with the yaw floor
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
exec tools/gpu_steps.sh \
  "r3_obs_c3p|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devo.so RACE_POLICY=example python tools/race_phases.py level0 2 PYB COMPARE 2048" \
  "r3_obs_c4|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devo.so python tools/race_phases.py level3 4 PYB_DW COMPETE 4096" \
  "r3_cmd5|300|python -u -m pytest -m gpu -v -s --timeout 250 --timeout-method thread tests/test_commander_gpu.py" \
  "r3_tobs_c4|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devt.so python tools/race_phases.py level3 4 PYB_DW COMPETE 4096"
