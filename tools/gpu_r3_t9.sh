#!/bin/bash
# round 3: hardcoded-controller teacher forcing with per-step detail; fp32 noise replay detail;
# slowest-wave phase breakdown for config 4 and the actor-driven config 3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
exec tools/gpu_steps.sh \
  "r3_cmd2|300|python -u -m pytest -m gpu -v -s --timeout 250 --timeout-method thread tests/test_commander_gpu.py -k hardcoded_controller_teacher" \
  "r3_noise2|200|python -u -m pytest -m gpu -v --timeout 150 --timeout-method thread tests/test_noise_injection.py" \
  "r3_ph_c4_slow|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devt.so python tools/race_phases.py level3 4 PYB_DW COMPETE 4096" \
  "r3_ph_c3p_slow|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devt.so RACE_POLICY=example python tools/race_phases.py level0 2 PYB COMPARE 2048"
