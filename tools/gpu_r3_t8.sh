#!/bin/bash
# round 3: where the quad reset's cycles go (reset sub-phase marks), hover phases fp32 / fp64
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
tools/gpu_steps.sh \
  "r3_rp_c4_f32|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devr.so python tools/race_phases.py level3 4 PYB_DW COMPETE 4096" \
  "r3_rp_c4_f64|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devr.so RACE_PRECISION=fp64 python tools/race_phases.py level3 4 PYB_DW COMPETE 4096" \
  "r3_hph|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devt.so python tools/hover_phases.py 4096" \
  "r3_hph64|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devt.so HOVER_PRECISION=fp64 python tools/hover_phases.py 4096"
tools/gpu_steps.sh \
  "r3_ph_c3p_f32|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devt.so RACE_POLICY=example python tools/race_phases.py level0 2 PYB COMPARE 2048" \
  "r3_ph_c3p_f64|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devt.so RACE_POLICY=example RACE_PRECISION=fp64 python tools/race_phases.py level0 2 PYB COMPARE 2048"
tools/gpu_steps.sh \
  "r3_noise|300|python -u -m pytest -m gpu -v --timeout 250 --timeout-method thread tests/test_noise_injection.py tests/test_race_gpu.py -k 'injected or teacher_forced_step or quad_matches or full_size_subset'"
tools/gpu_steps.sh \
  "r3_cmd|400|python -u -m pytest -m gpu -v -s --timeout 350 --timeout-method thread tests/test_commander_gpu.py"
