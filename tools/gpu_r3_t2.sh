#!/bin/bash
# round 3: fp64 math probe + diagnosis of the config-4-size sub-step + remaining new tests + f64 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
tools/gpu_steps.sh \
  "r3_math|300|python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests/test_math_gpu.py" \
  "r3_diag|300|python -u tools/diag_c4sub.py PYB_DW" \
  "r3_t2|900|python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests/test_race_gpu.py tests/test_hover_gpu.py tests/test_closed_form_gpu.py -k 'config4_size or full_size_subset or teacher_forced_step or benched or fp64 or newton or free_fall'" \
  "r3_ab64|400|tools/ab.sh gym_pybullet_adrp_amd/libadrp_base.so gym_pybullet_adrp_amd/libadrp.so 3 --precision fp64 --steps 2000 --warmup 200 --no-configs --no-sweep"
