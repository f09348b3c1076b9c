#!/bin/bash
# round 3: full GPU suite with the fp64 contact GJK in the fp32 kernels and the cycle exit; reset A/B;
# phases; instruction-mix PMC passes of config 4 (fp32, fp64)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
tools/gpu_steps.sh \
  "r3_suite3|600|python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests" \
  "r3_reset_ab3|200|python tools/reset_ab.py level3 4 PYB_DW COMPETE 4096 fp32 && python tools/reset_ab.py level0 2 PYB COMPARE 2048 fp32" \
  "r3_ph3_c4|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devt.so python tools/race_phases.py level3 4 PYB_DW COMPETE 4096" \
  "r3_ph3_c3p|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devt.so RACE_POLICY=example python tools/race_phases.py level0 2 PYB COMPARE 2048"
rc=$?
[ $rc -ge 124 ] && exit $rc
tools/pmc_mix.sh mix_c4_f32 level3 4 PYB_DW COMPETE 4096 fp32 > gpurun_out/pmc_mix_c4_f32.log 2>&1 || exit $?
tools/pmc_mix.sh mix_c4_f64 level3 4 PYB_DW COMPETE 4096 fp64 > gpurun_out/pmc_mix_c4_f64.log 2>&1 || exit $?
exit $rc
