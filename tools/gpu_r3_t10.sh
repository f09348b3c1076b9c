#!/bin/bash
# round 3: re-run of the hardcoded / noise tests with the documented exclusions; the auto-reset's
# cost (autoreset on / off); GJK counters under the actor (config 3); instruction-cache counters
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/pmc_r3ic
R="$(pwd)"
IC="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"
exec tools/gpu_steps.sh \
  "r3_cmd3|300|python -u -m pytest -m gpu -v -s --timeout 250 --timeout-method thread tests/test_commander_gpu.py -k hardcoded_controller_teacher" \
  "r3_noise3|200|python -u -m pytest -m gpu -v --timeout 150 --timeout-method thread tests/test_noise_injection.py" \
  "r3_reset_ab|200|python tools/reset_ab.py level3 4 PYB_DW COMPETE 4096 fp32 && python tools/reset_ab.py level3 4 PYB_DW COMPETE 4096 fp64 && python tools/reset_ab.py level0 2 PYB COMPARE 2048 fp32" \
  "r3_gjk_c3p|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devg.so RACE_POLICY=example python tools/race_phases.py level0 2 PYB COMPARE 2048" \
  "r3_gjk_c4|200|ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devg.so python tools/race_phases.py level3 4 PYB_DW COMPETE 4096" \
  "r3_ic_c4|120|cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc $IC --output-format csv -d $R/gpurun_out/pmc_r3ic/c4 -o p -- python3 $R/tools/pmc_race_steps.py level3 4 PYB_DW COMPETE 4096 40 $R" \
  "r3_ic_c3|120|cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc $IC --output-format csv -d $R/gpurun_out/pmc_r3ic/c3 -o p -- python3 $R/tools/pmc_race_steps.py level0 2 PYB COMPARE 2048 40 $R" \
  "r3_ic_h|120|cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc $IC --output-format csv -d $R/gpurun_out/pmc_r3ic/h -o p -- python3 $R/tools/pmc_steps.py 4096 60 fp64 $R"
