#!/bin/bash
# round 3: race suite after the LDS constant block + XCD-aware block order; phases fp32/fp64; bench race lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
L=gym_pybullet_adrp_amd/libadrp_devt.so
tools/gpu_steps.sh \
  "r3_race|400|python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_race_gpu.py tests/test_sharding_gpu.py" \
  "r3_ph_c4_f32|200|ADRP_LIB=$L python tools/race_phases.py level3 4 PYB_DW COMPETE 4096" \
  "r3_ph_c4_f64|200|ADRP_LIB=$L RACE_PRECISION=fp64 python tools/race_phases.py level3 4 PYB_DW COMPETE 4096" \
  "r3_ph_c3_f32|200|ADRP_LIB=$L python tools/race_phases.py level0 2 PYB COMPARE 2048" \
  "r3_c4_f32|200|python bench.py --no-cpu-baseline --task race --level level3 --drones 4 --envs 4096 --physics PYB_DW --racemode COMPETE --precision fp32 --steps 400 --warmup 40" \
  "r3_c4_f64|200|python bench.py --no-cpu-baseline --task race --level level3 --drones 4 --envs 4096 --physics PYB_DW --racemode COMPETE --precision fp64 --steps 400 --warmup 40"
