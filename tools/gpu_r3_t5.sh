#!/bin/bash
# round 3: phase profiles fp32 vs fp64 quad race kernels, FETCH_SIZE calibration, config-4-size test
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/calib
L=gym_pybullet_adrp_amd/libadrp_devt.so
R="$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "r3_ph_c4_f32|200|ADRP_LIB=$L python tools/race_phases.py level3 4 PYB_DW COMPETE 4096" \
  "r3_ph_c4_f64|200|ADRP_LIB=$L RACE_PRECISION=fp64 python tools/race_phases.py level3 4 PYB_DW COMPETE 4096" \
  "r3_ph_c3_f64|200|ADRP_LIB=$L RACE_PRECISION=fp64 python tools/race_phases.py level0 2 PYB COMPARE 2048" \
  "r3_calib_f|90|cd /tmp && TMPDIR=/tmp timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/calib/f -o p -- $R/tools/fetch_calib" \
  "r3_calib_w|90|cd /tmp && TMPDIR=/tmp timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/calib/w -o p -- $R/tools/fetch_calib" \
  "r3_c4size|400|python -u -m pytest -m gpu -x -v -s --timeout 350 --timeout-method thread tests/test_race_gpu.py -k config4_size"
