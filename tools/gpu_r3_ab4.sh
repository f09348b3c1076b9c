#!/bin/bash
# A/B libadrp_ab0.so (round-3 start) vs libadrp.so: hover main line (fp64, fp32), config 4 fp64;
# hover / race / closed-form parity tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
C4="--task race --level level3 --drones 4 --envs 4096 --physics PYB_DW --racemode COMPETE --steps 200 --warmup 20 --no-configs"
A=gym_pybullet_adrp_amd/libadrp_ab0.so; B=gym_pybullet_adrp_amd/libadrp.so
timeout -k 10 300 tools/ab.sh $A $B 2 --no-configs --no-sweep &&
timeout -k 10 300 tools/ab.sh $A $B 1 --no-configs --no-sweep --precision fp32 &&
timeout -k 10 300 tools/ab.sh $A $B 1 $C4 --precision fp64 &&
timeout -k 10 500 python -u -m pytest tests/test_hover_gpu.py tests/test_closed_form_gpu.py tests/test_race_gpu.py tests/test_math_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab4_tests.log 2>&1; rc=$?
tail -3 gpurun_out/ab4_tests.log; exit $rc
