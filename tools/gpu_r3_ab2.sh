#!/bin/bash
# A/B libadrp_ab0.so (before) vs libadrp.so (after): fp64 hover main line, config 4 fp64 / fp32,
# actor-driven config 3 fp32 / fp64; GJK call counts (GJK-stats build); race + hover parity tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
C3P="--task race --level level0 --drones 2 --envs 2048 --policy example --steps 200 --warmup 20 --no-configs"
C4="--task race --level level3 --drones 4 --envs 4096 --physics PYB_DW --racemode COMPETE --steps 200 --warmup 20 --no-configs"
A=gym_pybullet_adrp_amd/libadrp_ab0.so; B=gym_pybullet_adrp_amd/libadrp.so
timeout -k 10 300 tools/ab.sh $A $B 2 --no-configs --no-sweep &&
timeout -k 10 300 tools/ab.sh $A $B 2 $C4 --precision fp64 &&
timeout -k 10 300 tools/ab.sh $A $B 2 $C4 --precision fp32 &&
timeout -k 10 300 tools/ab.sh $A $B 2 $C3P --precision fp32 &&
timeout -k 10 300 tools/ab.sh $A $B 2 $C3P --precision fp64 &&
ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devg.so RACE_POLICY=example timeout -k 10 200 python tools/race_phases.py level0 2 PYB COMPARE 2048 > gpurun_out/phases_c3p_gjk.log 2>&1 &&
grep -o '"gjk": {[^}]*}' gpurun_out/phases_c3p_gjk.log; grep -o '"wave_total_p50_p90_p99_max": [^]]*]' gpurun_out/phases_c3p_gjk.log;
timeout -k 10 500 python -u -m pytest tests/test_race_gpu.py tests/test_hover_gpu.py tests/test_closed_form_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/race_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/race_gpu.log; exit $rc
