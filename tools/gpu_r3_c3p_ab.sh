#!/bin/bash
# contact search A/B: libadrp_ab0.so (before) vs libadrp.so (after) on the actor-driven config 3,
# both precisions; GJK call counts of the new tree (GJK-stats build); the race parity tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
C3P="--task race --level level0 --drones 2 --envs 2048 --policy example --steps 200 --warmup 20 --no-configs"
A=gym_pybullet_adrp_amd/libadrp_ab0.so; B=gym_pybullet_adrp_amd/libadrp.so
timeout -k 10 300 tools/ab.sh $A $B 2 $C3P --precision fp32 &&
timeout -k 10 300 tools/ab.sh $A $B 2 $C3P --precision fp64 &&
ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devg.so RACE_POLICY=example timeout -k 10 200 python tools/race_phases.py level0 2 PYB COMPARE 2048 > gpurun_out/phases_c3p_gjk.log 2>&1 &&
grep -o '"gjk": {[^}]*}' gpurun_out/phases_c3p_gjk.log; grep -o '"wave_total_p50_p90_p99_max": [^]]*]' gpurun_out/phases_c3p_gjk.log;
timeout -k 10 400 python -u -m pytest tests/test_race_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/race_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/race_gpu.log; exit $rc
