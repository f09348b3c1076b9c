#!/bin/bash
# A/B libadrp_prev.so vs libadrp.so (branch-free sinc exp map in the race step): config 4 both
# precisions, config 3 fp64; then the whole GPU suite
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
C4="--task race --level level3 --drones 4 --envs 4096 --physics PYB_DW --racemode COMPETE --steps 200 --warmup 20 --no-configs"
C3="--task race --level level0 --drones 2 --envs 2048 --steps 200 --warmup 20 --no-configs"
A=gym_pybullet_adrp_amd/libadrp_prev.so; B=gym_pybullet_adrp_amd/libadrp.so
timeout -k 10 300 tools/ab.sh $A $B 2 $C4 --precision fp64 &&
timeout -k 10 300 tools/ab.sh $A $B 2 $C4 --precision fp32 &&
timeout -k 10 300 tools/ab.sh $A $B 1 $C3 --precision fp64 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab6_tests.log 2>&1; rc=$?
tail -3 gpurun_out/ab6_tests.log; exit $rc
