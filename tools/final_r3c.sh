#!/bin/bash
# round-3 final evidence of the late tree: config 4 fp64 A/B against the round-3 start, the GPU suite,
# smoke, the default bench line (final_r3a.sh), rocprof stats of the graph-replayed launches
# (final_r3b.sh) and the PMC passes (pmc_r3.sh)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
mkdir -p gpurun_out
C4="--task race --level level3 --drones 4 --envs 4096 --physics PYB_DW --racemode COMPETE --steps 200 --warmup 20 --no-configs"
timeout -k 10 300 tools/ab.sh gym_pybullet_adrp_amd/libadrp_ab0.so gym_pybullet_adrp_amd/libadrp.so 1 $C4 --precision fp64 || exit $?
tools/final_r3a.sh; rc=$?
[ $rc -ne 0 ] && exit $rc
tools/final_r3b.sh; rc=$?
[ $rc -ne 0 ] && exit $rc
tools/pmc_r3.sh > gpurun_out/pmc_r3.log 2>&1; rc=$?
tail -n 3 gpurun_out/pmc_r3.log; exit $rc
