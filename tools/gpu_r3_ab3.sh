#!/bin/bash
# A/B libadrp_ab0.so (round-3 start) vs libadrp.so (fp64 chain forms): hover main line, config 4 in
# both precisions, actor-driven config 3; then the whole GPU suite and smoke
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
C3P="--task race --level level0 --drones 2 --envs 2048 --policy example --steps 200 --warmup 20 --no-configs"
C4="--task race --level level3 --drones 4 --envs 4096 --physics PYB_DW --racemode COMPETE --steps 200 --warmup 20 --no-configs"
A=gym_pybullet_adrp_amd/libadrp_ab0.so; B=gym_pybullet_adrp_amd/libadrp.so
timeout -k 10 300 tools/ab.sh $A $B 2 --no-configs --no-sweep &&
timeout -k 10 300 tools/ab.sh $A $B 2 $C4 --precision fp64 &&
timeout -k 10 300 tools/ab.sh $A $B 1 $C4 --precision fp32 &&
timeout -k 10 300 tools/ab.sh $A $B 1 $C3P --precision fp32 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r3_pytest_gpu.log
[ $rc -eq 0 ] && timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r3_smoke.log 2>&1; rc2=$?
tail -2 gpurun_out/r3_smoke.log; exit $(( rc | rc2 ))
