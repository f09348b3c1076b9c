#!/bin/bash
# phase profile of the benched race kernels (timing dev build), random targets and actor-driven
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
L=gym_pybullet_adrp_amd/libadrp_devt.so
ADRP_LIB=$L timeout -k 10 200 python tools/race_phases.py level0 2 PYB COMPARE 2048 > gpurun_out/phases_c3.log 2>&1; echo "c3 rc $?"
ADRP_LIB=$L RACE_POLICY=example timeout -k 10 200 python tools/race_phases.py level0 2 PYB COMPARE 2048 > gpurun_out/phases_c3p.log 2>&1; echo "c3p rc $?"
ADRP_LIB=$L timeout -k 10 200 python tools/race_phases.py level3 4 PYB_DW COMPETE 4096 > gpurun_out/phases_c4.log 2>&1; echo "c4 rc $?"
tail -2 gpurun_out/phases_c3.log gpurun_out/phases_c3p.log gpurun_out/phases_c4.log
