#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devt.so RACE_POLICY=example timeout -k 10 200 python tools/race_phases.py level0 2 PYB COMPARE 2048 > gpurun_out/phases_c3p.log 2>&1; echo "c3p rc $?"
grep config gpurun_out/phases_c3p.log || tail -5 gpurun_out/phases_c3p.log
