#!/bin/bash
# hover phase profile (timing build) at E = 4096 in both precisions
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devt.so HOVER_PRECISION=fp64 timeout -k 10 200 python tools/hover_phases.py 4096 > gpurun_out/hph_fp64.log 2>&1 &&
ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devt.so HOVER_PRECISION=fp32 timeout -k 10 200 python tools/hover_phases.py 4096 > gpurun_out/hph_fp32.log 2>&1; rc=$?
tail -20 gpurun_out/hph_fp64.log gpurun_out/hph_fp32.log; exit $rc
