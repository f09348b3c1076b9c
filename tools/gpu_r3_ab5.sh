#!/bin/bash
# A/B libadrp_prev.so (final-evidence tree) vs libadrp.so (sinc exp map in the hover step): hover main
# line both precisions; then the hover / closed-form / math GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
A=gym_pybullet_adrp_amd/libadrp_prev.so; B=gym_pybullet_adrp_amd/libadrp.so
timeout -k 10 300 tools/ab.sh $A $B 2 --no-configs --no-sweep &&
timeout -k 10 300 tools/ab.sh $A $B 2 --no-configs --no-sweep --precision fp32 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab5_tests.log 2>&1; rc=$?
tail -3 gpurun_out/ab5_tests.log; exit $rc
