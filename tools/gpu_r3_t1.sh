#!/bin/bash
# round 3: the new parity tests (config 5 shards, Newton's first law, config-4-size sub-step,
# hover truncation margins, GND_DRAG_DW full-size subset)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread \
  tests/test_sharding_gpu.py tests/test_closed_form_gpu.py tests/test_race_gpu.py tests/test_hover_gpu.py \
  -k "config5 or packed or newton or free_fall or config4_size or full_size_subset or teacher_forced_step or benched" \
  > gpurun_out/r3_t1.log 2>&1
rc=$?
tail -30 gpurun_out/r3_t1.log
exit $rc
