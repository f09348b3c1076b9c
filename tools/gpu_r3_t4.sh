#!/bin/bash
# round 3: full GPU suite + the default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
tools/gpu_steps.sh \
  "r3_suite|1000|python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests" \
  "r3_bench|600|python -u bench.py --steps 20 --warmup 5"
