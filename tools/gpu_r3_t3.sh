#!/bin/bash
# round 3: fixed config-4-size test, new command/registry/vec_env tests, new bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
tools/gpu_steps.sh \
  "r3_c4size|300|python -u -m pytest -m gpu -x -v -s --timeout 250 --timeout-method thread tests/test_race_gpu.py -k config4_size" \
  "r3_cmd|300|python -u -m pytest -m gpu -v --timeout 250 --timeout-method thread tests/test_commander_gpu.py tests/test_registry.py tests/test_vec_env.py" \
  "r3_bench|600|python -u bench.py --steps 20 --warmup 5"
