#!/bin/bash
# round-3 evidence, part a: the GPU test suite, smoke, the driver's default bench line
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
mkdir -p gpurun_out
T=(
  "r3_pytest_gpu|600|cd $R && python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread"
  "r3_smoke|200|cd $R && python -c 'import __graft_entry__ as g; g.smoke()'"
  "r3_bench|900|cd $R && python bench.py"
)
exec "$R/tools/gpu_steps.sh" "${T[@]}"
