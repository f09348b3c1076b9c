#!/bin/bash
# One GPU session: parity tests, bench, kernel-trace profile, HBM PMC passes (E = 4096 and 2^20).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r1}"
exec "$R/tools/gpu_steps.sh" \
  "pytest_gpu|400|cd $R && python -m pytest tests -m gpu -x -q" \
  "bench|300|cd $R && python bench.py" \
  "prof_$TAG|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o bench -- python3 $R/bench.py --steps 2000 --no-cpu-baseline" \
  "pmcf4k|200|cd /tmp && export TMPDIR=/tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcf4k_$TAG -o p -- python3 $R/tools/pmc_steps.py 4096 200 fp32 $R" \
  "pmcw4k|200|cd /tmp && export TMPDIR=/tmp && rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcw4k_$TAG -o p -- python3 $R/tools/pmc_steps.py 4096 200 fp32 $R" \
  "pmcf1m|200|cd /tmp && export TMPDIR=/tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcf1m_$TAG -o p -- python3 $R/tools/pmc_steps.py 1048576 40 fp32 $R" \
  "pmcw1m|200|cd /tmp && export TMPDIR=/tmp && rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcw1m_$TAG -o p -- python3 $R/tools/pmc_steps.py 1048576 40 fp32 $R"
