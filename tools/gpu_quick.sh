#!/bin/bash
# GPU suite + the race bench lines (config 4, config 3, config 3 with the actor)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc $?"
tail -3 gpurun_out/pytest_gpu.log
for spec in "c4|--task race --level level3 --drones 4 --envs 4096 --physics PYB_DW --racemode COMPETE" "c3|--task race --level level0 --drones 2 --envs 2048" "c3p|--task race --level level0 --drones 2 --envs 2048 --policy example"; do
  n="${spec%%|*}"; a="${spec#*|}"
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --warmup 20 $a > gpurun_out/bench_$n.log 2>&1
  python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/bench_$n.log') if l.startswith('{')][-1])
print('$n', f\"kernel_us {d['roofline']['kernel_us']:.2f} med {d['roofline']['kernel_us_median']:.2f} step_us {d['ms_per_step']*1e3:.2f} value {d['value']:.4e}\")
"
done
