#!/bin/bash
# A/B/n: several libadrp builds / run-time switches on the same GPU box, interleaved round-robin,
# one bench.py line each (tools/ab.sh with any number of arms).  BENCH_ARGS holds the bench.py args.
# usage: BENCH_ARGS="--task race ..." tools/abn.sh ROUNDS ARM1 ARM2 ...
#   an arm is a library path, optionally followed by ,VAR=value switches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R="$1"; shift
mkdir -p gpurun_out
for r in $(seq 1 "$R"); do
  for ARM in "$@"; do
    IFS=',' read -r -a parts <<< "$ARM"
    envs=("ADRP_LIB=${parts[0]}" "${parts[@]:1}")
    # shellcheck disable=SC2086
    env "${envs[@]}" timeout -k 10 120 python bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/abn_last.log 2>&1 || { tail -5 gpurun_out/abn_last.log; exit 1; }
    python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/abn_last.log') if l.startswith('{')][-1])
r=d['roofline']
print(f\"{sys.argv[1]:60s} kernel_us {r['kernel_us']:8.3f} step_us {d['ms_per_step']*1e3:8.3f} value {d['value']:.4e}\", flush=True)
" "$ARM"
  done
done
