#!/bin/bash
# A/B two libadrp builds / run-time switches on the same GPU box, interleaved (A B A B ...), one
# bench.py line each.  An arm is a library path, optionally followed by ,VAR=value switches, e.g.
#   tools/ab.sh gym_pybullet_adrp_amd/libadrp.so,ADRP_RACE_QUAD=0 gym_pybullet_adrp_amd/libadrp.so 3 --task race
# usage: tools/ab.sh ARM_A ARM_B ROUNDS [bench.py args...]
# prints per run: arm, kernel_us (events around the graph-replayed timed region / K), eager dispatch events, us per step, value
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
A="$1"; B="$2"; R="$3"; shift 3
mkdir -p gpurun_out
for r in $(seq 1 "$R"); do
  for ARM in "$A" "$B"; do
    IFS=',' read -r -a parts <<< "$ARM"
    envs=("ADRP_LIB=${parts[0]}" "${parts[@]:1}")
    env "${envs[@]}" timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab_last.log 2>&1 || { tail -5 gpurun_out/ab_last.log; exit 1; }
    python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/ab_last.log') if l.startswith('{')][-1])
r=d['roofline']
print(f\"{sys.argv[1]:60s} kernel_us {r['kernel_us']:8.3f} eager {r.get('eager_dispatch_us', float('nan')):8.3f} step_us {d['ms_per_step']*1e3:8.3f} value {d['value']:.4e}\")
" "$ARM"
  done
done
