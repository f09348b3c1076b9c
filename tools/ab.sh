#!/bin/bash
# A/B two libadrp builds on the same GPU box, interleaved (A B A B ...), one bench.py line each.
# usage: tools/ab.sh LIB_A LIB_B ROUNDS [bench.py args...]
# prints per run: lib, kernel_us (dispatch events), us per step (graph replay), value
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
A="$1"; B="$2"; R="$3"; shift 3
mkdir -p gpurun_out
for r in $(seq 1 "$R"); do
  for L in "$A" "$B"; do
    ADRP_LIB="$L" timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab_last.log 2>&1 || { tail -5 gpurun_out/ab_last.log; exit 1; }
    python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/ab_last.log') if l.startswith('{')][-1])
print(f\"{sys.argv[1]:40s} kernel_us {d['roofline']['kernel_us']:8.3f} med {d['roofline']['kernel_us_median']:8.3f} step_us {d['ms_per_step']*1e3:8.3f} value {d['value']:.4e}\")
" "$L"
  done
done
