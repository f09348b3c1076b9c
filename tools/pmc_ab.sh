#!/bin/bash
# One PMC pass (instruction counts + wave cycles) of the config-4 race step for each library given,
# fp64 and fp32: whether a kernel change moved the executed instruction mix.
# usage: tools/pmc_ab.sh TAG LIB [LIB ...]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
O="$R/gpurun_out/pmcab_$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM"
for P in fp64 fp32; do
  for LIB in "$@"; do
    n="$(basename "$LIB" .so)_$P"
    export ADRP_LIB="$R/$LIB"
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$O/$n" -o p -- python3 "$R/tools/pmc_race_steps.py" level3 4 PYB_DW COMPETE 4096 30 "$R" "$P" > "$O/$n.log" 2>&1
    rc=$?
    echo "=== $n exit $rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
python3 - "$O" <<'PY'
import csv, glob, statistics, sys, os
o = sys.argv[1]
for d in sorted(glob.glob(o + "/*/")):
    vals = {}
    for f in glob.glob(d + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "race_step" in r.get("Kernel_Name", ""):
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    med = {k: statistics.median(v[8:] if len(v) > 16 else v) / 1024 for k, v in vals.items()}
    print(os.path.basename(d.rstrip("/")), " ".join(f"{k.replace('SQ_', '')}={v:.0f}" for k, v in sorted(med.items())))
PY
