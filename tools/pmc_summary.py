"""Summarise rocprofv3 --pmc CSVs: mean per-dispatch counter of the hover step kernel."""
import csv
import glob
import json
import sys

out = {}
for path in sys.argv[1:]:
    for f in glob.glob(path + "/**/*counter_collection.csv", recursive=True):
        rows = list(csv.DictReader(open(f)))
        for r in rows:
            if "hover_step_kernel" not in r.get("Kernel_Name", ""):
                continue
            key = (f.split("/")[-3] if "/" in f else f, r["Counter_Name"])
            out.setdefault(key, []).append(float(r["Counter_Value"]))
res = {f"{k[0]}:{k[1]}": {"dispatches": len(v), "mean": sum(v) / len(v), "min": min(v), "max": max(v)}
       for k, v in out.items()}
print(json.dumps(res, indent=1))
