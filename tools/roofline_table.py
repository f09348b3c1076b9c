"""Fold a `tools/gpu.sh prof TAG` run into per-grid rocprof statistics and one roofline table.

usage: python tools/roofline_table.py gpurun_out/TAG ROUND [BENCH_JSON ...]
       (e.g. gpurun_out/r6p r6 profiles/r6_bench.json profiles/r6_bench_k20.json)

For every workload directory prof_<cfg>/ of the run (rocprofv3 --kernel-trace of `bench.py
--graph-only ...`, whose JSON line is in prof_<cfg>.log):
  - the step kernel's launches are split by grid size: the benched env count (the most frequent
    grid) and, for the hover line, the roofline sweep's larger grids (bench.py roofline_sweep);
    profiles/ROUND_rocprof_<cfg>_E<E>_kernel_stats.csv holds one row per (kernel, grid), so the
    mean of the benched launches is never mixed with the sweep's;
  - profiles/ROUND_roofline.json holds, per workload: algorithmic bytes (and flops, race) per launch
    from the bench record, the rocprof mean / median at the benched grid, the frac recomputed from
    them, the bench line's own frac (HIP events around the graph-replayed timed region / K) and the
    ratio of the two, and the PMC counter traffic (profiles/pmc_traffic.json); for the hover line
    the sweep rows with their own rocprof means and fractions;
  - for every BENCH_JSON given (full bench lines, not under the profiler): each workload's `frac`
    from that line's summary next to the rocprof-recomputed one.
"""
import csv
import json
import os
import sys
from collections import defaultdict

import numpy as np

HBM_PEAK = 8000.0
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STEP_KERNELS = ("hover_step_kernel", "race_step_kernel", "race_quad_kernel", "race_step")


def bench_line(log):
    for line in reversed(open(log).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    return None


def launches(trace):
    out = defaultdict(list)
    with open(trace) as fh:
        for r in csv.DictReader(fh):
            name = r["Kernel_Name"]
            if not any(k in name for k in STEP_KERNELS):
                continue
            grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            out[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    return out


def short(name):
    s = name.split("(")[0]
    return s.replace("void adrp::", "").replace("adrp::", "")


SUMMARY_KEY = {"c2_fp64": "value", "c2_fp32": "config2_f32", "c3_fp64": "config3", "c3_fp32": "config3_f32",
               "c3p_fp64": "config3_policy", "c3p_fp32": "config3_policy_f32", "c4_fp64": "config5",
               "c4_fp32": "config5_f32"}


def main(run_dir, rnd, benches=()):
    pmc = {}
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(p):
        pmc = json.load(open(p))
    table = {"run": os.path.basename(os.path.normpath(run_dir)), "hbm_peak_GBps": HBM_PEAK,
             "note": "frac_rocprof = bytes_per_launch / rocprof mean kernel duration at the benched grid / peak; "
                     "frac_bench = the same bytes / the bench line's kernel_us (HIP events around the graph-replayed "
                     "timed region / K, which includes the graph's inter-launch gaps)", "workloads": {}}
    for d in sorted(os.listdir(run_dir)):
        if not d.startswith("prof_") or not os.path.isdir(os.path.join(run_dir, d)):
            continue
        cfg = d[len("prof_"):]
        trace = [os.path.join(dp, f) for dp, _, fs in os.walk(os.path.join(run_dir, d)) for f in fs
                 if f.endswith("kernel_trace.csv")]
        log = os.path.join(run_dir, d + ".log")
        if not trace or not os.path.exists(log):
            continue
        rec = bench_line(log)
        L = launches(trace[0])
        if not L or rec is None:
            continue
        main_key = max(L, key=lambda k: len(L[k]))
        rows = []
        for (name, grid), ns in sorted(L.items(), key=lambda kv: kv[0][1]):
            a = np.asarray(ns, float)
            rows.append({"Name": short(name), "Grid": grid, "Calls": len(a), "TotalNs": int(a.sum()),
                         "AverageNs": float(a.mean()), "MedianNs": float(np.median(a)), "MinNs": int(a.min()),
                         "MaxNs": int(a.max()), "P99Ns": float(np.percentile(a, 99))})
        rl = rec["roofline"]
        E = rec.get("envs_per_gpu") or 4096
        out_csv = os.path.join(ROOT, "profiles", f"{rnd}_rocprof_{cfg}_E{E}_kernel_stats.csv")
        with open(out_csv, "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=list(rows[0]))
            w.writeheader()
            for r in rows:
                if (r["Grid"] == main_key[1]):
                    w.writerow(r)
        mean_us = float(np.mean(L[main_key])) / 1e3
        bpl = rl.get("bytes_per_launch") or (rl.get("hbm") or {}).get("bytes_per_launch")
        ent = {"kernel": short(main_key[0]), "grid": main_key[1], "envs": E, "launches": len(L[main_key]),
               "rocprof_mean_us": mean_us, "rocprof_median_us": float(np.median(L[main_key])) / 1e3,
               "rocprof_p99_us": float(np.percentile(L[main_key], 99)) / 1e3,
               "rocprof_max_us": float(np.max(L[main_key])) / 1e3,
               "max_over_mean": float(np.max(L[main_key])) / float(np.mean(L[main_key])),
               "bytes_per_launch": bpl, "bench_kernel_us": rl["kernel_us"],
               "stats_csv": os.path.relpath(out_csv, ROOT)}
        if rl["bound"] == "hbm":
            ent["frac_rocprof"] = bpl / (mean_us * 1e-6) / 1e9 / HBM_PEAK
            ent["frac_bench"] = rl["frac"]
            ent["traffic"] = rl.get("traffic")
        else:
            fl = rl.get("flops_per_launch")
            ent.update({"bound": "valu", "flops_per_launch": fl, "peak_TFLOPs": rl["peak"],
                        "frac_rocprof": None if fl is None else fl / (mean_us * 1e-6) / 1e12 / rl["peak"],
                        "frac_bench": rl["frac"],
                        "hbm_frac_rocprof": bpl / (mean_us * 1e-6) / 1e9 / HBM_PEAK,
                        "hbm_frac_bench": rl["hbm"]["frac"], "traffic": rl.get("traffic")})
        if ent.get("frac_rocprof") and ent.get("frac_bench"):
            ent["bench_over_rocprof"] = ent["frac_bench"] / ent["frac_rocprof"]
        sweep = rl.get("sweep")
        others = sorted((k for k in L if k != main_key and k[0] == main_key[0]), key=lambda k: k[1])
        if sweep and others:
            srows = []
            for s, k in zip(sorted(sweep, key=lambda r: r["envs"]), others):
                m = float(np.mean(L[k])) / 1e3
                b = bpl / E * s["envs"]
                srows.append({"envs": s["envs"], "grid": k[1], "launches": len(L[k]), "rocprof_mean_us": m,
                              "bytes_per_launch": b, "frac_rocprof": b / (m * 1e-6) / 1e9 / HBM_PEAK,
                              "bench_kernel_us": s["kernel_us"], "frac_bench": s["frac"]})
                with open(out_csv.replace(f"_E{E}_", f"_E{s['envs']}_"), "w", newline="") as fh:
                    w = csv.DictWriter(fh, fieldnames=list(rows[0]))
                    w.writeheader()
                    for r in rows:
                        if r["Grid"] == k[1]:
                            w.writerow(r)
            ent["sweep"] = srows
        table["workloads"][cfg] = ent
    for b in benches:
        line = bench_line(b)
        if line is None or "summary" not in line:
            continue
        name = os.path.relpath(b, ROOT)
        table.setdefault("bench_records", {})[name] = {
            "cmd_form": f"K = {line['steps']}, W = {line['warmup']}", "value": line["value"]}
        for cfg, ent in table["workloads"].items():
            rec = line["summary"].get(SUMMARY_KEY.get(cfg, ""), {})
            if "frac" in rec and rec["frac"] and ent.get("frac_rocprof"):
                ent.setdefault("bench_lines", {})[name] = {
                    "kernel_us": rec.get("k_us"), "frac": rec["frac"],
                    "frac_over_rocprof": rec["frac"] / ent["frac_rocprof"]}
    out = os.path.join(ROOT, "profiles", f"{rnd}_roofline.json")
    with open(out, "w") as fh:
        json.dump(table, fh, indent=1)
    for cfg, e in table["workloads"].items():
        print(f"{cfg:10s} {e['kernel'][:60]:60s} E={e['envs']:6d} n={e['launches']:5d} rocprof {e['rocprof_mean_us']:7.2f} us "
              f"bench {e['bench_kernel_us']:7.2f} us frac_rocprof {e.get('frac_rocprof') or 0:.4f} "
              f"frac_bench {e.get('frac_bench') or 0:.4f}")
        for bn, bl in e.get("bench_lines", {}).items():
            print(f"{'':10s} {bn}: kernel {bl['kernel_us']} us frac {bl['frac']:.4f} ({bl['frac_over_rocprof']:.3f} x rocprof)")
        for s in e.get("sweep", []):
            print(f"{'':10s} sweep E={s['envs']:8d} rocprof {s['rocprof_mean_us']:8.2f} us frac {s['frac_rocprof']:.3f} "
                  f"(bench {s['frac_bench']:.3f})")
    print("wrote", out)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
