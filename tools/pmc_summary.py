"""Summarise rocprofv3 --pmc passes of a step kernel into per-launch HBM bytes.

usage: python tools/pmc_summary.py OUT.json KEY FETCH_DIR WRITE_DIR [KEY FETCH_DIR WRITE_DIR ...]
       python tools/pmc_summary.py --valu OUT.json KEY FLOPS_DIR BUSY_DIR [...]
       python tools/pmc_summary.py --alg OUT.json KEY FLOPS_DIR DRONES_PER_LAUNCH [...]

--valu: the VALU roofline of a step kernel from two passes, FLOPS_DIR =
SQ_INSTS_VALU_FLOPS_FP32, SQ_INSTS_VALU_FLOPS_FP32_TRANS, SQ_INSTS_VALU_FLOPS_FP64, SQ_INSTS_VALU and
BUSY_DIR = SQ_INSTS_VALU_FMA_F32, SQ_INSTS_VALU_ADD_F32, SQ_INSTS_VALU_MUL_F32, SQ_INSTS_VALU_TRANS_F32,
SQ_ACTIVE_INST_VALU, SQ_WAVE_CYCLES, SQ_BUSY_CYCLES + GRBM_GUI_ACTIVE.  flops_per_launch = the FLOPS
counters (counted per active lane by the SQ); the instruction-mix estimate 64 x (2 FMA + ADD + MUL +
TRANS) is kept beside it (it counts inactive lanes too).  valu_busy = SQ_ACTIVE_INST_VALU (quad-cycles
summed over SIMDs) / (CUs x GRBM_GUI_ACTIVE per XCD), rocprof's VALUBusy: the fraction of SIMD-cycles a
VALU instruction was executing.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  MI355X_MICROARCH.md (HBM section): on gfx950
FETCH_SIZE reports half the bytes of wide coalesced reads, so it is doubled; WRITE_SIZE is
taken as is.  Keys starting with ``race_`` select the race step kernels (race_step_q4 / race_step_kernel), the others
hover_step_kernel.  The first 8 dispatches (cold caches, first-touch) are skipped; the median of
the rest is reported.
"""
import csv
import glob
import json
import statistics
import sys


def counter(d, name, kernel):
    vals = []
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r.get("Kernel_Name", "") and r["Counter_Name"] == name:
                vals.append((int(r.get("Dispatch_Id", len(vals))), float(r["Counter_Value"])))
    vals = [v for _, v in sorted(vals)]
    steady = vals[8:] if len(vals) > 16 else vals
    if not steady:
        raise SystemExit(f"no {name} rows for {kernel} under {d}")
    return statistics.median(steady), len(vals)


CUS = 256


def valu(out_path, rest):
    try:
        rec = json.load(open(out_path))
    except (OSError, ValueError):
        rec = {}
    for i in range(0, len(rest), 3):
        key, fdir, bdir = rest[i:i + 3]
        kernel = "race_step" if key.startswith("race_") else "hover_step_kernel"   # race_step_q4 / race_step_kernel
        c = {n: counter(fdir, n, kernel)[0] for n in ("SQ_INSTS_VALU_FLOPS_FP32", "SQ_INSTS_VALU_FLOPS_FP32_TRANS",
                                                      "SQ_INSTS_VALU_FLOPS_FP64", "SQ_INSTS_VALU")}
        c.update({n: counter(bdir, n, kernel)[0] for n in (
            "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_TRANS_F32",
            "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE")})
        # the FLOPS counters count per wave-instruction (their sum equals 2 FMA + ADD + MUL + TRANS): x 64 lanes
        flops = 64 * (c["SQ_INSTS_VALU_FLOPS_FP32"] + c["SQ_INSTS_VALU_FLOPS_FP32_TRANS"] + c["SQ_INSTS_VALU_FLOPS_FP64"])
        mix = 64 * (2 * c["SQ_INSTS_VALU_FMA_F32"] + c["SQ_INSTS_VALU_ADD_F32"] + c["SQ_INSTS_VALU_MUL_F32"]
                    + c["SQ_INSTS_VALU_TRANS_F32"])
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs in the per-dispatch record: per-XCD cycles = / 8
        busy = c["SQ_ACTIVE_INST_VALU"] / (CUS * c["GRBM_GUI_ACTIVE"] / 8) if c["GRBM_GUI_ACTIVE"] else None
        keep = {k: v for k, v in rec.get(key, {}).items() if k.startswith("algorithmic_")}   # the flop model
        rec[key] = {**keep, "kernel": kernel, "flops_per_launch": flops, "flops_instruction_mix_estimate": mix,
                    "valu_insts_per_launch": c["SQ_INSTS_VALU"], "valu_busy": busy, "counters": c,
                    "method": "rocprofv3 --pmc, two passes (FLOPS counters; instruction mix + busy); median over "
                              "dispatches after the first 8"}
        print(key, json.dumps(rec[key]))
    json.dump(rec, open(out_path, "w"), indent=1)


def calib(out_path, fdir, wdir, bytes_per_launch):
    """tools/fetch_calib: FETCH_SIZE / WRITE_SIZE per launch over the known streamed bytes, per
    access width (4 / 8 / 16 B per lane)"""
    rec = {"bytes_per_launch": bytes_per_launch,
           "method": "tools/fetch_calib.hip: one coalesced streaming pass over 256 MiB per launch, "
                     "median over launches after the first 8; ratio = counter bytes / streamed bytes"}
    for w in (4, 8, 16):
        f, _ = counter(fdir, "FETCH_SIZE", f"calib_read{w}")
        wr, _ = counter(wdir, "WRITE_SIZE", f"calib_write{w}")
        rec[f"read{w}"] = {"fetch_size_kib": f, "ratio": f * 1024 / bytes_per_launch}
        rec[f"write{w}"] = {"write_size_kib": wr, "ratio": wr * 1024 / bytes_per_launch}
        print(w, rec[f"read{w}"], rec[f"write{w}"])
    json.dump(rec, open(out_path, "w"), indent=1)


def alg(out_path, rest):
    """--alg OUT.json KEY FLOPS_DIR DRONES_PER_LAUNCH [...]: the flop model of a race workload from a
    FLOPS pass of the one-lane fp32 kernel (ADRP_RACE_QUAD=0: one lane per drone, no redundant
    lanes): algorithmic_flops_per_drone_step = its FLOPS counters x 64 / drones per launch, kept on
    KEY (and on its fp64 twin) beside the four-lane kernel's executed counters"""
    try:
        rec = json.load(open(out_path))
    except (OSError, ValueError):
        rec = {}
    for i in range(0, len(rest), 3):
        key, fdir, drones = rest[i], rest[i + 1], int(rest[i + 2])
        c = {n: counter(fdir, n, "race_step_kernel")[0] for n in (
            "SQ_INSTS_VALU_FLOPS_FP32", "SQ_INSTS_VALU_FLOPS_FP32_TRANS", "SQ_INSTS_VALU_FLOPS_FP64")}
        per = 64 * sum(c.values()) / drones
        for k in (key, key.replace("_fp32_", "_fp64_")):
            rec.setdefault(k, {})
            rec[k]["algorithmic_flops_per_drone_step"] = per
            rec[k]["algorithmic_source"] = ("SQ_INSTS_VALU_FLOPS_* of the one-lane race_step_kernel (one lane per "
                                            "drone, no redundant lanes; ADRP_RACE_QUAD=0) on the same workload, fp32, "
                                            "tools/gpu.sh pmc; the same algorithm in either precision")
        print(key, per)
    json.dump(rec, open(out_path, "w"), indent=1)


def main():
    if sys.argv[1] == "--alg":
        return alg(sys.argv[2], sys.argv[3:])
    if sys.argv[1] == "--valu":
        return valu(sys.argv[2], sys.argv[3:])
    if sys.argv[1] == "--calib":
        return calib(sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5]))
    out_path, rest = sys.argv[1], sys.argv[2:]
    try:
        rec = json.load(open(out_path))
    except (OSError, ValueError):
        rec = {}
    for i in range(0, len(rest), 3):
        key, fdir, wdir = rest[i:i + 3]
        kernel = "race_step" if key.startswith("race_") else "hover_step_kernel"   # race_step_q4 / race_step_kernel
        fetch_kib, nf = counter(fdir, "FETCH_SIZE", kernel)
        write_kib, nw = counter(wdir, "WRITE_SIZE", kernel)
        rd = fetch_kib * 1024 * 2
        wr = write_kib * 1024
        rec[key] = {"kernel": kernel, "hbm_bytes_per_launch": rd + wr, "read_bytes": rd, "write_bytes": wr,
                    "fetch_size_kib_median": fetch_kib, "write_size_kib_median": write_kib,
                    "dispatches": [nf, nw],
                    "method": "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes; FETCH_SIZE x2 "
                              "(gfx950 correction), median over dispatches after the first 8"}
        print(key, json.dumps(rec[key]))
    json.dump(rec, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
