"""Turn the rocprofv3 PMC passes of tools/gpu_pmc.sh into HBM bytes per k_spmv launch.

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE under-counts wide streaming
reads (MI355X_MICROARCH.md, HBM section), so the counts are converted with factors
measured in the same call on streams of a known byte count (scripts/pmc_calib.hip: 8-B and
16-B lanes, 1 GiB, beyond the Infinity Cache).  The SpMV reads its values with 8-B lanes,
so the 8-B read factor applies to its FETCH_SIZE.

usage: python tools/pmc_report.py gpurun_out/pmc [config] > profiles/<tag>_spmv_pmc.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

CALIB_BYTES = 1 << 30


def load(d):
    """kernel name -> list of counter values (one per dispatch)"""
    out = defaultdict(list)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                out[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return out


def mean_of(d, key):
    vals = [v for k, vs in d.items() if key in k for v in vs]
    if not vals:
        raise SystemExit(f"kernel {key} not found")
    return sum(vals) / len(vals), len(vals)


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    cfgname = sys.argv[2] if len(sys.argv) > 2 else "global2"
    cf, cw = load(os.path.join(root, "calib_FETCH_SIZE")), load(os.path.join(root, "calib_WRITE_SIZE"))
    sf, sw = load(os.path.join(root, "spmv_FETCH_SIZE")), load(os.path.join(root, "spmv_WRITE_SIZE"))
    r8, _ = mean_of(cf, "k_read8")
    r16, _ = mean_of(cf, "k_read16")
    w8, _ = mean_of(cw, "k_write8")
    f8 = CALIB_BYTES / (r8 * 1024)
    f16 = CALIB_BYTES / (r16 * 1024)
    fw = CALIB_BYTES / (w8 * 1024)
    fs, nf = mean_of(sf, "k_spmv")
    ws, nw = mean_of(sw, "k_spmv")
    rd = fs * 1024 * f8
    wr = ws * 1024 * fw
    trace = {}
    for f in glob.glob(os.path.join(root, "spmv_trace", "**", "*kernel_stats.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if "k_spmv" in row["Name"]:
                    trace = {"calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"])}
    print(json.dumps({
        "config": cfgname, "kernel": ", ".join(sorted({k.split("(")[0] for k in sf if "k_spmv" in k})), "condition": "Infinity Cache flushed before each launch",
        "launches": nf, "fetch_kib": fs, "write_kib": ws,
        "calibration": {"read8_factor": round(f8, 4), "read16_factor": round(f16, 4),
                        "write8_factor": round(fw, 4), "bytes": CALIB_BYTES},
        "read_bytes_per_launch": int(rd), "write_bytes_per_launch": int(wr),
        "hbm_bytes_per_launch": int(rd + wr), "trace": trace}, indent=1))


if __name__ == "__main__":
    main()
