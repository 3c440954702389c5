"""Per-kernel HBM bytes of one benchmark Newton step from the rocprofv3 PMC passes of
scripts/gpu_pmc.sh (FETCH_SIZE, WRITE_SIZE in KiB, converted with the factors measured
in the same call on streams of known size, see tools/pmc_report.py).

usage: python tools/pmc_kernels.py gpurun_out/pmc [top] > profiles/<tag>_kernels_pmc.json
"""
import json
import os
import sys

from pmc_report import CALIB_BYTES, load, mean_of


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("iemic::", "").split("(")[0]


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    cf, cw = load(os.path.join(root, "calib_FETCH_SIZE")), load(os.path.join(root, "calib_WRITE_SIZE"))
    f8 = CALIB_BYTES / (mean_of(cf, "k_read8")[0] * 1024)
    fw = CALIB_BYTES / (mean_of(cw, "k_write8")[0] * 1024)
    bf, bw = load(os.path.join(root, "bench_FETCH_SIZE")), load(os.path.join(root, "bench_WRITE_SIZE"))
    rows = []
    for k, vs in bf.items():
        wv = bw.get(k, [0.0])
        rd = sum(vs) / len(vs) * 1024 * f8
        wr = sum(wv) / len(wv) * 1024 * fw
        rows.append({"kernel": short(k), "launches": len(vs), "read_bytes_per_launch": int(rd),
                     "write_bytes_per_launch": int(wr), "hbm_bytes_per_launch": int(rd + wr),
                     "hbm_bytes_total": int((rd + wr) * len(vs))})
    rows.sort(key=lambda r: -r["hbm_bytes_total"])
    print(json.dumps({"condition": "one benchmark Newton step (global2 branch state), in-solve, warm caches",
                      "calibration": {"read8_factor": round(f8, 4), "write8_factor": round(fw, 4)},
                      "kernels": rows[:top]}, indent=1))


if __name__ == "__main__":
    main()
