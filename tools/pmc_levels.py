"""Per-(kernel, grid) HBM bytes of one benchmark Newton step from the PMC passes of
scripts/gpu_pmc.sh: the multigrid levels and cyclic-reduction steps are the same kernel on
grids of different sizes.  Counter values are scaled with the calibration of
tools/pmc_report.py (FETCH_SIZE / WRITE_SIZE in KiB).

usage: python tools/pmc_levels.py gpurun_out/pmc [kernel-substring ...] > profiles/<tag>_levels_pmc.md
"""
import collections
import csv
import glob
import os
import sys

from pmc_report import CALIB_BYTES, load, mean_of


def per_grid(root, ctr):
    f = glob.glob(os.path.join(root, f"bench_{ctr}", "*counter_collection.csv"))[0]
    d = collections.defaultdict(list)
    with open(f) as fh:
        for row in csv.DictReader(fh):
            if row["Counter_Name"] != ctr:
                continue
            name = row["Kernel_Name"].replace("(anonymous namespace)::", "").replace("iemic::", "").split("(")[0]
            d[(name, int(row["Grid_Size"]))].append(float(row["Counter_Value"]))
    return d


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    keys = sys.argv[2:] or ["k_mg_zl", "k_mg_rc", "k_mg_entry", "k_cr_multi", "k_cr_tail"]
    cf, cw = load(os.path.join(root, "calib_FETCH_SIZE")), load(os.path.join(root, "calib_WRITE_SIZE"))
    f8 = CALIB_BYTES / (mean_of(cf, "k_read8")[0] * 1024)
    fw = CALIB_BYTES / (mean_of(cw, "k_write8")[0] * 1024)
    rd, wr = per_grid(root, "FETCH_SIZE"), per_grid(root, "WRITE_SIZE")
    print("| kernel | grid (threads) | launches | read MB / launch | write MB / launch |")
    print("|---|---|---|---|---|")
    for (name, grid), vs in sorted(rd.items(), key=lambda kv: (kv[0][0], -kv[0][1])):
        if not any(k in name for k in keys):
            continue
        w = wr.get((name, grid), [0.0])
        print(f"| {name} | {grid} | {len(vs)} | {sum(vs) / len(vs) * 1024 * f8 / 1e6:.2f} | "
              f"{sum(w) / len(w) * 1024 * fw / 1e6:.2f} |")


if __name__ == "__main__":
    main()
