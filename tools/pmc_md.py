"""Markdown table of a PMC kernel table (bench_data/pmc_<tag>.json, tools/pmc_table.py).

usage: python tools/pmc_md.py bench_data/pmc_r06.json "<call>" "<note on the sources>" > profiles/r06_pmc_kernels.md
"""
import json
import sys


def main():
    d = json.load(open(sys.argv[1]))
    call = sys.argv[2] if len(sys.argv) > 2 else "?"
    note = sys.argv[3] if len(sys.argv) > 3 else ""
    ks = d["kernels"]
    ms_tot, gb = d["step_kernel_ms"], d["step_hbm_bytes"] / 1e9
    print(f"# Round {d['tag'][1:]}: HBM bytes per kernel of one benchmark Newton step ({d['config']}, FGMRES, compressed basis)\n")
    print(f"Source: `{sys.argv[1]}` (tools/pmc_table.py over scripts/gpu_pmc.sh, call [{call}]: FETCH_SIZE and "
          f"WRITE_SIZE passes, calibrated on 1 GiB streams: read factor {d['calibration']['read8_factor']}, write factor "
          f"{d['calibration']['write8_factor']}; launch times from a kernel-trace pass of the same command).  "
          f"src_digest {d['src_digest'][:16]}{': ' + note if note else ''}.\n")
    print(f"Step (context set-up plus one Newton step): {gb:.1f} GB of counter bytes, {ms_tot:.1f} ms of kernel time "
          f"({gb / ms_tot:.2f} TB/s); dominant kernel {d['dominant']}.\n")
    print("| kernel | launches | MB / launch | avg µs | ms / step | TB/s | frac of 8 TB/s |")
    print("|---|---|---|---|---|---|---|")
    rows = sorted((k for k in ks if k.get("avg_us")), key=lambda k: -k["launches"] * k["avg_us"])
    for k in rows[:26]:
        ms = k["launches"] * k["avg_us"] / 1e3
        tbs = k["hbm_bytes_per_launch"] / (k["avg_us"] * 1e-6) / 1e12
        print(f"| {k['kernel']} | {k['launches']} | {k['hbm_bytes_per_launch'] / 1e6:.1f} | {k['avg_us']:.2f} | "
              f"{ms:.2f} | {tbs:.2f} | {tbs / 8:.2f} |")


if __name__ == "__main__":
    main()
