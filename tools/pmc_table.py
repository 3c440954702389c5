"""Per-kernel table of one benchmark Newton step for bench.py's roofline fields: HBM bytes per
launch from the rocprofv3 PMC passes of scripts/gpu_pmc.sh (FETCH_SIZE / WRITE_SIZE in KiB,
converted with the factors measured in the same call on streams of known size, see
tools/pmc_report.py) and the average launch time from a kernel-trace pass of the same
command.  Keyed by the digest of the device sources (iemic._lib.src_digest), so bench.py
uses it only for the kernels it was measured on.

usage: python tools/pmc_table.py gpurun_out/pmc <tag> > bench_data/pmc_<tag>.json
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "i-emic_amd"), os.path.dirname(os.path.abspath(__file__))]

from pmc_report import CALIB_BYTES, load, mean_of  # noqa: E402


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("iemic::", "")
    if n.startswith("void "):
        n = n[5:]
    depth, out = 0, []
    for ch in n:                       # cut the argument list, keep template arguments
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out).strip()


def trace_stats(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Name"])
                calls, avg = int(row["Calls"]), float(row["AverageNs"])
                if k in out:                      # the same name from several files
                    c0, a0 = out[k]
                    out[k] = (c0 + calls, (a0 * c0 + avg * calls) / (c0 + calls))
                else:
                    out[k] = (calls, avg)
    return out


def main():
    from iemic._lib import src_digest
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    tag = sys.argv[2] if len(sys.argv) > 2 else "r04"
    cf, cw = load(os.path.join(root, "calib_FETCH_SIZE")), load(os.path.join(root, "calib_WRITE_SIZE"))
    f8 = CALIB_BYTES / (mean_of(cf, "k_read8")[0] * 1024)
    fw = CALIB_BYTES / (mean_of(cw, "k_write8")[0] * 1024)
    bf, bw = load(os.path.join(root, "bench_FETCH_SIZE")), load(os.path.join(root, "bench_WRITE_SIZE"))
    tr = trace_stats(os.path.join(root, "bench_trace"))
    rows = {}
    for k, vs in bf.items():
        name = short(k)
        wv = bw.get(k, [0.0])
        r = rows.setdefault(name, {"kernel": name, "launches": 0, "read": 0.0, "write": 0.0})
        r["launches"] += len(vs)
        r["read"] += sum(vs) * 1024 * f8
        r["write"] += sum(wv) / len(wv) * len(vs) * 1024 * fw
    out = []
    for r in rows.values():
        n = r["launches"]
        calls, avg_ns = tr.get(r["kernel"], (0, 0.0))
        b = (r["read"] + r["write"]) / n
        out.append({"kernel": r["kernel"], "launches": n, "hbm_bytes_per_launch": int(b),
                    "hbm_bytes_total": int(r["read"] + r["write"]), "trace_calls": calls,
                    "avg_us": round(avg_ns / 1e3, 3), "total_ms": round(calls * avg_ns / 1e6, 3),
                    "gbs": round(b / avg_ns, 1) if avg_ns else None})
    out.sort(key=lambda r: -r["total_ms"])
    dom = out[0]["kernel"] if out else None
    print(json.dumps({
        "tag": tag, "src_digest": src_digest(), "config": "global2",
        "condition": ("bench.py --steps 1 --warmup 0 --no-cpu --newton-seq 0 --no-stream: context set-up plus one "
                      "benchmark Newton step (global2 branch state), in-solve, warm caches; PMC passes "
                      "FETCH_SIZE and WRITE_SIZE in separate runs, avg_us from a kernel-trace run of the "
                      "same command"),
        "calibration": {"read8_factor": round(f8, 4), "write8_factor": round(fw, 4), "bytes": CALIB_BYTES},
        "step_hbm_bytes": int(sum(r["hbm_bytes_total"] for r in out)),
        "step_kernel_ms": round(sum(r["total_ms"] for r in out), 3),
        "dominant": dom, "kernels": out}, indent=1))


if __name__ == "__main__":
    main()
