"""Per-stream kernel time of a rocpd kernel trace of an in-process rank group
(scripts/band_iters.py N:npx under rocprofv3 --kernel-trace): every rank drives its own
library stream, so a stream's kernel durations are that rank's kernels (measured while the
other ranks share the GPU: an upper bound of a rank on its own GPU).  Prints, per stream,
the launches and the kernel milliseconds, and for the busiest one the top kernels.

usage: python tools/rank_kernels.py <results.db> [fgmres steps]"""
import collections
import sqlite3
import sys


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("iemic::", "").replace("void ", "").split("(")[0]


def main(path, steps=0):
    c = sqlite3.connect(path)
    per = collections.defaultdict(list)
    for name, sid, dur in c.execute("select name, stream_id, duration from kernels"):
        per[sid].append((short(name), dur / 1e3))
    rows = sorted(per.items(), key=lambda kv: -sum(d for _, d in kv[1]))
    print("| stream | launches | kernel ms |" + (" us / FGMRES step |" if steps else ""))
    print("|---|---|---|" + ("---|" if steps else ""))
    for sid, ks in rows:
        tot = sum(d for _, d in ks)
        print(f"| {sid} | {len(ks)} | {tot / 1e3:.2f} |" + (f" {tot / steps:.1f} |" if steps else ""))
    sid, ks = rows[0]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for n, d in ks:
        agg[n][0] += 1
        agg[n][1] += d
    print(f"\nbusiest stream {sid}:\n\n| kernel | calls | avg us | ms |\n|---|---|---|---|")
    for n, (k, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:20]:
        print(f"| {n} | {k} | {t / k:.2f} | {t / 1e3:.2f} |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 0)
