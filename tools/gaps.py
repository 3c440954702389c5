"""Idle time on the GPU between consecutive kernels of a rocpd kernel trace, charged to the
kernel that follows the gap (launch-rate and host-synchronisation stalls).

usage: python tools/gaps.py <results.db> [top]
"""
import collections
import sqlite3
import sys


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("iemic::", "").replace("void ", "").split("(")[0]


def main(path, top=25):
    c = sqlite3.connect(path)
    rows = list(c.execute("select name, start, end from kernels order by start"))
    gap = collections.defaultdict(list)
    prev_end = None
    prev_name = None
    for name, s, e in rows:
        if prev_end is not None:
            g = (s - prev_end) / 1e3
            if 0 < g < 5000:     # ignore gaps between separate phases
                gap[(short(prev_name), short(name))].append(g)
        prev_end = max(e, prev_end or e)
        prev_name = name
    tot = sum(sum(v) for v in gap.values())
    print(f"total gap {tot / 1e3:.1f} ms over {sum(len(v) for v in gap.values())} launches")
    print("| after | before | count | total (ms) | avg (us) |")
    print("|---|---|---|---|---|")
    for (a, b), v in sorted(gap.items(), key=lambda kv: -sum(kv[1]))[:top]:
        print(f"| {a} | {b} | {len(v)} | {sum(v) / 1e3:.2f} | {sum(v) / len(v):.1f} |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)
