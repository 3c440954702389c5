"""Summarise a rocprofv3 rocpd database (kernel trace) as a per-kernel stats table.

usage: python tools/rocpd_summary.py <results.db> [> profiles/<name>.md]
"""
import collections
import sqlite3
import sys


def rows_of(c):
    try:
        # the top_kernels view reports durations in microseconds
        return [(n, k, t, a) for n, k, t, a, _ in
                c.execute("select name, total_calls, total_duration, average, percentage from top_kernels")]
    except sqlite3.OperationalError:
        # databases without the summary views: aggregate the kernel table (ns)
        d = collections.defaultdict(list)
        for name, dur in c.execute("select name, duration from kernels"):
            d[name].append(dur / 1e3)
        return sorted(((n, len(v), sum(v), sum(v) / len(v)) for n, v in d.items()), key=lambda r: -r[2])


def main(path):
    c = sqlite3.connect(path)
    rows = rows_of(c)
    total = sum(r[2] for r in rows) or 1.0
    print(f"# kernel stats: {path.split('/')[-1]}\n")
    print("| kernel | calls | total (ms) | avg (us) | % |")
    print("|---|---|---|---|---|")
    for name, calls, tot, avg in rows:
        short = name.replace("(anonymous namespace)::", "").replace("iemic::", "").split("(")[0]
        print(f"| {short} | {calls} | {tot / 1e3:.3f} | {avg:.2f} | {100 * tot / total:.2f} |")


if __name__ == "__main__":
    main(sys.argv[1])
