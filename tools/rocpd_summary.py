"""Summarise a rocprofv3 rocpd database (kernel trace) as a per-kernel stats table.

usage: python tools/rocpd_summary.py <results.db> [> profiles/<name>.md]
"""
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage "
                          "from top_kernels"))
    print(f"# kernel stats: {path.split('/')[-1]}\n")
    # the top_kernels view reports durations in microseconds
    print("| kernel | calls | total (ms) | avg (us) | % |")
    print("|---|---|---|---|---|")
    for name, calls, tot, avg, pct in rows:
        short = name.replace("(anonymous namespace)::", "").replace("iemic::", "").split("(")[0]
        print(f"| {short} | {calls} | {tot / 1e3:.3f} | {avg:.2f} | {pct:.2f} |")


if __name__ == "__main__":
    main(sys.argv[1])
