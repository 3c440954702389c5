"""Per-dispatch view of a rocpd kernel trace: duration by (kernel, grid size), and the
launch sequence of one period (e.g. one preconditioner apply).

usage: python tools/kernel_seq.py <results.db> [kernel-substring ...]
"""
import collections
import sqlite3
import sys


def main(path, pats):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    rows = list(c.execute("select * from kernels order by start"))
    ix = {n: i for i, n in enumerate(cols)}
    stats = collections.defaultdict(list)
    for r in rows:
        name = r[ix["name"]].replace("(anonymous namespace)::", "").replace("iemic::", "").split("(")[0]
        if pats and not any(p in name for p in pats):
            continue
        grid = r[ix["grid_size_x"]] if "grid_size_x" in ix else r[ix["grid_x"]]
        stats[(name, grid)].append((r[ix["end"]] - r[ix["start"]]) / 1e3)
    print("| kernel | grid | calls | avg (us) | min (us) |")
    print("|---|---|---|---|---|")
    for (name, grid), d in sorted(stats.items(), key=lambda kv: -sum(kv[1])):
        print(f"| {name} | {grid} | {len(d)} | {sum(d) / len(d):.2f} | {min(d):.2f} |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
