"""Per (kernel, grid) timing from a rocprofv3 rocpd database: where a solve's time goes by
launch shape (levels of the multigrid, cyclic-reduction levels, ...).

usage: python tools/kernel_grid.py <results.db> [steps] [top]
"""
import collections
import re
import sqlite3
import sys


def short(name):
    name = re.sub(r"^void ", "", name).replace("(anonymous namespace)::", "").replace("iemic::", "")
    return re.split(r"\(", name)[0]


def main():
    path = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    c = sqlite3.connect(path)
    d = collections.defaultdict(list)
    for name, gx, gy, dur in c.execute("select name, grid_x, grid_y, duration from kernels"):
        d[(short(name), gx, gy)].append(dur)
    rows = sorted(d.items(), key=lambda kv: -sum(kv[1]))
    print("| kernel | grid | calls | avg (us) | ms/step |\n|---|---|---|---|---|")
    for (n, gx, gy), v in rows[:top]:
        print(f"| {n} | {gx}x{gy} | {len(v)} | {sum(v) / len(v) / 1e3:.2f} | {sum(v) / steps / 1e6:.2f} |")
    ks = sorted(c.execute("select start, end from kernels"))
    print(f"\nbusy {sum(e - s for s, e in ks) / steps / 1e6:.1f} ms/step, span {(ks[-1][1] - ks[0][0]) / steps / 1e6:.1f} ms/step")


if __name__ == "__main__":
    main()
