"""Multi-GPU projection of the bench's Newton step for latitude bands, from measured inputs:
the one-GPU kernel trace of the step (rocprofv3 --kernel-trace rocpd database: every launch's
duration and grid), the FGMRES steps and exchange batches / all-reduces per step of the N-band
runs (scripts/band_iters.py, in-process ranks), and the launch floor (the shortest dependent
launch of the trace).  The model, per FGMRES step at N bands:

    t(N) = sum over the step's launches of max(floor, t1 * f) + batches * t_b + allreduces * t_ar

with f = 1 for the replicated launches (the Schur cyclic reduction, k_cr_*, which every rank
runs on the whole 2-D problem, and the coarsest multigrid GEMV) and f = 1/N for the others
(their grids cover the rank's own cells); t_b and t_ar are the RCCL latencies of one exchange
batch and one small all-reduce over xGMI, which one-GPU boxes cannot measure: the table is
printed for a range of them.  The Newton step is t(N) x steps(N) plus the step's set-up
(F, J, preconditioner) kept at its one-GPU value (an upper bound: the Schur set-up is
replicated, the rest shrinks).

usage: python tools/project.py <results.db> <fgmres steps in the trace> <newton ms untraced>
           <setup ms> N:steps:batches:allreduces ...
"""
import collections
import sqlite3
import sys

REPLICATED = ("k_cr_pk", "k_cr_tail", "k_cr_final", "k_gemv_w", "k_gemv")


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("iemic::", "").replace("void ", "")
    return n.split("(")[0]


def main():
    db, steps, newton_ms, setup_ms = sys.argv[1], int(sys.argv[2]), float(sys.argv[3]), float(sys.argv[4])
    runs = [tuple(float(x) for x in a.split(":")) for a in sys.argv[5:]]
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, duration from kernels"))
    per = collections.defaultdict(list)
    for name, dur in rows:
        per[short(name)].append(dur / 1e3)
    # the launches of the FGMRES steps: kernels called at least once per step
    step = {k: v for k, v in per.items() if len(v) >= steps}
    floor = min(sum(v) / len(v) for v in step.values())
    t1 = sum(sum(v) for v in step.values()) / steps
    rep = sum(sum(v) for k, v in step.items() if k.startswith(REPLICATED)) / steps
    n_launch = sum(len(v) for v in step.values()) / steps
    print(f"one GPU: {n_launch:.1f} launches and {t1:.1f} us of kernels per FGMRES step (traced), "
          f"{rep:.1f} us of them replicated; launch floor {floor:.2f} us")
    print()
    lat = [(5, 8), (8, 12), (15, 25), (30, 50)]
    hdr = " | ".join(f"t_b {b} / t_ar {a} us" for b, a in lat)
    print(f"| N | FGMRES steps | kernels us / step | batches / step | all-reduces / step | {hdr} |")
    print("|---|---|---|---|---|" + "---|" * len(lat))
    # traced -> untraced, on the one-GPU run's FGMRES steps (the trace may hold several
    # Newton steps: `steps` counts all of its FGMRES steps)
    it1 = next((it for N, it, _, _ in runs if N == 1), steps)
    scale = newton_ms / (t1 * it1 / 1e3 + setup_ms)
    for N, it, nb, nar in runs:
        kern = 0.0
        for k, v in step.items():
            f = 1.0 if (k.startswith(REPLICATED) or N == 1) else 1.0 / N
            kern += sum(max(floor, d * f) for d in v) / steps
        cells = []
        for b, a in lat:
            ms = (kern * scale + nb * b + nar * a) * it / 1e3 + setup_ms
            cells.append(f"{ms:.1f} ms ({newton_ms / ms:.2f}x)")
        print(f"| {int(N)} | {int(it)} | {kern * scale:.0f} | {nb} | {nar} | " + " | ".join(cells) + " |")


if __name__ == "__main__":
    main()
