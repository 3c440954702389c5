"""Newton-step benchmark of the THCM ocean hot path (BASELINE.json metric).

One step = one full Newton step of the 2-degree global ocean (192x76x16, 1,400,832
unknowns) on the GPU: residual F, Jacobian assembly, preconditioner
set-up, FGMRES solve of J dx = -F to the relative tolerance 1e-8 (Belos semantics,
Ocean.C:1060-1137), x += dx and the new residual (transient/Newton.H:92-99).  Every step
restarts from the same state, resident in HBM (the reset is a device-to-device copy inside
the timed region): by default the near-solution branch state bench_data/<config>_cf05.npz
(the 2-degree model continued from rest to Combined Forcing 0.5, scripts/branch_state.py),
with --state synthetic SURVEY §8d's splitmix64 state (seed 20261015; a Newton step from it
diverges).  The state is named in config["state"].

Multi-GPU (``--gpus N``): one process per GPU.  Run as ``python bench.py --gpus N`` the
script starts its N ranks itself (a ``torch.distributed.run`` child process, before anything
touches the GPU); under an external ``torch.distributed.run`` it is one rank and checks that
WORLD_SIZE equals N.  The same 2-degree problem is split into N latitude bands (``--npx 1``,
the default; ``--npx 0`` the reference's Decomp2D rule, TRIOS_Domain.C:88-109, 8 GPUs: 4 x 2,
48 x 38 columns each -- x cuts through the zonal flow cost FGMRES steps): halo
exchanges and Krylov reductions over RCCL (``--transport rccl``), or through the library's
host transport over gloo (``--transport host``: several ranks may share one GPU, to check
the decomposition on a one-GPU box); the preconditioner's Schur problem and coarsest T/S level
are global, the rest couples across subdomain edges through halos -- strong
scaling; the step time is the max over ranks.  The line reports the ranks the communicator
itself saw (``ranks_seen``: ncclCommCount under RCCL) and the communication per FGMRES step.

Prints ONE JSON line (rank 0) with the metric, the SpMV roofline of the same run (HIP
events on the library's stream) and the CPU baseline (the oracle port, rank 0, N=1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "i-emic_amd"))

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
PMC_TAG = "r06"         # bench_data/pmc_<tag>.json: per-kernel PMC bytes and trace times of a step


def pmc_table(config: str):
    """The measured per-kernel table of one benchmark step (tools/pmc_table.py), if it was
    measured on the device sources this tree builds (its src_digest) and this config."""
    path = os.path.join(ROOT, "bench_data", f"pmc_{PMC_TAG}.json")
    if not os.path.exists(path):
        return None, f"no table {os.path.relpath(path, ROOT)}"
    with open(path) as f:
        t = json.load(f)
    from iemic._lib import src_digest
    if t.get("src_digest") != src_digest():
        return None, f"{os.path.relpath(path, ROOT)} was measured on other kernel sources"
    if t.get("config") != config:
        return None, f"{os.path.relpath(path, ROOT)} holds config {t.get('config')}"
    return t, None


def spmv_bytes(nnz: int, n: int) -> int:
    """CSR-equivalent algorithmic bytes of one SpMV."""
    return 12 * nnz + 20 * n + 4


def stencil_ell_bytes(ncell: int, nslot: int, n: int) -> int:
    """Bytes the implicit-index stencil-ELL SpMV must move: values + x + y."""
    return 8 * ncell * nslot + 16 * n


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1,
                   help="ranks, one per GPU (started here unless WORLD_SIZE is set)")
    p.add_argument("--transport", default="rccl", choices=["rccl", "host"],
                   help="rccl: RCCL over xGMI, one GPU per rank; host: the library's host transport "
                        "over gloo (ranks may share a GPU)")
    p.add_argument("--npx", type=int, default=1,
                   help="x parts of the process grid (1: latitude bands, the default: the fewest exchange "
                        "batches per FGMRES step, DESIGN.md §7; 0: the reference's Decomp2D rule)")
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--config", default="global2")
    p.add_argument("--mixing", type=int, default=1,
                   help="THCM 'Mixing' (vmix): 1 as in run/ocean/global/ocean_params.xml")
    p.add_argument("--prec", type=int, default=2, help="0 none, 1 block Jacobi, 2 block GS")
    p.add_argument("--state", default="branch", choices=["branch", "synthetic"],
                   help="branch: the near-solution state bench_data/<config>_cf05.npz (the config "
                        "continued from rest to Combined Forcing 0.5, scripts/branch_state.py); "
                        "synthetic: the splitmix64 state of SURVEY.md §8d")
    p.add_argument("--amp-ts", type=float, default=1e-3,
                   help="T/S amplitude of the synthetic state (DESIGN.md: benchmark state)")
    p.add_argument("--newton-seq", type=int, default=3,
                   help="untimed Newton iterations from the benchmark state, reported as the "
                        "residual sequence")
    p.add_argument("--tol", type=float, default=1e-8)
    p.add_argument("--krylov", type=int, default=90)
    p.add_argument("--restarts", type=int, default=20)
    p.add_argument("--ts-sweeps", type=int, default=12)
    p.add_argument("--orth", default="DCGS2", choices=["DCGS2", "DGKS"])
    p.add_argument("--solver", default="FGMRES", choices=["FGMRES", "IDR"],
                   help="Krylov method (IDR: IDRSolver.H's IDR(s), --idr-s)")
    p.add_argument("--idr-s", type=int, default=4)
    p.add_argument("--dyn-iters", type=int, default=None,
                   help="defect-correction passes on the dynamics block of the block GS (default 4; "
                        "8 at 1 degree, where the passes without the Schur solve pay: DESIGN.md section 4)")
    p.add_argument("--dyn-omega", type=float, default=0.95, help="step of the correction passes")
    p.add_argument("--dyn-mr", action="store_true", help="minimal-residual step per pass")
    p.add_argument("--ts-mg", type=int, default=1,
                   help="T/S aggregation-multigrid V-cycles (0: --ts-sweeps plain sweeps)")
    p.add_argument("--mg-sweeps", type=int, default=1, help="sweeps per multigrid level")
    p.add_argument("--ts-at", type=int, default=0,
                   help="form the T/S right-hand side after this many dynamics passes (0: the last); "
                        "earlier lets the T/S multigrid run on a second stream beside the rest")
    p.add_argument("--schur-passes", type=int, default=2,
                   help="this many dynamics passes solve the Schur system: the first k - 1 and the last "
                        "(the others take pbar = 0; 0: every pass)")
    p.add_argument("--spmv-reps", type=int, default=0,
                   help="extra back-to-back (hot Infinity Cache) SpMV launches, reported apart")
    p.add_argument("--no-stream", action="store_true",
                   help="skip the STREAM-copy probe (scripts/gpu_pmc.sh: its 1 GiB copies are no part of the step)")
    p.add_argument("--cold-reps", type=int, default=0,
                   help="extra SpMV launches after an Infinity Cache flush, reported apart")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--save-x1", default=None,
                   help="write the state after the last timed Newton step (gathered from all ranks) "
                        "and the starting state to this .npz (rank 0), for parity checks")
    p.add_argument("--cpu-samples", type=int, default=10,
                   help="timed CPU Newton steps (the line reports their median and spread)")
    p.add_argument("--cpu-warmup", type=int, default=2,
                   help="untimed CPU Newton steps before the timed ones (SURVEY §8d: 2)")
    p.add_argument("--mode", default="newton", choices=["newton", "continuation"],
                   help="continuation: config C5, one pseudo-arclength continuation step of the "
                        "1-degree ocean (run/ocean settings) from bench_data/<config>_cf05.npz")
    p.add_argument("--ds", type=float, default=0.1, help="continuation step size (--mode continuation)")
    p.add_argument("--cont-tol", type=float, default=1e-4,
                   help="FGMRES tolerance of the continuation's solves (run/ocean solver_params.xml: 1e-4)")
    p.add_argument("--cpu-child", default=None, help=argparse.SUPPRESS)
    p.add_argument("--cpu-iters", type=int, default=8,
                   help="FGMRES iterations of the bounded CPU sample (--mode continuation)")
    a = p.parse_args()
    if a.dyn_iters is None:
        a.dyn_iters = 8 if a.config == "global1" else 4
    return a


def schur_where(k, n):
    """which of the n dynamics passes solve the Schur system (iemic_krylov.schur_passes k)"""
    if k <= 0 or k >= n:
        return ", every dynamics pass"
    if k == 1:
        return f", the first of the {n} dynamics passes only"
    first = "the first" if k == 2 else f"the first {k - 1}"
    return f", {k} of the {n} dynamics passes ({first} and the last)"


def quiet_cores(n, dt=0.5):
    """n CPUs of this process's affinity mask on n distinct physical cores, the least busy
    ones over dt seconds of /proc/stat (a shared host's other jobs load some cores: pinning the
    baseline's threads to cores 0..n-1 made its samples spread by 26 %).  Returns (cpus, the
    busiest chosen core's busy fraction), or (None, None) where /proc is not readable."""
    try:
        aff = sorted(os.sched_getaffinity(0))

        def stat():
            out = {}
            with open("/proc/stat") as f:
                for ln in f:
                    if ln.startswith("cpu") and ln[3].isdigit():
                        a = ln.split()
                        v = [int(t) for t in a[1:]]
                        out[int(a[0][3:])] = (v[3] + v[4], sum(v))
            return out

        s0 = stat()
        time.sleep(dt)
        s1 = stat()
        busy = {}
        for c in aff:
            if c in s0 and c in s1:
                tot = s1[c][1] - s0[c][1]
                busy[c] = 1.0 - (s1[c][0] - s0[c][0]) / tot if tot > 0 else 0.0
        core = {}
        for c in busy:
            try:
                with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                    sib = f.read().strip()
            except OSError:
                sib = str(c)
            core.setdefault(sib, []).append(c)
        # a core's load is its busiest sibling's; one CPU (the lowest sibling) per core
        ranked = sorted(((max(busy[c] for c in cs), min(cs)) for cs in core.values()))
        if len(ranked) < n:
            return None, None
        pick = ranked[:n]
        return sorted(c for _, c in pick), round(max(b for b, _ in pick), 3)
    except (OSError, ValueError, AttributeError):
        return None, None


def cpu_baseline(cfg, L, x, args):
    """The CPU baseline of the Newton line (cpu_baseline_run), in a child process started
    after the GPU work: a fresh interpreter that loads numpy and the oracle only (no torch, no
    HIP), so its OpenMP runtime starts with the binding below and no other thread pool shares
    the cores.  OMP_PROC_BIND=close over explicit places: one thread per physical core, the
    OMP_NUM_THREADS least busy cores of the affinity mask (quiet_cores), pinned for the whole
    run (OMP_PLACES=cores when /proc cannot tell, or when the caller set OMP_PLACES)."""
    import subprocess
    import tempfile
    env = dict(os.environ)
    env.setdefault("OMP_PROC_BIND", "close")
    if "OMP_PLACES" not in env:
        cpus, load = quiet_cores(int(env.get("OMP_NUM_THREADS", os.cpu_count() or 1)))
        if cpus:
            env["OMP_PLACES"] = ",".join("{%d}" % c for c in cpus)
            env["IEMIC_CPU_PICK"] = f"{len(cpus)} least busy cores (busiest {load:.0%} over 0.5 s before)"
        else:
            env["OMP_PLACES"] = "cores"
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "state.npz")
        np.savez(path, x=x, L=L)
        cmd = [sys.executable, os.path.abspath(__file__), "--cpu-child", path, "--config", args.config,
               "--mixing", str(args.mixing), "--tol", repr(args.tol), "--krylov", str(args.krylov),
               "--restarts", str(args.restarts), "--ts-sweeps", str(args.ts_sweeps),
               "--dyn-iters", str(args.dyn_iters), "--dyn-omega", repr(args.dyn_omega),
               "--ts-mg", str(args.ts_mg), "--ts-at", str(args.ts_at), "--schur-passes", str(args.schur_passes),
               "--cpu-samples", str(args.cpu_samples), "--cpu-warmup", str(args.cpu_warmup)]
        out = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, check=True, text=True).stdout
    return json.loads(out.strip().splitlines()[-1])


def cpu_baseline_child(args):
    """bench.py --cpu-child <npz>: the CPU baseline process (cpu_baseline)"""
    from iemic import config as cf
    cfg = cf.preset(args.config, mixing=args.mixing)
    with np.load(args.cpu_child, allow_pickle=False) as d:
        x, L = d["x"], d["L"]
    print(json.dumps(cpu_baseline_run(cfg, L, x, args)), flush=True)


def cpu_baseline_run(cfg, L, x, args):
    """The oracle port timed on the host cores for one full Newton step of the same
    workload with the same algorithm: F and J assembly, the block Gauss-Seidel set-up (4
    damped defect-correction passes on the dynamics block, one T/S aggregation-multigrid
    V-cycle with z-line smoothing: oracle/prec_oracle.c, the GPU apply's CPU twin; Schur by
    band LU), FGMRES(krylov) with restarts to the same tolerance (CGS2), x += dx, new F.
    args.cpu_warmup untimed steps, then args.cpu_samples timed steps (10 after 2
    warm-ups); the value is their median."""
    from oracle import oracle as orc
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    places = os.environ.get('OMP_PLACES', 'unset')
    pick = os.environ.get("IEMIC_CPU_PICK")
    bind = f"OMP_PROC_BIND={os.environ.get('OMP_PROC_BIND', 'unset')}, OMP_PLACES={places if not pick else pick}"
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    o = orc.Oracle(cfg.ref_dict(), L, cfg.par_list())
    samples = []
    nwarm = max(0, args.cpu_warmup)
    for it in range(nwarm + max(1, args.cpu_samples)):
        T0 = time.perf_counter()
        t = time.perf_counter()
        F = o.rhs(x)
        t_rhs = time.perf_counter() - t
        t = time.perf_counter()
        val, _ = o.jacobian(x)
        t_jac = time.perf_counter() - t
        t = time.perf_counter()
        P = orc.BlockGS(o, val, args.ts_sweeps, dyn_iters=args.dyn_iters, dyn_omega=args.dyn_omega,
                        ts_mg=args.ts_mg, ts_at=args.ts_at, schur_passes=args.schur_passes)
        t_prec = time.perf_counter() - t
        t = time.perf_counter()
        dx, its, rel, _ = P.fgmres(np.ascontiguousarray(-F), tol=args.tol, m=args.krylov,
                                   maxit=args.krylov * (args.restarts + 1))
        t_solve = time.perf_counter() - t
        F1 = o.rhs(x + dx)
        if it >= nwarm:
            samples.append(time.perf_counter() - T0)
        del P
    order = [v * 1e3 for v in samples]
    ms = sorted(order)
    med = float(np.median(ms))
    q1, q3 = (float(v) for v in np.percentile(ms, [25, 75]))
    return {
        "value": round(med, 1), "unit": "ms/Newton-step", "cores": cores, "kind": "port",
        "samples_ms": [round(v, 1) for v in ms], "samples_in_order_ms": [round(v, 1) for v in order],
        "spread_ms": round(ms[-1] - ms[0], 1),
        "spread_frac": round((ms[-1] - ms[0]) / med, 4), "iqr_frac": round((q3 - q1) / med, 4),
        "warmup": nwarm, "binding": bind, "places": places, "affinity_cpus": aff,
        "sample": (f"median of {len(ms)} timed full Newton steps after {nwarm} untimed warm-up steps "
                   f"on the oracle C port (OpenMP {cores} threads, {bind}; a child process without "
                   f"torch), same state and algorithm; last: F {t_rhs*1e3:.0f} ms, "
                   f"J {t_jac*1e3:.0f} ms, block GS set-up {t_prec*1e3:.0f} ms (dyn x{args.dyn_iters}, "
                   f"T/S multigrid x{args.ts_mg}), FGMRES({args.krylov}) {its} iterations to {rel:.1e} "
                   f"in {t_solve:.1f} s"),
        "iters": its, "norm_f0": float(np.linalg.norm(F)), "norm_f1": float(np.linalg.norm(F1)),
    }


RUN_OCEAN_CONT = {                  # run/ocean/continuation_params.xml
    "continuation parameter": "Combined Forcing", "initial step size": 1.0e-3,
    "minimum step size": 1.0e-8, "maximum step size": 1.0, "Newton tolerance": 1.0e-2,
    "destination tolerance": 1.0e-4, "epsilon increment": 1.0e-5, "normalize strategy": "N",
    "corrector residual test": "D", "state tangent scaling": 1.0,
    "enable Newton Chord hybrid solve": False, "predictor bound": 3000.0,
    "post processing": "never"}


class Ranks:
    """This process's rank of the run (one per GPU, or several per GPU with --transport
    host): torch.distributed set up, the device chosen, the RCCL id broadcast; builds the
    rank's Ocean subdomain and takes max-over-ranks timings."""

    def __init__(self, args):
        import torch
        self.torch = torch
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        self.host = args.transport == "host"
        self.args = args
        self.dist = None
        ndev = torch.cuda.device_count()
        if self.world > 1 and not self.host and ndev < self.world:
            print(f"bench.py: rank {self.rank}: {self.world} RCCL ranks need {self.world} GPUs, {ndev} visible",
                  file=sys.stderr)
            sys.exit(2)
        self.device = local % max(1, ndev) if self.host else local
        if self.world > 1:
            import torch.distributed as dist
            torch.cuda.set_device(self.device)
            if self.host:
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.device))
            self.dist = dist
        self.dev = torch.device("cuda", self.device)
        torch.cuda.set_device(self.dev)
        self.tdev = "cpu" if self.host else self.dev
        self.comm_id, self.tp = None, None
        if self.world > 1 and self.host:
            from iemic.transport import GlooTransport
            self.tp = GlooTransport()
        elif self.world > 1:
            from iemic.ocean import Ocean
            idt = torch.zeros(128, dtype=torch.uint8, device=self.dev)
            if self.rank == 0:
                idt.copy_(torch.frombuffer(bytearray(Ocean.unique_id()), dtype=torch.uint8))
            dist.broadcast(idt, 0)
            self.comm_id = bytes(idt.cpu().numpy().tobytes())

    def ocean(self, cfg, **kw):
        """this rank's Ocean (the Decomp2D subdomain of --npx); exits 2 unless the communicator
        reports WORLD_SIZE ranks"""
        from iemic.ocean import Ocean
        oc = Ocean(cfg, device=self.device, rank=self.rank, nranks=self.world, comm_id=self.comm_id,
                   npx=self.args.npx, transport=self.tp, **kw)
        self.ranks_seen, self.transport = oc.comm_size()
        if self.ranks_seen != self.world:
            print(f"bench.py: rank {self.rank}: the communicator reports {self.ranks_seen} ranks, "
                  f"WORLD_SIZE {self.world}", file=sys.stderr)
            sys.exit(2)
        return oc

    def barrier(self):
        self.torch.cuda.synchronize()
        if self.dist:
            self.dist.barrier()

    def max(self, v: float) -> float:
        if not self.dist:
            return v
        t = self.torch.tensor([v], device=self.tdev, dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def check_agree(self):
        """all ranks saw the same communicator size"""
        if not self.dist:
            return
        rs = self.torch.tensor([self.ranks_seen, -self.ranks_seen], device=self.tdev, dtype=self.torch.float64)
        self.dist.all_reduce(rs, op=self.dist.ReduceOp.MAX)
        if int(rs[0]) != self.world or int(-rs[1]) != self.world:
            print(f"bench.py: ranks disagree on the communicator size ({rs.tolist()})", file=sys.stderr)
            sys.exit(2)

    def gather_ref(self, x):
        """a global reference-ordered host vector of which each rank filled its own rows"""
        if not self.dist:
            return x
        t = self.torch.from_numpy(np.ascontiguousarray(x)).to(self.tdev)
        self.dist.all_reduce(t)
        return t.cpu().numpy()

    def fields(self, oc) -> dict:
        lay = oc.layout()
        return {"n_gpus": self.world, "ranks_seen": self.ranks_seen,
                "process_grid": [lay["npx"], lay["npy"]],
                "parallelism": (f"decomp2d {lay['npx']}x{lay['npy']}" if self.world > 1 else "single"),
                "transport": self.transport if self.world > 1 else "none"}

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def bench_continuation(args, R: Ranks):
    """Config C5: one pseudo-arclength continuation step (Continuation.H:230-298: Euler
    predictor, Newton corrector on the bordered system with two solves per Jacobian,
    587-813) of the 1-degree global ocean (384x152x32, 11.2 M unknowns) with the
    reference's run/ocean settings (continuation_params.xml: Newton tolerance 1e-2;
    solver_params.xml: FGMRES tolerance 1e-4), from the near-solution branch state
    bench_data/<config>_cf05.npz (the model continued on the GPU from rest to Combined
    Forcing 0.5, scripts/branch_state.py, fp32-rounded).  The tangent (an Euler tangent: one
    solve with dF/dpar) is formed once, untimed; every timed step restarts from that state,
    tangent and step size ds.  The continuation's vectors live in HBM (iemic.ocean.DeviceOps):
    on N ranks each holds its subdomain's rows and every dot / norm is summed over the ranks
    (the reference's Utils::dot on the Epetra solve map) -- strong scaling, max over ranks."""
    from iemic import config as cf
    from iemic.continuation import Continuation
    cfg = cf.preset(args.config, mixing=args.mixing)
    fix = os.path.join(ROOT, "bench_data", f"{args.config}_cf05.npz")
    with np.load(fix, allow_pickle=False) as d:
        x0 = d["x"].astype(np.float64)
        par0 = float(d["par"])
    sp = {"FGMRES tolerance": args.cont_tol, "FGMRES iterations": args.krylov, "FGMRES restarts": args.restarts,
          "Dyn iterations": args.dyn_iters, "Dyn damping": args.dyn_omega, "TS multigrid cycles": args.ts_mg}
    oc = R.ocean(cfg, solver_params=sp)
    solves = []
    oc.solve_hook = solves.append
    oc.setState(x0)
    oc.setPar("Combined Forcing", par0)
    cont = Continuation(oc, {**RUN_OCEAN_CONT, "initial step size": args.ds})
    ops = cont.ops
    cont.initialize()
    cont.createInitialTangent()
    saved = (cont.state, cont.par, cont.stateDot, cont.parDot)   # device vectors, never modified

    def step():
        st, par, sd, pd = saved
        ops.set_state(st)
        oc.setPar("Combined Forcing", par)
        cont.state, cont.par, cont.stateDot, cont.parDot, cont.ds = st, par, sd, pd, args.ds
        cont.store()
        solves.clear()
        R.barrier()
        t = time.perf_counter()
        rc = cont.step()
        R.barrier()
        return rc, time.perf_counter() - t, list(solves)

    for _ in range(args.warmup):
        step()
    oc.comm_stats()
    recs = [step() for _ in range(args.steps)]
    comm = oc.comm_stats()
    ms = R.max(sum(r[1] for r in recs) / len(recs) * 1e3)
    R.check_agree()
    rc, _, sv = recs[-1]
    its = [s.iters for s in sv]
    # SpMV roofline of the 1-degree operator (this rank's rows): HIP events on the library
    # stream, hot, after the timed steps
    oc.computeJacobian()
    sp_ms = oc.time_spmv(20)
    from iemic import _lib
    nnz = int(_lib.lib().iemic_graph_nnz(oc._h))
    nown = oc.layout()["own_rows"]
    bsp = spmv_bytes(nnz, nown)
    ell = stencil_ell_bytes(nown // 6, 104, nown)
    achieved = bsp / (sp_ms * 1e-3) / 1e9
    real = ell / (sp_ms * 1e-3) / 1e9
    its_total = max(1, sum(its))
    out = {"metric": "1-degree continuation-step wall time (config C5: predictor + bordered Newton corrector)",
           "value": round(ms, 1), "unit": "ms/continuation-step", "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(ms, 1), "higher_is_better": False,
           "scaling": "strong" if R.world > 1 else "none", "vs_baseline": None, "dtype": "f64",
           "data": ("near-solution state: global1 continued on the GPU from rest to Combined Forcing "
                    f"{par0:.5f} with the reference's run/ocean settings (scripts/branch_state.py; "
                    "bench_data/global1_cf05.npz, fp32-rounded); Euler tangent formed untimed"),
           "config": {"workload": f"{args.config} {cfg.n}x{cfg.m}x{cfg.l} Mixing={args.mixing}, one "
                                  f"continuation step ds={args.ds:g} (Newton tol 1e-2, FGMRES tol {args.cont_tol:g})",
                      "rows": cfg.nrows, "nnz_rank0": nnz, "krylov_dim": args.krylov, "restarts": args.restarts},
           **R.fields(oc),
           "comm": {"per_fgmres_step": {k: round(v / (its_total * args.steps), 2) for k, v in comm.items()},
                    "rank": R.rank},
           "continuation": {"rc": rc, "newton_iters": cont.newtonIter, "par": cont.par,
                            "norm_f": cont.normRHStest, "norm_rhs": cont.normRHS, "fgmres_iters": its,
                            "solve_ms": [round(s.t_total_ms, 1) for s in sv],
                            "vectors": "device (iemic_vec_*, summed over the ranks)"},
           "roofline": {"kernel": "k_spmv7 (1-degree operator, rank 0's rows, HIP events, 20 back-to-back launches)",
                        "bound": "hbm", "achieved": round(real, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(real / HBM_PEAK_GBS, 4), "traffic": None, "bytes_basis": "stencil_ell_bytes",
                        "achieved_csr": round(achieved, 1), "frac_csr": round(achieved / HBM_PEAK_GBS, 4),
                        "algorithmic_bytes": bsp, "stencil_ell_bytes": ell, "launch_us": round(sp_ms * 1e3, 2)},
           "cpu_baseline": None}
    if not args.no_cpu and R.world == 1:
        out["cpu_baseline"] = cpu_continuation_sample(cfg, oc, cont, saved, its, args)
    if R.rank == 0:
        print(json.dumps(out), flush=True)


def cpu_continuation_sample(cfg, oc, cont, saved, its, args):
    """Bounded CPU sample of the C5 step on the oracle port (16 threads): F, J, the block
    GS set-up and args.cpu_iters FGMRES iterations timed at the predicted state, scaled to
    the GPU step's work (its Newton iterations' F/J/set-up and its FGMRES iterations)."""
    from oracle import oracle as orc
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    L = oc.landmask().reshape(cfg.l + 2, cfg.m + 2, cfg.n + 2)
    o = orc.Oracle(cfg.ref_dict(), L, cfg.par_list())
    st, par, sd, pd = saved
    x = cont.ops.to_host(st) + args.ds * cont.ops.to_host(sd)
    o.set_par(19, par + args.ds * pd)        # Combined Forcing (par2int COMB = 19)
    t = time.perf_counter()
    F = o.rhs(x)
    t_rhs = time.perf_counter() - t
    t = time.perf_counter()
    val, _ = o.jacobian(x)
    t_jac = time.perf_counter() - t
    t = time.perf_counter()
    P = orc.BlockGS(o, val, args.ts_sweeps, dyn_iters=args.dyn_iters, dyn_omega=args.dyn_omega,
                    ts_mg=args.ts_mg, schur_passes=args.schur_passes)
    t_prec = time.perf_counter() - t
    t = time.perf_counter()
    _, k, _, _ = P.fgmres(np.ascontiguousarray(-F), tol=1e-30, m=args.cpu_iters, maxit=args.cpu_iters)
    t_it = (time.perf_counter() - t) / max(1, k)
    newton = cont.newtonIter
    # per Newton iteration: F for dF/dpar (2 F evaluations; the first iteration 3), J,
    # preconditioner set-up; the predictor's F; the FGMRES iterations of the step's solves
    est = ((2 * newton + 2) * t_rhs + newton * (t_jac + t_prec) + sum(its) * t_it) * 1e3
    return {"value": round(est, 1), "unit": "ms/continuation-step", "cores": cores, "kind": "port",
            "sample": (f"bounded sample on the oracle C port ({cores} threads) at the step's predicted state: "
                       f"F {t_rhs*1e3:.0f} ms, J {t_jac*1e3:.0f} ms, block GS set-up {t_prec*1e3:.0f} ms, "
                       f"{k} FGMRES iterations at {t_it*1e3:.0f} ms each; scaled to the GPU step's "
                       f"{newton} Newton iterations and {sum(its)} FGMRES iterations ({its})"),
            "timed": True, "extrapolated": True}


def bench_coupled(args, R: Ranks):
    """Config C4: the coupled ocean + atmosphere model at 4 degrees (run/coupled: ocean
    96x38x12 with Coupled Temperature = 1, Mixing 1; the atmosphere on the same grid),
    one Newton step of CoupledModel (F, J, the block Gauss-Seidel preconditioner set-up,
    FGMRES or IDR(s) to tol, update, F).  On N ranks the ocean is split into Decomp2D
    subdomains and the atmosphere replicated (CoupledModel.C:274-343); max over ranks."""
    from iemic import config as cf
    from iemic.coupled import RUN_COUPLED_ATMOS, Atmosphere, CoupledModel
    cfg = cf.preset("coupled4")
    fix = os.path.join(ROOT, "bench_data", "coupled4_cf015.npz")
    branch = args.state == "branch" and os.path.exists(fix)
    if branch:
        # near-solution state of both models: the coupled model continued on the GPU from
        # rest with run/coupled's settings to Combined Forcing 0.15
        # (scripts/coupled_branch_state.py), fp32-rounded
        with np.load(fix, allow_pickle=False) as d:
            xo_b, xa_b, comb = d["x"].astype(np.float64), d["xa"].astype(np.float64), float(d["par"])
    else:
        comb = cfg.start_params["Combined Forcing"]
    oc = R.ocean(cfg, solver_params={"Dyn iterations": args.dyn_iters})
    atm = Atmosphere(oc, {**RUN_COUPLED_ATMOS, "Combined Forcing": comb})
    sp = {"FGMRES iterations": args.krylov, "FGMRES restarts": args.restarts,
          "FGMRES tolerance": args.tol, "Solver": args.solver, "IDR s": args.idr_s}
    cm = CoupledModel(oc, atm, sp)
    cm.setPar("Combined Forcing", comb)
    L = oc.landmask().reshape(cfg.l + 2, cfg.m + 2, cfg.n + 2)
    if branch:
        xo, xa = xo_b, xa_b
    else:
        xo = cf.synthetic_state(cfg, L, amp_ts=args.amp_ts)
        # the atmosphere state of the coupled fixture (idealized profile + seeded noise,
        # tests/golden/make_golden_coupled.py atmos_state)
        with np.load(os.path.join(ROOT, "bench_data", "coupled4_atmos.npz"), allow_pickle=False) as d:
            xa = d["xa"].astype(np.float64)

    def step():
        oc.setState(xo)
        atm.setState(xa)
        return cm.newtonStep()

    for _ in range(args.warmup):
        step()
    R.barrier()
    oc.comm_stats()
    recs = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        recs.append(step())
    R.barrier()
    ms = R.max((time.perf_counter() - t0) / args.steps * 1e3)
    comm = oc.comm_stats()
    R.check_agree()
    r = recs[-1]
    seq = []
    if args.newton_seq > 0:
        oc.setState(xo)
        atm.setState(xa)
        for _ in range(args.newton_seq):
            q = cm.newtonStep(allow_unconverged=True)
            seq.append({k: q[k] for k in ("norm_f0", "norm_f1", "iters", "converged") if k in q})
    # SpMV roofline: the ocean block's k_spmv7 (HIP events on the library stream, hot)
    from iemic import _lib
    oc.setState(xo)
    oc.computeJacobian()
    sp_ms = oc.time_spmv(50)
    nnz = int(_lib.lib().iemic_graph_nnz(oc._h))
    bsp = spmv_bytes(nnz, cfg.nrows)
    achieved = bsp / (sp_ms * 1e-3) / 1e9
    out = {"metric": "coupled ocean+atmosphere Newton-step wall time (config C4)",
           "value": round(ms, 3), "unit": "ms/Newton-step", "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": False,
           "scaling": "strong" if R.world > 1 else "none", "vs_baseline": None, "dtype": "f64",
           **R.fields(oc),
           "comm": {"per_newton_step": {k: round(v / args.steps, 1) for k, v in comm.items()}, "rank": R.rank},
           "data": (("near-solution state of both models: coupled4 continued on the GPU from rest with "
                     "run/coupled's settings to Combined Forcing 0.15 (scripts/coupled_branch_state.py; "
                     "bench_data/coupled4_cf015.npz, fp32-rounded); states reset from host each step")
                    if branch else
                    (f"synthetic ocean state (splitmix64, T,S ~ U(+-{args.amp_ts:g})), atmosphere "
                     "state bench_data/coupled4_atmos.npz (idealized profile + seeded noise); "
                     "Combined Forcing 0.5; states reset from host each step")),
           "config": {"workload": "coupled4: ocean 96x38x12 (coupled T, Mixing 1) + atmosphere "
                                  "96x38 (T, q, A, P), one Newton step", "rows": cm.N,
                      "solver": args.solver if args.solver == "FGMRES" else f"IDR({args.idr_s})",
                      "prec": "forward block Gauss-Seidel: ocean block GS, atmosphere exact"},
           "newton": {**r, "sequence": seq},
           "roofline": {"kernel": "k_spmv7 (ocean block, 4 degrees; HIP events, 50 back-to-back launches)",
                        "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                        "algorithmic_bytes": bsp, "launch_us": round(sp_ms * 1e3, 2)},
           "cpu_baseline": None}
    if not args.no_cpu and R.world == 1:
        from oracle import atmos_oracle as ao
        from oracle import oracle as orc
        cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
        cb = orc.coupled_newton_step(cfg, L, xo, xa, comb, ao.COUPLED_RUN_PARAMS, ts_sweeps=args.ts_sweeps,
                                     dyn_iters=args.dyn_iters, dyn_omega=args.dyn_omega, ts_mg=args.ts_mg,
                                     schur_passes=args.schur_passes, tol=args.tol, m=args.krylov, maxit=args.krylov * (args.restarts + 1))
        out["cpu_baseline"] = {
            "value": round(cb["total"] * 1e3, 1), "unit": "ms/Newton-step", "cores": cores, "kind": "port",
            "sample": (f"timed, one full coupled Newton step on the CPU restatements ({cores} OpenMP threads "
                       f"for the ocean): oracle/thcm_oracle.c in coupled mode (bitwise vs the reference "
                       f"Fortran) + oracle/atmos_oracle.py, forward block GS (ocean prec_oracle.c, "
                       f"atmosphere sparse LU), FGMRES({args.krylov}) in numpy: F {cb['t_rhs']*1e3:.0f} ms, "
                       f"J {cb['t_jac']*1e3:.0f} ms, set-up {cb['t_prec']*1e3:.0f} ms, {cb['iters']} iterations "
                       f"to {cb['rel']:.1e} in {cb['t_solve']:.1f} s"),
            "iters": cb["iters"]}
        out["newton"]["norm_f0_cpu"] = cb["norm_f0"]
        out["newton"]["norm_f1_cpu"] = cb["norm_f1"]
    if R.rank == 0:
        print(json.dumps(out), flush=True)


def launch(args) -> int:
    """--gpus N > 1 outside torch.distributed.run: start the N ranks as a torch.distributed.run
    child (nothing in this process touches the GPU: device_count() does not initialise it) and
    return its exit code."""
    import socket
    import subprocess
    if args.transport == "rccl":
        import torch
        ndev = torch.cuda.device_count()
        if ndev < args.gpus:
            print(f"bench.py: --gpus {args.gpus} needs {args.gpus} GPUs for RCCL (one per rank), "
                  f"{ndev} visible (--transport host runs several ranks on one GPU)", file=sys.stderr)
            return 2
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.cpu_child:
        cpu_baseline_child(args)
        return
    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and world_env is None:
        sys.exit(launch(args))
    world = int(world_env or "1")
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE = {world} ranks were started", file=sys.stderr)
        sys.exit(2)
    R = Ranks(args)
    try:
        if args.config == "coupled4":
            bench_coupled(args, R)
        elif args.mode == "continuation":
            bench_continuation(args, R)
        else:
            bench_newton(args, R)
    finally:
        R.close()


def bench_newton(args, R: Ranks):
    """The BASELINE metric: one full Newton step of the 2-degree ocean (module docstring)."""
    import torch
    from iemic import _lib
    from iemic import config as cf
    rank, world, dev = R.rank, R.world, R.dev
    dist = R.dist

    cfg = cf.preset(args.config, mixing=args.mixing)
    sp = {"Preconditioner": args.prec, "FGMRES tolerance": args.tol,
          "FGMRES iterations": args.krylov, "FGMRES restarts": args.restarts,
          "TS sweeps": args.ts_sweeps, "Orthogonalization": args.orth,
          "Dyn iterations": args.dyn_iters,
          "Dyn damping": args.dyn_omega, "Dyn minimal residual": args.dyn_mr,
          "TS multigrid cycles": args.ts_mg, "Multigrid sweeps": args.mg_sweeps,
          "Solver": args.solver, "IDR s": args.idr_s, "TS after dyn pass": args.ts_at,
          "Schur passes": args.schur_passes}
    oc = R.ocean(cfg, solver_params=sp)
    ranks_seen, transport = R.ranks_seen, R.transport
    L = oc.landmask().reshape(cfg.l + 2, cfg.m + 2, cfg.n + 2)
    fix = os.path.join(ROOT, "bench_data", f"{args.config}_cf05.npz")
    state = args.state if (args.state == "synthetic" or os.path.exists(fix)) else "synthetic"
    if state == "branch":
        with np.load(fix, allow_pickle=False) as d:
            x0h = d["x"].astype(np.float64)
        if args.mixing != 1:
            raise SystemExit("the branch state was continued with Mixing = 1")
        data = ("near-solution state: global2 continued on the GPU from rest to Combined Forcing "
                "0.5 with the reference's run/ocean continuation settings (scripts/branch_state.py; "
                "bench_data/global2_cf05.npz, fp32-rounded); one Newton step at Combined Forcing 0.5 "
                "from it. SURVEY §8d's synthetic U(+-0.1) T/S state is not a Newton iterate "
                "(the step from it diverges; --state synthetic)")
    else:
        x0h = cf.synthetic_state(cfg, L, amp_ts=args.amp_ts)
        data = (f"synthetic (splitmix64 seed 20261015 state, u,v,w,p ~ U(+-1e-3), T,S ~ "
                f"U(+-{args.amp_ts:g}); Combined Forcing 0.5)")
    x0 = torch.from_numpy(x0h).to(dev)
    L_ = _lib.lib()
    torch.cuda.synchronize()

    def step():
        _lib.check(L_.iemic_set_state_dev(oc._h, x0.data_ptr()), "set_state_dev")
        return oc.newtonStep()

    for _ in range(args.warmup):
        step()
    R.barrier()
    oc.comm_stats()                      # reset the counters: the timed steps only
    infos = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        infos.append(step())
    R.barrier()
    dt = time.perf_counter() - t0
    ms = R.max(dt / args.steps * 1e3)
    comm = oc.comm_stats()
    its_total = sum(i.solve.iters for i in infos)
    R.check_agree()

    if args.save_x1:
        # the updated state of the last timed step: each rank's owned rows, summed over ranks
        x1 = R.gather_ref(oc.getState())
        if rank == 0:
            np.savez(args.save_x1, x0=x0h, x1=x1)

    # SpMV roofline: the k_spmv launches of the timed Newton steps themselves (HIP events
    # on the library stream around every SpMV inside FGMRES; at N > 1 the span includes
    # the halo exchange), so the rocprofv3 average of the same command agrees.
    n_sp = sum(i.solve.n_spmv for i in infos)
    spmv_ms = sum(i.solve.t_spmv_ms for i in infos) / max(1, n_sp)
    nnz = int(L_.iemic_graph_nnz(oc._h))          # rows owned by this GPU
    lay = oc.layout()
    nown = lay["own_rows"]
    bsp = spmv_bytes(nnz, nown)
    achieved = bsp / (spmv_ms * 1e-3) / 1e9
    # the in-solve SpMV (k_spmv7c) reads the coefficients of the active cells only (packed per
    # Jacobian, BlockGS::spc) and writes their rows (FGMRES's compressed basis); x is read
    # whole: its stencil-ELL minimum
    nact = oc.active_cells() if args.solver == "FGMRES" and args.orth == "DCGS2" and args.prec == 2 else 0
    ell = (8 * 104 * nact + 8 * nown + 8 * 6 * nact) if nact else stencil_ell_bytes(nown // 6, 104, nown)
    extra = {}
    if args.spmv_reps > 0 or args.cold_reps > 0:
        oc.setState(x0h)
        oc.computeJacobian()
        if args.spmv_reps > 0:
            extra["hot_us"] = round(oc.time_spmv(args.spmv_reps) * 1e3, 2)
        if args.cold_reps > 0:
            fl = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
            torch.cuda.synchronize()
            extra["cold_us"] = round(oc.time_spmv_cold(fl.data_ptr(), fl.numel(),
                                                       args.cold_reps) * 1e3, 2)
            del fl
    # measured per-kernel PMC bytes and trace times of this step (bench_data/pmc_<tag>.json)
    traffic, trace_us, step_rf, dom_rf = None, None, None, None
    tab, why = pmc_table(args.config) if world == 1 else (None, "one GPU only")
    if tab:
        ks = {r["kernel"]: r for r in tab["kernels"]}
        for kn in ("k_spmv7c", "k_spmv7<true>", "k_spmv7"):
            if kn in ks:
                traffic = ks[kn]["hbm_bytes_per_launch"]
                trace_us = ks[kn]["avg_us"]
                break
        sb = tab["step_hbm_bytes"]
        step_rf = {"hbm_bytes": sb, "ms": round(ms, 3), "achieved": round(sb / (ms * 1e-3) / 1e9, 1),
                   "frac": round(sb / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                   "source": f"bench_data/pmc_{PMC_TAG}.json (PMC counter bytes of one step) / live ms_per_step"}
        d = ks[tab["dominant"]]
        dg = d["hbm_bytes_per_launch"] / (d["avg_us"] * 1e-6) / 1e9
        dom_rf = {"kernel": d["kernel"], "share": round(d["total_ms"] / tab["step_kernel_ms"], 4),
                  "hbm_bytes_per_launch": d["hbm_bytes_per_launch"], "avg_us": d["avg_us"],
                  "achieved": round(dg, 1), "frac": round(dg / HBM_PEAK_GBS, 4),
                  "source": f"bench_data/pmc_{PMC_TAG}.json (PMC bytes / rocprofv3 kernel-trace average)"}

    real_gbps = (traffic if traffic else ell) / (spmv_ms * 1e-3) / 1e9

    # STREAM-copy rate of this box: device-to-device copy of 1 GiB, read +
    # write bytes / time, median of 5 -- the achievable HBM rate beside the 8 TB/s spec
    stream = None
    if rank == 0 and not args.no_stream:
        a = torch.empty(1 << 27, dtype=torch.float64, device=dev)
        b = torch.empty_like(a)
        a.fill_(1.0)
        ts = []
        for _ in range(6):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            b.copy_(a)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        stream = round(2 * a.numel() * 8 / (float(np.median(ts[1:])) * 1e-3) / 1e9, 1)
        del a, b

    # the Newton residual sequence from the benchmark state (untimed)
    seq = []
    if args.newton_seq > 0:
        _lib.check(L_.iemic_set_state_dev(oc._h, x0.data_ptr()), "set_state_dev")
        for _ in range(args.newton_seq):
            inf = oc.newtonStep(allow_unconverged=True)
            seq.append({"norm_f0": inf.norm_f0, "norm_f1": inf.norm_f1, "fgmres_iters": inf.solve.iters,
                        "converged": inf.solve.converged})

    last = infos[-1]
    s = last.solve
    out = {
        "metric": "Newton-step wall time + SpMV achieved HBM GB/s, 2deg global ocean",
        "value": round(ms, 3), "unit": "ms/Newton-step", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
        "higher_is_better": False, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": data,
        "config": {"workload": f"{args.config} {cfg.n}x{cfg.m}x{cfg.l} Mixing={args.mixing}, one Newton "
                               f"step (F, J, prec, FGMRES tol {args.tol:g}, update, F)",
                   "rows": cfg.nrows, "nnz": nnz, "prec": args.prec,
                   "krylov_dim": args.krylov, "restarts": args.restarts, "orth": args.orth,
                   "solver": args.solver if args.solver == "FGMRES" else f"IDR({args.idr_s})",
                   "ts_sweeps": args.ts_sweeps, "dyn_iters": args.dyn_iters, "dyn_omega": args.dyn_omega, "dyn_mr": args.dyn_mr,
                   "schur": "cyclic reduction (fp64, exact)" + schur_where(args.schur_passes, args.dyn_iters),
                   "state": (f"branch (bench_data/{args.config}_cf05.npz, CF 0.5)" if state == "branch"
                             else f"synthetic (splitmix64 seed 20261015, T/S amp {args.amp_ts:g})"),
                   "ts_mg": args.ts_mg, "mg_sweeps": args.mg_sweeps, "ts_at": args.ts_at,
                   "schur_passes": args.schur_passes,
                   "parallelism": (f"decomp2d {lay['npx']}x{lay['npy']}" if world > 1 else "single"),
                   "transport": transport if world > 1 else "none",
                   "subdomain_rank0": {"cols": [lay["ib0"], lay["ib1"]], "rows": [lay["jb0"], lay["jb1"]]}},
        "newton": {"iters": s.iters, "converged": s.converged,
                   "explicit_rel_res": s.explicit_rel_res, "norm_f0": last.norm_f0,
                   "norm_f1": last.norm_f1, "t_rhs_ms": last.t_rhs_ms,
                   "t_jac_ms": last.t_jac_ms, "t_prec_ms": last.t_prec_ms,
                   "t_solve_ms": last.t_solve_ms, "t_solve_prec_ms": s.t_prec_ms,
                   "t_solve_spmv_ms": s.t_spmv_ms, "t_solve_orth_ms": s.t_orth_ms,
                   "dgks_reorth": s.reorth, "sequence": seq},
        "hbm_copy_gbps": stream,
        "ranks_seen": ranks_seen,
        "process_grid": [lay["npx"], lay["npy"]],
        "comm": {"per_fgmres_step": {k: round(v / max(1, its_total), 2) for k, v in comm.items()},
                 "per_newton_step": {k: round(v / args.steps, 1) for k, v in comm.items()},
                 "rank": rank},
        "spmv_gbps": round(achieved, 1),
        # frac on the bytes the kernel really moves: the PMC counter bytes per launch when the
        # table matches these sources, else the stencil-ELL minimum (values + x + y); the
        # CSR-equivalent figure of SURVEY §8d (12 nnz + 20 N) is kept apart as frac_csr
        "roofline": {"kernel": "k_spmv (per GPU, rank 0; in-solve launches)", "bound": "hbm",
                     "achieved": round(real_gbps, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(real_gbps / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "bytes_basis": "traffic (PMC)" if traffic else "stencil_ell_bytes",
                     "achieved_csr": round(achieved, 1), "frac_csr": round(achieved / HBM_PEAK_GBS, 4),
                     "algorithmic_bytes": bsp, "stencil_ell_bytes": ell, "active_cells": nact,
                     "ell_gbps": round(ell / (spmv_ms * 1e-3) / 1e9, 1),
                     # launch_us: HIP events of every in-solve SpMV launch of the timed steps,
                     # recorded by the dispatch itself (hipExtLaunchKernelGGL start / stop
                     # events on the library stream: the kernel's own begin and end);
                     # trace_us: the rocprofv3 kernel-trace average of the same kernel in the
                     # same command (bench_data/pmc_<tag>.json)
                     "launch_us": round(spmv_ms * 1e3, 2), "launches": n_sp, "trace_us": trace_us,
                     "step": step_rf, "dominant": dom_rf, **({"table": why} if why else {}), **extra},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        cb = cpu_baseline(cfg, L, x0h, args)
        out["newton"]["norm_f0_rel_diff_vs_oracle"] = abs(last.norm_f0 - cb.pop("norm_f0")) / last.norm_f0
        out["newton"]["norm_f1_cpu"] = cb.pop("norm_f1")
        out["cpu_baseline"] = cb
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
