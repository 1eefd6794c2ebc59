"""Headline benchmark: batched MHPC solves/s (2WB+2SRB trot, BASELINE.json configs[2]/[3]).

One step = one full controller solve of the whole per-GPU batch: mhpc_initialize
(references + PD warm start, MHPCLocomotion::initialization) + mhpc_solve
(MultiPhaseDDP::solve with max_AL_iter=2, max_DDP_iter=3), inputs resident in HBM.
`value` = problems solved by all ranks / max-over-ranks wall time of the K timed steps.
Weak scaling: every rank owns `--batch-per-gpu` independent problems (contiguous shard of
the global x0 stream); there is no collective in the solve itself, only the barrier and
max-reduction of the timing contract and, after the timed region, the all-gather of the
per-problem summaries (RCCL) that rank 0 checks against a 1-GPU solve of the global batch.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch-per-gpu B]
  python bench.py --batch-sweep 1,16,64,256,1024,4096,8192     (1 GPU, one line per batch)

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts the N ranks itself
(one process per GPU, before anything touches the GPU); under torch.distributed.run it is
one of them.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0    # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
FP64_PEAK_TFS = 78.6     # MI355X FP64 vector spec (SURVEY.md 8d secondary roofline)


# ---------------------------------------------------------------------------------------
# rank launcher (parent process: never touches the GPU)
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, script: str = None, argv=None) -> int:
    """Start n ranks of `script` (default: this file with this command line; RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* set as torch.distributed.run would) and wait for
    them; the first failing rank's exit code wins and stops the others."""
    script = script or os.path.abspath(__file__)
    argv = sys.argv[1:] if argv is None else list(argv)
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script] + argv, env=env))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in pending:  # one rank failed: the collectives would hang the rest
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc


# ---------------------------------------------------------------------------------------
def usable_cpus() -> int:
    """CPUs this process may run on: the affinity mask, capped by a cgroup CPU quota (the
    GPU box gives a job a share of the host; os.cpu_count() reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_baseline(desc, opt, sample: int, threads: int, label: str = "C3"):
    """The CPU oracle (restatement of MultiPhaseDDP::solve + the reference's own CasADi
    kernels, oracle/_ref) on the first `sample` problems of the same workload, one problem
    per thread: init+solve, and initialization alone (solve-only = the difference)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import oracle as O
    except Exception as e:  # pragma: no cover
        return None, f"oracle import failed: {e}"
    if not O.available():
        return None, "oracle/_ref not built on this machine"
    from mhpc_minimal_env_amd import configs
    x0 = configs.x0_for(desc, sample)
    O.solve(desc, opt.to_c(), x0[:min(8, sample)], nthreads=threads)  # warm the page cache
    t0 = time.perf_counter()
    O.solve(desc, opt.to_c(), x0, nthreads=threads, do_solve=False)
    t_init = time.perf_counter() - t0
    t0 = time.perf_counter()
    O.solve(desc, opt.to_c(), x0, nthreads=threads)
    dt = time.perf_counter() - t0
    solve_only = sample / (dt - t_init) if dt > t_init else None
    return {
        "value": sample / dt, "unit": "solves/s", "cores": threads, "kind": "port",
        "solve_only_per_s": solve_only, "host_cpus": os.cpu_count(),
        "sample": (f"{sample} {label} problems (same x0 stream), init+solve {dt:.2f} s wall "
                   f"(initialization alone {t_init:.2f} s), CPU restatement of "
                   f"MultiPhaseDDP::solve (g++ -O3) calling the reference's own CasADi kernels "
                   f"(oracle/_ref), one problem per thread on {threads} threads = the CPUs "
                   f"this job may use (affinity / cgroup quota; the host reports "
                   f"{os.cpu_count()})"),
    }, None


def cpu_baseline_mixed(args, opt, threads: int):
    """The CPU oracle on a sample of the mixed workload: the first `n` problems of the same
    global stream (layout b % 6), solved layout by layout on `threads` threads; value = problems
    / total wall time."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import oracle as O
    except Exception as e:  # pragma: no cover
        return None, f"oracle import failed: {e}"
    if not O.available():
        return None, "oracle/_ref not built on this machine"
    descs, _ = layouts_of("mixed", 6)
    # about 15 s of CPU work: C5 problems cost ~3x a C3 problem
    n = args.cpu_sample or 6 * max(1, int(cpu_sample_for(descs[0], opt, threads, seconds=15.0) / 10))
    lay = layouts_of("mixed", n)[1]
    x0 = x0_of("mixed", descs[0], n)
    dt = 0.0
    for l, d in enumerate(descs):
        idx = np.where(lay == l)[0]
        if len(idx) == 0:
            continue
        xl = x0[idx] if d.n_wb > 0 else x0[idx][:, :6]
        t0 = time.perf_counter()
        O.solve(d, opt.to_c(), xl, nthreads=threads)
        dt += time.perf_counter() - t0
    return {"value": n / dt, "unit": "solves/s", "cores": threads, "kind": "port",
            "host_cpus": os.cpu_count(),
            "sample": (f"{n} mixed-workload problems (same x0 stream and layouts), init+solve "
                       f"{dt:.2f} s wall, the CPU restatement of MultiPhaseDDP::solve calling the "
                       f"reference's CasADi kernels (oracle/_ref), one problem per thread on "
                       f"{threads} threads, layout by layout")}, None


def cpu_sample_for(desc, opt, threads: int, seconds: float) -> int:
    """Problems for about `seconds` of CPU-baseline work: time a probe of 2 problems per
    thread and scale (the GPU box's host speed is not known in advance)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    if not O.available():
        return 0
    from mhpc_minimal_env_amd import configs
    n = 2 * threads
    t0 = time.perf_counter()
    O.solve(desc, opt.to_c(), configs.x0_for(desc, n), nthreads=threads)
    per = (time.perf_counter() - t0) / n
    return int(min(max(seconds / max(per, 1e-6), n), 131072))


def load_pmc(kernel: str, batch: int, wl: str = "c3"):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary of the same
    workload and batch size (profiles/pmc_traffic_b<batch>.json for C3,
    profiles/pmc_traffic_<workload>_b<batch>.json otherwise; tools/pmc_summary.py):
    (bytes, file), (None, None) when no such summary is committed."""
    name = f"pmc_traffic_b{batch}.json" if wl == "c3" else f"pmc_traffic_{wl}_b{batch}.json"
    path = os.path.join("profiles", name)
    if not os.path.exists(os.path.join(ROOT, path)):
        return None, None
    try:
        with open(os.path.join(ROOT, path)) as f:
            d = json.load(f)
        return d.get("kernels", {}).get(kernel.split("(")[0], {}).get("hbm_bytes_per_launch"), path
    except Exception:
        return None, None


def roofline_of(stats: dict, batch: int, wl: str = "c3") -> dict:
    """HBM roofline of the kernel with the largest device time (+ its FP64 VALU rate in the
    reference's dense flop count, SURVEY.md 8d secondary roofline)."""
    dom = max(stats, key=lambda k: stats[k]["ms"])
    ks = stats[dom]
    per_launch_s = ks["ms"] / 1e3 / max(ks["launches"], 1)
    bytes_per_launch = ks["alg_bytes"] / max(ks["launches"], 1)
    flops_per_launch = ks.get("alg_flops", 0.0) / max(ks["launches"], 1)
    achieved = bytes_per_launch / per_launch_s / 1e9 if per_launch_s > 0 else 0.0
    traffic, src = load_pmc(dom, batch, wl)
    r = {"kernel": dom, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
         "traffic_source": src, "alg_bytes_per_launch": bytes_per_launch,
         "avg_launch_ms": per_launch_s * 1e3}
    # every kernel with an algorithmic byte model, for the kernels beside the dominant one
    per = {}
    for k, v in stats.items():
        if v["launches"] <= 0 or v["alg_bytes"] <= 0 or v["ms"] <= 0:
            continue
        t = v["ms"] / 1e3 / v["launches"]
        a = v["alg_bytes"] / v["launches"] / t / 1e9
        per[k.split("(")[0]] = {"avg_launch_ms": t * 1e3, "achieved": a, "frac": a / HBM_PEAK_GBS,
                                "traffic": load_pmc(k, batch, wl)[0]}
    r["per_kernel"] = per
    if flops_per_launch > 0 and per_launch_s > 0:
        tf = flops_per_launch / per_launch_s / 1e12
        model = ("per trial knot: the reference's dynamics in CasADi generated-code operation "
                 "counts (Dyn_BS/FS 2301, Dyn_FL 1441, FBDynamics 44) + feedback + Euler step"
                 if dom.startswith("k_rollout") else
                 "reference dense formulation (compute_Qfunction + valuefunction_update per "
                 "knot, impact-aware step)")
        r["valu"] = {"achieved": tf, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                     "frac": tf / FP64_PEAK_TFS, "alg_flops_per_launch": flops_per_launch,
                     "flop_model": model}
    return r


def workload(name: str):
    from mhpc_minimal_env_amd import configs
    from mhpc_minimal_env_amd import locomotion as L
    if name == "mixed":
        return configs.mixed_descs()[0], L.HSDDP_OPTION()
    return getattr(configs, f"{name}_desc")(), L.HSDDP_OPTION()


def layouts_of(name: str, B: int, offset: int = 0):
    """Per-problem layouts of a workload: (descs, layout of each problem) or None.  mixed:
    global problem g takes configs.mixed_descs()[g % 6] (C3 at its four gait points, C5 at two)."""
    if name != "mixed":
        return None
    from mhpc_minimal_env_amd import configs
    descs = configs.mixed_descs()
    return descs, ((offset + np.arange(B)) % len(descs)).astype(np.int32)


def x0_of(name: str, desc, B: int, offset: int = 0):
    from mhpc_minimal_env_amd import configs
    lay = layouts_of(name, B, offset)
    if lay is None:
        return configs.x0_for(desc, B, offset=offset)
    return configs.x0_rows(lay[0], lay[1], offset=offset)


def metric_of(name: str) -> str:
    if name == "mixed":
        return "MHPC solves/sec (mixed gait schedules: 2WB+2SRB trot at 4 gait points, 4WB+6SRB bound at 2)"
    return ("MHPC solves/sec (2WB+2SRB trot)" if name == "c3"
            else "MHPC solves/sec (4WB+6SRB bound)" + (", fp32" if name == "c5f32" else ""))


def workload_text(name: str) -> str:
    if name == "mixed":
        head = ("mixed: problem b has its own phase layout, configs.mixed_descs()[b % 6] = C3 "
                "(2 WB + 2 SRB, PRONK 0.08 s) starting at mode 1 / 2 / 3 / 4 and C5 (4 WB + 6 SRB, "
                "BOUND) starting at mode 1 / 3, one handle, every launch over all six layouts")
    else:
        head = ("C3: 2 WB (modes 1,2) + 2 SRB (modes 3,4), Gait(PRONK) 0.08 s, N=80/phase"
                if name == "c3" else "C5: Gait() BOUND, 4 WB + 6 SRB, N=80/100 alternating")
    return head + ", HSDDP max_AL=2 max_DDP=3; step = initialization + solve of the whole batch"


class Solver:
    """One handle on this rank's GPU, stepping init + solve of its batch."""

    def __init__(self, desc, opt, x0, device, variants=("auto", "auto", "auto", 0, 0), layouts=None,
                 sweep_bits=0):
        from mhpc_minimal_env_amd import capi
        from mhpc_minimal_env_amd import locomotion as L
        self.capi = capi
        self.loco = L.MHPCLocomotion(desc=desc, option=opt, batch=x0.shape[0], device=device)
        if layouts is not None:  # per-problem phase layouts (gait schedules)
            self.loco.set_layouts(*layouts)
        self.loco.set_kernel_variant(bws=variants[0], rollout=variants[1], overlap=variants[2],
                                     sub_batches=variants[3], ro_store=variants[4],
                                     sweep_bits=sweep_bits)
        self.loco.set_initial_condition(x0)
        self.lib, self.h = capi.lib(), self.loco._h
        capi.check(self.lib.mhpc_set_x0(self.h, capi.dptr(self.loco._x0)), "mhpc_set_x0")

    def step(self):
        self.capi.check(self.lib.mhpc_initialize(self.h), "mhpc_initialize")
        self.capi.check(self.lib.mhpc_solve(self.h, None), "mhpc_solve")

    def summary(self, offset: int):
        """Per-problem summary of the last solve (sharding.summary_dtype); the status is
        decoded from the decision trace (abort bit) and the cost."""
        from mhpc_minimal_env_amd import sharding
        sc = self.loco.get_scalars()
        aborted = ((sc["trace"] >> 21) & 1).any(axis=1)
        status = np.where(aborted, 1, np.where(np.isfinite(sc["J"]), 0, 2)).astype(np.int32)
        return sharding.make_summary(offset, sc["J"], sc["viol"], status, sc["V"], sc["trace"])

    def close(self):
        self.loco.close()


def run_c2(args, desc, opt, x0, B, rank, world, local_rank, dist, torch):
    """C2: one WB phase (mode 1, N=120); after a solve (untimed setup) every
    step evaluates 256 trial rollouts (forward_sweep_dynamics_only at the C2 step grid) of
    each problem's nominal + gains.  value = rollouts/s over all ranks."""
    from mhpc_minimal_env_amd import configs
    from mhpc_minimal_env_amd import locomotion as L
    eps = configs.c2_eps(256)
    loco = L.MHPCLocomotion(desc=desc, option=opt, batch=B, device=local_rank)
    loco.set_initial_condition(x0)
    loco.initialization()
    loco.solve_mhpc()
    for _ in range(args.warmup):
        loco.rollout_costs(eps)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    dev_ms = 0.0
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dev_ms += loco.rollout_costs(eps)["ms"]
    barrier()
    dt = time.perf_counter() - t0
    tens = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local_rank}")
    if dist is not None:
        dist.all_reduce(tens, op=dist.ReduceOp.MAX)
        dt = float(tens[0])
    if rank == 0:
        n = world * B * len(eps) * args.steps
        # algorithmic bytes per launch: nominal x,u + K + du of every knot read once per
        # problem (the trials share them), J / viol written per trial
        N = desc.N[0]
        alg = B * ((N - 1) * 8.0 * (18 + 56 + 4) + 16.0 * len(eps))
        per_launch_s = dev_ms / 1e3 / args.steps
        achieved = alg / per_launch_s / 1e9 if per_launch_s > 0 else 0.0
        cpu = {"value": None, "reason": "disabled"}
        if world == 1 and not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as O
            if O.available():
                ns = min(B, 8)
                r = O.rollout_costs(desc, opt.to_c(), x0[:ns], eps, nthreads=1)
                cpu = {"value": ns * len(eps) / r["rollout_cpu_seconds"], "unit": "rollouts/s",
                       "cores": 1, "kind": "port",
                       "sample": f"{ns} C2 problems x {len(eps)} step sizes after the same solve, "
                                 f"oracle forward_sweep_dynamics_only (reference CasADi "
                                 f"kernels), 1 thread, {r['rollout_cpu_seconds']:.2f} s"}
            else:
                cpu = {"value": None, "reason": "oracle/_ref not built on this machine"}
        line = {
            "metric": "C2 trial rollouts/sec (1 WB phase N=120, 256 step sizes per nominal)",
            "value": n / dt, "unit": "rollouts/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (x0 = reference default + splitmix64 perturbation)",
            "config": {"workload": "C2: WB mode 1, dt=(float)(0.08f/120), N=120; step = 256 "
                                   "trial rollouts (costs) of every problem's nominal+gains",
                       "batch_per_gpu": B, "global_batch": world * B,
                       "parallelism": f"batch-sharded x{world}"},
            "roofline": {"kernel": "k_eps_rollout", "bound": "hbm", "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": None, "alg_bytes_per_launch": alg,
                         "avg_launch_ms": per_launch_s * 1e3},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), file=_LINE_OUT or sys.stdout, flush=True)
    loco.close()
    if dist is not None:
        dist.destroy_process_group()


def knot_steps_per_rollout(wl, desc) -> int:
    """Rollout knots of one problem for SURVEY.md 8(d)'s "knot-steps/s" diagnostic (the serial
    knot-steps of the reference's solve: every knot swept backward, failed attempts included,
    plus one rollout's knots per forward sweep and per line search, whose trials run side by
    side: one rollout deep).  0 for the mixed workload, whose batch counters do not separate
    its layouts, and for C2."""
    if wl not in ("c3", "c5", "c5f32"):
        return 0
    return sum(desc.N[p] - 1 for p in range(desc.n_phases))

def run_sweep(args, torch):
    """One JSON line per batch size (1 GPU): throughput and the latency of one controller
    solve (init + solve of the batch; at batch 1 the real-time MPC tick of
    MHPCLocomotion::solve_mhpc, MHPCLocomotion.cpp:167-195)."""
    from mhpc_minimal_env_amd import configs
    desc, opt = workload(args.workload)
    for B in [int(b) for b in args.batch_sweep.split(",")]:
        s = Solver(desc, opt, x0_of(args.workload, desc, B), 0,
                   (args.bws_variant, args.ro_variant, args.overlap, args.sub_batches, args.ro_store),
                   layouts=layouts_of(args.workload, B))
        for _ in range(args.warmup):
            s.step()
        solve_ms = 0.0
        ddp = knots = 0
        kroll = knot_steps_per_rollout(args.workload, desc)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            s.step()
            c = s.loco.get_counters()
            solve_ms += c["solve_ms"]
            ddp += c["ddp_iters"]
            knots += c["bws_knots"] + (c["fwd_sweeps"] + c["ddp_iters"]) * kroll
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        # per-kernel event timing in separate steps (see main)
        s.loco.set_profiling(True)
        s.loco.reset_kernel_stats()
        prof_steps = args.profile_steps if args.profile_steps is not None else args.steps
        for _ in range(prof_steps):
            s.step()
        torch.cuda.synchronize()
        s.loco.set_profiling(False)
        stats = s.loco.kernel_stats()
        print(json.dumps({
            "metric": metric_of(args.workload), "batch": B, "value": B * args.steps / dt,
            "unit": "solves/s", "ms_per_step": dt / args.steps * 1e3,
            "latency_ms_per_solve_call": dt / args.steps * 1e3,
            "solve_only_ms": solve_ms / args.steps,
            "solve_only_per_s": B * args.steps / (solve_ms / 1e3) if solve_ms > 0 else None,
            "ddp_iters_per_s": ddp / dt, "knot_steps_per_s": knots / dt if kroll else None,
            "steps": args.steps, "warmup": args.warmup,
            "dtype": "f32" if args.workload == "c5f32" else "f64",
            "kernel_ms_per_step": {k: v["ms"] / max(prof_steps, 1) for k, v in stats.items()},
            "profiled_steps": prof_steps,
            "roofline": roofline_of(stats, B, args.workload),
        }), flush=True)
        s.close()


_LINE_OUT = None  # stdout of the JSON line once library output is diverted (process group)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch-per-gpu", type=int, default=None,
                    help="problems per GPU (default: c3 1024, c5 4096, c2 1)")
    ap.add_argument("--workload", choices=["c3", "c5", "c5f32", "c2", "mixed"], default="c3",
                    help="c3: the headline 2WB+2SRB solve (BASELINE configs[2]); c5: 4WB+6SRB "
                         "bound solve (fp64), c5f32: the same in the fp32 instantiation "
                         "(BASELINE configs[4]); c2: 256 trial rollouts of one nominal per problem; "
                         "mixed: per-problem gait schedules (C3 / C5 layouts at several gait "
                         "points in one batch)")
    ap.add_argument("--no-north-star", action="store_true",
                    help="c3 at N=1: skip the extra batch-4096 measurement (north_star_b4096)")
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="CPU-baseline problems (default: ~15 s of CPU work on the usable cores)")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="CPU-baseline threads (default: every CPU this job may use)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-shard-check", action="store_true",
                    help="N > 1: skip rank 0's 1-GPU re-solve of the global batch")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="N > 1 process group: nccl = RCCL over xGMI (default); gloo only for "
                         "tests on a 1-GPU box (with --share-gpu)")
    ap.add_argument("--dist", action="store_true",
                    help="initialise the process group even at N = 1 (runs the RCCL timing / "
                         "all-gather / shard-check path on a one-GPU box; launch under "
                         "torch.distributed.run)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="test only: every rank uses GPU 0 (rehearsal of the N-rank path on one GPU)")
    ap.add_argument("--bws-variant", default="auto",
                    help="pin the backward-sweep launch variant (capi.BWS_VARIANTS; tuning only)")
    ap.add_argument("--ro-variant", default="auto",
                    help="pin the line-search launch variant (capi.RO_VARIANTS; tuning only)")
    ap.add_argument("--overlap", default="auto", choices=["auto", "on", "off"],
                    help="partials beside the SRB half of the backward sweep (tuning only)")
    ap.add_argument("--profile-steps", type=int, default=None,
                    help="steps run after the timed region with per-launch HIP events (kernel "
                         "times, roofline); default = --steps")
    ap.add_argument("--ro-store", type=int, default=0,
                    help="line-search trials that store their records (0: default; tuning only)")
    ap.add_argument("--sweep-bits", type=int, default=0,
                    help="backward-sweep arithmetic: 0 / 64 double (default), 32 float (c5f32 only)")
    ap.add_argument("--sub-batches", type=int, default=0,
                    help="concurrently scheduled sub-batches per GPU, 1..4 (0 = automatic; tuning only)")
    ap.add_argument("--batch-sweep", default=None,
                    help="comma-separated batch sizes: one JSON line each (1 GPU)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)

    import torch
    if args.batch_sweep:
        if world != 1:
            print("bench.py: --batch-sweep runs on one GPU", file=sys.stderr)
            sys.exit(2)
        return run_sweep(args, torch)
    dist = None
    if args.share_gpu:
        local_rank = 0
    # tensors of the timing / gather collectives live where the backend wants them
    tdev = torch.device(f"cuda:{local_rank}") if args.backend == "nccl" else torch.device("cpu")
    if world > 1 or args.dist:
        # RCCL prints a version banner on stdout when a communicator comes up; the contract's
        # stdout is the one JSON line, so from here on library chatter goes to stderr and the
        # line to a duplicate of the original stdout
        global _LINE_OUT
        sys.stdout.flush()
        _LINE_OUT = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)
        import torch.distributed as dist
        if args.backend == "nccl":
            torch.cuda.set_device(local_rank)
            dist.init_process_group("nccl", device_id=tdev)
        else:
            dist.init_process_group("gloo")
        assert dist.get_world_size() == args.gpus

    from mhpc_minimal_env_amd import configs, sharding

    B = args.batch_per_gpu or {"c3": 1024, "c5": 4096, "c5f32": 4096, "c2": 1,
                               "mixed": 4096}[args.workload]
    desc, opt = workload(args.workload)
    x0 = x0_of(args.workload, desc, B, offset=rank * B)
    if args.workload == "c2":
        return run_c2(args, desc, opt, x0, B, rank, world, local_rank, dist, torch)
    variants = (args.bws_variant, args.ro_variant, args.overlap, args.sub_batches, args.ro_store)
    s = Solver(desc, opt, x0, local_rank, variants, layouts=layouts_of(args.workload, B, rank * B),
               sweep_bits=args.sweep_bits)
    for _ in range(args.warmup):
        s.step()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    solve_ms = 0.0
    ddp_iters = 0
    knot_steps = 0
    kroll = knot_steps_per_rollout(args.workload, desc)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        s.step()
        c = s.loco.get_counters()
        solve_ms += c["solve_ms"]
        ddp_iters += c["ddp_iters"]
        knot_steps += c["bws_knots"] + (c["fwd_sweeps"] + c["ddp_iters"]) * kroll
    barrier()
    dt = time.perf_counter() - t0
    # per-kernel HIP-event timing (an event pair around every launch) in separate steps after
    # the timed region, so the events do not sit between the timed kernels
    s.loco.set_profiling(True)
    s.loco.reset_kernel_stats()
    prof_steps = args.profile_steps if args.profile_steps is not None else args.steps
    for _ in range(prof_steps):
        s.step()
    torch.cuda.synchronize()
    s.loco.set_profiling(False)

    stats = s.loco.kernel_stats()
    tens = torch.tensor([dt, solve_ms / 1e3, float(ddp_iters), float(knot_steps)],
                        dtype=torch.float64, device=tdev)
    shard = None
    if dist is not None:
        tmax = tens[:2].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = tens[2:].clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        dt, solve_s, ddp_total, knot_total = float(tmax[0]), float(tmax[1]), float(tsum[0]), float(tsum[1])
        # per-problem summaries of every rank (RCCL all-gather; outside the timed region)
        allp = sharding.gather_summaries(s.summary(rank * B),
                                         device=tdev if args.backend == "nccl" else None)
        shard = {"ranks": dist.get_world_size(), "backend": dist.get_backend(),
                 "gathered_problems": int(len(allp))}
    else:
        solve_s, ddp_total, knot_total = solve_ms / 1e3, float(ddp_iters), float(knot_steps)
    s.close()

    if rank == 0:
        if shard is not None and not args.no_shard_check:
            # the same global x0 stream solved on one GPU: every gathered summary must be
            # bitwise identical
            one = Solver(desc, opt, x0_of(args.workload, desc, world * B), local_rank,
                         layouts=layouts_of(args.workload, world * B))
            one.step()
            ref = one.summary(0)
            one.close()
            same = all(np.array_equal(allp[k], ref[k], equal_nan=k != "trace")
                       for k in ("index", "J", "viol", "status", "V", "trace"))
            shard["check"] = {"problems": world * B, "bitwise_identical_to_1gpu": bool(same)}
            if not same:
                print("bench.py: sharded results differ from the 1-GPU solve", file=sys.stderr)
        total = world * B * args.steps
        # north star (BASELINE.json: solves/s at batch 4096 on one GPU): the same init + solve
        # step at 4096 problems, measured in this run after the headline's timed region
        ns = None
        if (world == 1 and args.workload == "c3" and B != 4096 and not args.no_north_star
                and dist is None):
            n4 = 4096
            s4 = Solver(desc, opt, x0_of("c3", desc, n4), local_rank)
            for _ in range(args.warmup):
                s4.step()
            torch.cuda.synchronize()
            t4 = time.perf_counter()
            for _ in range(args.steps):
                s4.step()
            torch.cuda.synchronize()
            d4 = time.perf_counter() - t4
            s4.close()
            ns = {"batch": n4, "value": n4 * args.steps / d4, "unit": "solves/s",
                  "ms_per_step": d4 / args.steps * 1e3, "steps": args.steps,
                  "note": "same step (initialization + solve of the whole batch) at the north-star "
                          "batch, timed after the headline's timed region"}
        # mixed: the alternative to one handle of per-problem layouts -- one homogeneous handle
        # per layout holding that layout's problems (same x0 rows), stepped one after the other
        # (each step = init + solve of every handle), timed in this run after the headline
        serial = None
        if world == 1 and args.workload == "mixed" and dist is None:
            descs, lop = layouts_of("mixed", B)
            hs = [Solver(descs[l], opt, x0[lop == l], local_rank) for l in range(len(descs))
                  if (lop == l).any()]
            for _ in range(args.warmup):
                for h in hs:
                    h.step()
            torch.cuda.synchronize()
            t5 = time.perf_counter()
            for _ in range(args.steps):
                for h in hs:
                    h.step()
            torch.cuda.synchronize()
            d5 = time.perf_counter() - t5
            for h in hs:
                h.close()
            serial = {"handles": len(hs), "value": B * args.steps / d5, "unit": "solves/s",
                      "ms_per_step": d5 / args.steps * 1e3,
                      "mixed_over_serial": (total / dt) / (B * args.steps / d5),
                      "note": "same problems, one homogeneous handle per layout, stepped in turn "
                              "(init + solve each), timed after the headline's timed region"}
        # c5f32: the same step with the float backward sweep (MHPC_VARIANT_SWEEP_BITS = 32; the
        # default fp32 sweep computes in double), timed after the headline
        fsw = None
        if world == 1 and args.workload == "c5f32" and args.sweep_bits == 0 and dist is None:
            sf = Solver(desc, opt, x0, local_rank, variants, sweep_bits=32)
            for _ in range(args.warmup):
                sf.step()
            torch.cuda.synchronize()
            t6 = time.perf_counter()
            for _ in range(args.steps):
                sf.step()
            torch.cuda.synchronize()
            d6 = time.perf_counter() - t6
            sf.close()
            fsw = {"value": B * args.steps / d6, "unit": "solves/s", "ms_per_step": d6 / args.steps * 1e3,
                   "note": "same step with the float backward sweep (sweep_bits 32), timed after the "
                           "headline's timed region"}
        cpu, why = (None, "disabled" if world == 1 else "reported at N=1 only")
        if world == 1 and not args.no_cpu_baseline:
            threads = args.cpu_threads or usable_cpus()
            if args.workload == "mixed":
                cpu, why = cpu_baseline_mixed(args, opt, threads)
            else:
                sample = args.cpu_sample or cpu_sample_for(desc, opt, threads, seconds=15.0)
                cpu, why = cpu_baseline(desc, opt, sample, threads, label=args.workload.upper()[:2])
        line = {
            "metric": metric_of(args.workload),
            "value": total / dt,
            "unit": "solves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32" if args.workload == "c5f32" else "f64",
            "data": "synthetic (x0 = reference default + splitmix64 perturbation)",
            "config": {
                "workload": workload_text(args.workload),
                **({"layouts": len(layouts_of("mixed", 6)[0])} if args.workload == "mixed" else {}),
                "batch_per_gpu": B,
                "global_batch": world * B,
                "parallelism": f"batch-sharded x{world}",
            },
            "ddp_iters_per_s": ddp_total / dt,
            "knot_steps_per_s": knot_total / dt if kroll else None,
            "solve_only_per_s": total / solve_s if solve_s > 0 else None,
            "kernel_ms_per_step": {k: v["ms"] / max(prof_steps, 1) for k, v in stats.items()},
            "profiled_steps": prof_steps,
            "roofline": roofline_of(stats, B, args.workload),
            "cpu_baseline": cpu if cpu is not None else {"value": None, "reason": why},
        }
        if ns is not None:
            line["north_star_b4096"] = ns
        if serial is not None:
            line["serial_homogeneous"] = serial
        if fsw is not None:
            line["float_sweep"] = fsw
        if args.workload == "c5f32":
            line["sweep_bits"] = args.sweep_bits or 64
        if shard is not None:
            line["sharding"] = shard
        print(json.dumps(line), file=_LINE_OUT or sys.stdout, flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
