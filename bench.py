"""Headline benchmark: batched MHPC solves/s (2WB+2SRB trot, BASELINE.json configs[2]/[3]).

One step = one full controller solve of the whole per-GPU batch: mhpc_initialize
(references + PD warm start, MHPCLocomotion::initialization) + mhpc_solve
(MultiPhaseDDP::solve with max_AL_iter=2, max_DDP_iter=3), inputs resident in HBM.
`value` = problems solved by all ranks / max-over-ranks wall time of the K timed steps.
Weak scaling: every rank owns `--batch-per-gpu` independent problems (contiguous shard of
the global x0 stream); there is no collective in the solve itself, only the barrier and
max-reduction of the timing contract.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch-per-gpu B]
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

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def cpu_baseline(desc, opt, sample: int, threads: int, label: str = "C3"):
    """The CPU oracle (restatement of MultiPhaseDDP::solve + the reference's own CasADi
    kernels, oracle/_ref) on the first `sample` problems of the same workload."""
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
    O.solve(desc, opt.to_c(), x0, nthreads=threads)
    dt = time.perf_counter() - t0
    return {
        "value": sample / dt, "unit": "solves/s", "cores": threads, "kind": "port",
        "sample": (f"{sample} {label} problems (same x0 stream), init+solve, CPU restatement of "
                   f"MultiPhaseDDP::solve calling the reference's own CasADi kernels "
                   f"(oracle/_ref), g++ -O2, {threads} threads, {dt:.2f} s wall"),
    }, None


def load_pmc(kernel: str, batch: int):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary of the same
    batch size (profiles/pmc_traffic_b<batch>.json, tools/pmc_summary.py)."""
    path = os.path.join(ROOT, "profiles", f"pmc_traffic_b{batch}.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get("kernels", {}).get(kernel.split("(")[0], {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


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
        print(json.dumps(line), flush=True)
    loco.close()
    if dist is not None:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch-per-gpu", type=int, default=None,
                    help="problems per GPU (default: c3 1024, c5 4096, c2 1)")
    ap.add_argument("--workload", choices=["c3", "c5", "c5f32", "c2"], default="c3",
                    help="c3: the headline 2WB+2SRB solve (BASELINE configs[2]); c5: 4WB+6SRB "
                         "bound solve (fp64), c5f32: the same in the fp32 instantiation "
                         "(BASELINE configs[4]); c2: 256 trial rollouts of one nominal per problem")
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="CPU-baseline problems (default: c3 16384, c5 8192)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"# note: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl")

    from mhpc_minimal_env_amd import capi, configs
    from mhpc_minimal_env_amd import locomotion as L

    B = args.batch_per_gpu or {"c3": 1024, "c5": 4096, "c5f32": 4096, "c2": 1}[args.workload]
    desc, opt = getattr(configs, f"{args.workload}_desc")(), L.HSDDP_OPTION()
    x0 = configs.x0_for(desc, B, offset=rank * B)
    if args.workload == "c2":
        return run_c2(args, desc, opt, x0, B, rank, world, local_rank, dist, torch)
    loco = L.MHPCLocomotion(desc=desc, option=opt, batch=B, device=local_rank)
    loco.set_initial_condition(x0)
    lib, h = capi.lib(), loco._h

    def step():
        capi.check(lib.mhpc_initialize(h), "mhpc_initialize")
        capi.check(lib.mhpc_solve(h, None), "mhpc_solve")

    capi.check(lib.mhpc_set_x0(h, capi.dptr(loco._x0)), "mhpc_set_x0")
    for _ in range(args.warmup):
        step()
    loco.set_profiling(True)
    loco.reset_kernel_stats()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    solve_ms = 0.0
    ddp_iters = 0
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        c = loco.get_counters()
        solve_ms += c["solve_ms"]
        ddp_iters += c["ddp_iters"]
    barrier()
    dt = time.perf_counter() - t0

    stats = loco.kernel_stats()
    tens = torch.tensor([dt, solve_ms / 1e3, float(ddp_iters)], dtype=torch.float64,
                        device=f"cuda:{local_rank}")
    if dist is not None:
        tmax = tens[:2].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = tens[2:].clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        dt, solve_s, ddp_total = float(tmax[0]), float(tmax[1]), float(tsum[0])
    else:
        solve_s, ddp_total = solve_ms / 1e3, float(ddp_iters)

    if rank == 0:
        total = world * B * args.steps
        # dominant kernel (largest device time in the timed region) for the roofline
        dom = max(stats, key=lambda k: stats[k]["ms"])
        ks = stats[dom]
        per_launch_s = ks["ms"] / 1e3 / max(ks["launches"], 1)
        bytes_per_launch = ks["alg_bytes"] / max(ks["launches"], 1)
        achieved = bytes_per_launch / per_launch_s / 1e9 if per_launch_s > 0 else 0.0
        roofline = {
            "kernel": dom, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
            "traffic": load_pmc(dom, B), "alg_bytes_per_launch": bytes_per_launch,
            "avg_launch_ms": per_launch_s * 1e3,
        }
        cpu, why = (None, "disabled")
        if world == 1 and not args.no_cpu_baseline:
            cpu, why = cpu_baseline(desc, opt, args.cpu_sample or
                                    (16384 if args.workload == "c3" else 8192),
                                    min(args.cpu_threads, os.cpu_count() or 1),
                                    label=args.workload.upper()[:2])
        line = {
            "metric": ("MHPC solves/sec (2WB+2SRB trot)" if args.workload == "c3"
                       else "MHPC solves/sec (4WB+6SRB bound)"
                       + (", fp32" if args.workload == "c5f32" else "")),
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
                "workload": (("C3: 2 WB (modes 1,2) + 2 SRB (modes 3,4), Gait(PRONK) 0.08 s, "
                              "N=80/phase" if args.workload == "c3" else
                              "C5: Gait() BOUND, 4 WB + 6 SRB, N=80/100 alternating")
                             + ", HSDDP max_AL=2 max_DDP=3; step = initialization + solve of "
                               "the whole batch"),
                "batch_per_gpu": B,
                "global_batch": world * B,
                "parallelism": f"batch-sharded x{world}",
            },
            "ddp_iters_per_s": ddp_total / dt,
            "solve_only_per_s": total / solve_s if solve_s > 0 else None,
            "kernel_ms_per_step": {k: v["ms"] / args.steps for k, v in stats.items()},
            "roofline": roofline,
            "cpu_baseline": cpu if cpu is not None else {"value": None, "reason": why},
        }
        print(json.dumps(line), flush=True)
    loco.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
