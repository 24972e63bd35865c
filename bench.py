#!/usr/bin/env python3
"""Benchmark: env-steps/s of one PPO iteration (collect + GAE + PPO update) on the
BASELINE.json workload, 4096 envs x 128 steps, synthetic Breakout-shaped
(4x84x84 uint8) envs on the device, NatureCNN actor-critic, fp32.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  N > 1: python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
             --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

A "step" is one full PPO iteration over the 4096 x 128 rollout.  The total env
count is fixed as N grows (strong scaling): rank g steps envs [g*4096/N, ...).
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ppo-exploration_amd"))

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s spec
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: f32-input MFMA (= f32 vector) dense peak


def pmc_traffic(kernel="wgrad_kernel<4, 84, 84, 8, 8, 4, 32, true>"):
    """HBM bytes per launch of the dominant kernel from the latest committed rocprofv3 --pmc
    summary (profiles/rNN_pmc_summary.json, made by tools/pmc_summary.py from separate
    FETCH_SIZE / WRITE_SIZE passes of this bench command, gfx950-corrected 2*FETCH + WRITE)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_summary.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f).get(kernel)
    return (None, None) if d is None else (d["hbm_bytes_per_launch_corrected"], os.path.relpath(files[-1], ROOT))


def gae_kernel_ms(alg, dual, reps=20):
    """Kernel time of the rollout's GAE launch (K1) at the config size: the same call on the
    rollout's own buffers, captured `reps` times in a graph and replayed, so the host's
    per-launch cost (~10 us, longer than the kernel) is not counted.  GAE is idempotent on
    its inputs, so re-running it after the timed region changes nothing."""
    import torch
    import native
    ro = alg.rollout
    T = alg.nstep - 1
    if dual:
        call = lambda: native.gae_dual(ro.rewards, ro.values, ro.masks, ro.values[T], ro.masks[T], ro.int_rewards,
                                       ro.int_values, ro.int_values[T], ro.gamma, ro.int_gamma, ro.gae_lam,
                                       ro.advantages, ro.returns, ro.int_advantages, ro.int_returns)
    else:
        call = lambda: native.gae(ro.rewards, ro.values, ro.masks, ro.values[T], ro.masks[T], ro.gamma, ro.gae_lam,
                                  ro.advantages, ro.returns)
    try:
        call()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                call()
        g.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps
    except Exception:  # capture not possible here: report no GAE roofline rather than a wrong one
        return None


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--algo", default="ppo", choices=["ppo", "rnd", "icm"])
    p.add_argument("--envs", type=int, default=4096)
    p.add_argument("--nstep", type=int, default=128)
    p.add_argument("--epochs", type=int, default=10)
    p.add_argument("--batch-size", type=int, default=16384)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=0)
    return p.parse_args()


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as tdist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False

    import native
    import ppo
    import logger

    env_id = {"ppo": "BreakoutNoFrameskip-v4", "icm": "BreakoutNoFrameskip-v4",
              "rnd": "MontezumaRevengeNoFrameskip-v4"}[args.algo]
    cls = {"ppo": ppo.PPO, "icm": ppo.PPO_ICM, "rnd": ppo.PPO_RND}[args.algo]
    np.random.seed(0)
    torch.manual_seed(0)
    kw = dict(rnd_start=0) if args.algo == "rnd" else {}
    alg = cls(env_id=env_id, n_envs=args.envs, nstep=args.nstep, batch_size=args.batch_size,
              n_epochs=args.epochs, seed=1234, quiet=True, **kw)
    logger.configure("bench", env_id, quiet=True)

    def iteration():
        alg.collect_samples()
        alg.train()

    for _ in range(args.warmup):
        iteration()

    # event timing of the dominant kernel (conv1 weight-gradient MFMA GEMM)
    # on the stream it is launched on
    prof_kernel = "ppox_nature_conv_wgrad:1"
    gae_kernel = "ppox_gae" if args.algo != "rnd" else "ppox_gae_dual"
    native.enable_event_timing([prof_kernel])

    torch.cuda.synchronize()
    if world > 1:
        tdist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        iteration()
    torch.cuda.synchronize()
    if world > 1:
        tdist.barrier()
    dt = time.perf_counter() - t0
    kt = native.event_times_ms(prof_kernel)
    native.enable_event_timing([])
    gae_ms = gae_kernel_ms(alg, args.algo == "rnd")
    if world > 1:
        t = torch.tensor([dt], device="cuda", dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        dt = float(t.item())

    env_steps = args.steps * args.envs * args.nstep
    value = env_steps / dt
    out = {
        "metric": "env-steps/sec (collect+GAE+PPO update), 4096 envs×128 steps @ 1/2/4/8 GPU",
        "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 2), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (Philox uint8 4x84x84 frames, Bernoulli rewards/dones, device envs)",
        "config": {"workload": f"{env_id} {args.algo.upper()} NatureCNN {args.envs} envs x {args.nstep} steps",
                   "n_envs": args.envs, "n_steps": args.nstep, "n_epochs": args.epochs,
                   "batch_size": args.batch_size, "minibatches_per_epoch": -(-args.envs * args.nstep // args.batch_size),
                   "parallelism": f"dp{world} (env-sharded, RCCL grad all-reduce)" if world > 1 else "single GPU"},
    }
    # roofline of the dominant kernel: ALGORITHMIC flops per launch / mean launch duration.
    # conv1 wgrad = 2 * batch * 400 output pixels * 256 (ci,ky,kx) * 32 output channels
    if kt:
        flops = [2.0 * a[2] * 400 * 256 * 32 for _, a in kt]
        mean_ms = float(np.mean([t for t, _ in kt]))
        ach = float(np.mean(flops)) / (mean_ms * 1e-3) / 1e12
        traffic, src = pmc_traffic()
        # algorithmic HBM bytes: u8 input (28224 B/sample) + f32 output grad (400*32*4 B/sample)
        alg_bytes = float(np.mean([a[2] for _, a in kt])) * (28224 + 400 * 32 * 4)
        out["roofline"] = {"kernel": "wgrad_kernel<conv1> (ppox_nature_conv_wgrad layer 1)", "bound": "mfma",
                           "achieved": round(ach, 2), "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                           "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": traffic,
                           "traffic_unit": "HBM bytes per launch (rocprofv3 PMC)", "traffic_source": src,
                           "alg_bytes_per_launch": alg_bytes, "launches": len(kt),
                           "mean_us": round(mean_ms * 1e3, 1), "alg_flops_per_launch": float(np.mean(flops))}
    if gae_ms:
        n_local = args.envs // world
        alg_bytes = (17 if gae_kernel == "ppox_gae" else 33) * args.nstep * n_local
        mean_ms = gae_ms
        ach = alg_bytes / (mean_ms * 1e-3) / 1e9
        out["gae_roofline"] = {"kernel": gae_kernel, "bound": "hbm", "achieved": round(ach, 1),
                               "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                               "mean_us": round(mean_ms * 1e3, 2), "alg_bytes_per_launch": alg_bytes,
                               "note": "config-size launch (graph replay of the rollout's own GAE call, "
                                       "kernel time only) is latency-bound; tools/gae_sweep.py sweeps N"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, ROOT)
        from oracle.baseline import atari_ppo_rate
        out["cpu_baseline"] = atari_ppo_rate(args.envs, args.nstep, args.epochs, args.batch_size,
                                             threads=args.cpu_threads or None)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
