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

PMC_LAUNCH_ROWS = 16384      # rows per conv launch in the committed PMC passes (tools/gpu_profile.sh)
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s spec
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: f32-input MFMA (= f32 vector) dense peak


def pmc_traffic(kernel):
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


# K6 conv ops: MACs per sample and activation bytes per sample
# (layer input 0 = the u8 frame stack, 28,224 B; f32 NHWC activations after)
CONV_MAC = {1: 400 * 256 * 32, 2: 81 * 512 * 64, 3: 49 * 576 * 64}
ACT_B = {0: 28224, 1: 20 * 20 * 32 * 4, 2: 9 * 9 * 64 * 4, 3: 7 * 7 * 64 * 4}
F16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense f16 / bf16 MFMA
# rocprofv3 kernel names of the conv entry points (for the PMC traffic lookup)
CONV_KERNEL = {("fwd", 1, True): "fwd1_split_kernel<1>",
               ("fwd", 2, True): "sgemm_kernel<SgFwd<32, 20, 20, 4, 4, 2, 64, false>, 4, 2>",
               ("fwd", 3, True): "sgemm_kernel<SgFwd<64, 9, 9, 3, 3, 1, 64, false>, 4, 2>",
               ("dgrad", 2, False): "igemm_kernel<DgradPMProblem<32, 20, 20, 4, 4, 2, 64, 1>>",
               ("dgrad", 2, True): "dgrad2_colp_kernel<true>",
               ("dgrad", 3, True): "sgemm_kernel<SgDgradPM<64, 9, 9, 3, 3, 1, 64>, 4, 2>",
               ("wgrad", 1, True): "wgrad_split_kernel<4, 84, 84, 8, 8, 4, 32, true, 256, true, 1>",
               ("wgrad", 2, True): "wgrad_split_kernel<32, 20, 20, 4, 4, 2, 64, false, 128, false, 1>",
               ("wgrad", 3, True): "wgrad_split_kernel<64, 9, 9, 3, 3, 1, 64, false, 64, false, 1>"}


def conv_roofline(key, kt, totals, solo_kt=None):
    """Roofline of the dominant conv launch: algorithmic FLOPs (2 x MACs x batch) per launch /
    mean HIP-event duration.  The f32 kernels run v_mfma_f32_32x32x2_f32 (peak 157.3 TF/s);
    the split-f16 kernels issue 3 f16 MFMA products per f32 MAC (2 when one operand is the
    u8 frame), so their f32-equivalent peak is 2500 / 3 (or / 2) TF/s."""
    import numpy as np
    name, layer = key.split(":")
    layer = int(layer)
    op = name.replace("ppox_nature_conv_", "").replace("_split", "")
    split = name.endswith("_split")
    batch = float(np.mean([a[2] for _, a in kt]))
    mean_ms = float(np.mean([t for t, _ in kt]))
    flops = 2.0 * CONV_MAC[layer] * batch
    ach = flops / (mean_ms * 1e-3) / 1e12
    products = (2 if (layer == 1 and op != "dgrad") else 3) if split else 1
    peak = F16_MFMA_PEAK_TFLOPS / products if split else FP32_MFMA_PEAK_TFLOPS
    # input + output (fwd), output grad + ReLU mask + input grad (dgrad), input + output grad (wgrad);
    # the split conv2 dgrad reads conv1's ReLU mask as the forward's bitmask (4 B per pixel)
    mask_b = 400 * 4 if (op == "dgrad" and layer == 2 and split) else ACT_B[layer - 1]
    per = ACT_B[layer] + (ACT_B[layer - 1] + mask_b if op == "dgrad" else ACT_B[layer - 1])
    kname = CONV_KERNEL.get((op, layer, split))
    traffic, src = pmc_traffic(kname) if kname else (None, None)
    tot = sum(totals.values()) or 1.0
    # the binding roofline is the larger of the two lower bounds on the launch: MFMA work at
    # the MFMA peak, or the algorithmic bytes at the HBM peak (conv2 dgrad moves 2.0 GB per
    # 87 GFLOP at B = 16384: 252 us of HBM vs 104 us of split-f16 MFMA)
    alg_bytes = batch * per
    t_mfma, t_hbm = flops / (peak * 1e12), alg_bytes / (HBM_PEAK_GBS * 1e9)
    mfma_frac = ach / peak
    hbm_ach = alg_bytes / (mean_ms * 1e-3) / 1e9
    if t_hbm > t_mfma:
        bound, a_val, p_val, unit = "hbm", round(hbm_ach, 1), HBM_PEAK_GBS, "GB/s"
    else:
        bound, a_val, p_val, unit = "mfma", round(ach, 2), round(peak, 1), "TFLOP/s"
    return {"kernel": f"{name} layer {layer}" + (f" = {kname}" if kname else ""), "bound": bound,
            "achieved": a_val, "peak": p_val, "unit": unit, "frac": round(a_val / p_val, 4),
            "traffic": traffic, "traffic_unit": "HBM bytes per launch (rocprofv3 PMC)", "traffic_source": src,
            "alg_bytes_per_launch": alg_bytes, "alg_flops_per_launch": flops,
            "launches": len(kt), "mean_us": round(mean_ms * 1e3, 1),
            "timing": ("HIP events around the timed region's launches on their stream; a launch that shares "
                       "the GPU with side-stream kernels also counts its wait for CUs held by them (the "
                       "persistent conv2 dgrad runs alone from 8192 rows: convs.BWD_SOLO_DGRAD2_BATCH)"),
            "mfma_achieved_tflops": round(ach, 2), "mfma_peak_tflops": round(peak, 1), "mfma_frac": round(mfma_frac, 4),
            "alg_hbm_GBs": round(hbm_ach, 1), "hbm_frac": round(hbm_ach / HBM_PEAK_GBS, 4),
            "lower_bound_us": {"mfma": round(t_mfma * 1e6, 1), "hbm": round(t_hbm * 1e6, 1)},
            "share_of_conv_time": round(totals.get(key, 0.0) / tot, 3),
            "selection": "largest total HIP-event time among the conv entry points in a one-stream warmup "
                         "iteration; the timed launches run beside the side-stream weight gradients "
                         "(convs.BWD_STREAMS), so mean_us includes any sharing of the GPU with them",
            "peak_note": "f32 MFMA 157.3 TF/s" if not split else
                         f"f16 MFMA 2500 TF/s / {products} products per f32 MAC (split-f16, fp32-class accuracy)",
            # the same launches in the one-stream warmup iteration: the kernel alone on the GPU
            "solo": _solo(solo_kt, flops / batch, alg_bytes / batch, peak, bound)}


def _solo(kt, flops_per_row, bytes_per_row, peak, bound):
    import numpy as np
    if not kt:
        return None
    ms = float(np.mean([t for t, _ in kt]))
    rows = float(np.mean([a[2] for _, a in kt]))
    tf = flops_per_row * rows / (ms * 1e-3) / 1e12
    gbs = bytes_per_row * rows / (ms * 1e-3) / 1e9
    return {"mean_us": round(ms * 1e3, 1), "launches": len(kt),
            "frac": round(gbs / HBM_PEAK_GBS if bound == "hbm" else tf / peak, 4),
            "mfma_frac": round(tf / peak, 4), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4)}


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


def gae_large_n(dual, T=128, N=1 << 20, reps=10):
    """K1 at a size where HBM, not latency, bounds it: kernel time by graph replay."""
    import torch
    import native
    f = lambda: torch.randn(T, N, device="cuda")
    r, v = f(), f()
    d = (torch.rand(T, N, device="cuda") < 0.01).to(torch.uint8)
    lv, ld = torch.randn(N, device="cuda"), d[-1].contiguous()
    outs = [torch.empty(T, N, device="cuda") for _ in range(4 if dual else 2)]
    if dual:
        ir, iv, liv = f(), f(), torch.randn(N, device="cuda")
        call = lambda: native.gae_dual(r, v, d, lv, ld, ir, iv, liv, 0.99, 0.99, 0.95, *outs)
    else:
        call = lambda: native.gae(r, v, d, lv, ld, 0.99, 0.95, outs[0], outs[1])
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
    except Exception:
        return None
    ms = s.elapsed_time(e) / reps
    bpe = 33 if dual else 17
    gbs = bpe * T * N / (ms * 1e-3) / 1e9
    return {"T": T, "N": N, "mean_us": round(ms * 1e3, 1), "alg_bytes_per_launch": bpe * T * N,
            "achieved": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--algo", default="ppo", choices=["ppo", "rnd", "icm", "es"])
    p.add_argument("--population", type=int, default=10000, help="ES: perturbations per generation")
    p.add_argument("--es-hidden", default="64,64", help="ES: hidden layer sizes")
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
    # PPOX_DIST_BACKEND=gloo rehearses the multi-rank path with several ranks on one GPU
    # (RCCL refuses two ranks on one device); the driver's runs use RCCL, one GPU per rank
    backend = os.environ.get("PPOX_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            tdist.init_process_group(backend)
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False

    import native
    import phases
    import ppo
    import logger

    if args.algo == "es":
        return bench_es(args, world, rank, tdist)

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

    # the conv entry points (K6), timed with HIP events on their launch stream; the warmup
    # iterations pick the dominant one (largest total time), the timed region times it
    conv_keys = [f"ppox_nature_conv_{op}{m}:{l}" for op in ("fwd", "dgrad", "wgrad") for m in ("", "_split")
                 for l in (1, 2, 3)]
    native.enable_event_timing(conv_keys)
    # the dominant kernel is picked from a warmup iteration on ONE stream: with the backward's
    # weight gradients on a side stream (convs.BWD_STREAMS) concurrent launches stretch each
    # other's event durations, so the pick would follow the overlap, not the kernel's own work;
    # the remaining warmup and the timed region run as configured
    import convs
    streams = convs.BWD_STREAMS
    for w in range(args.warmup):
        convs.BWD_STREAMS = streams and w > 0
        iteration()
        if w == 0:
            solo = {k: native.event_times_ms(k) for k in conv_keys}
            totals = {k: sum(t for t, _ in v) for k, v in solo.items()}
            native.enable_event_timing([])
    convs.BWD_STREAMS = streams
    if args.warmup == 0:
        totals, solo = {k: 0.0 for k in conv_keys}, {}
    prof_kernel = max(totals, key=totals.get) if any(totals.values()) else "ppox_nature_conv_dgrad:2"
    gae_kernel = "ppox_gae" if args.algo != "rnd" else "ppox_gae_dual"
    native.enable_event_timing([prof_kernel])

    phases.enable_timers()
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
    phase_ms = {k: {"gpu_ms": round(v["gpu_ms"] / args.steps, 2), "host_ms": round(v["host_ms"] / args.steps, 2)}
                for k, v in phases.summary().items()}
    phases.enable_timers(False)
    gae_ms = gae_kernel_ms(alg, args.algo == "rnd")
    if world > 1:
        t = torch.tensor([dt], device="cuda", dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        dt = float(t.item())

    env_steps = args.steps * args.envs * args.nstep
    value = env_steps / dt
    conv_impl = getattr(alg.policy.net, "conv_impl", None)
    out = {
        "metric": "env-steps/sec (collect+GAE+PPO update), 4096 envs×128 steps @ 1/2/4/8 GPU",
        "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 2), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (Philox uint8 4x84x84 frames, Bernoulli rewards/dones, device envs)",
        "config": {"workload": f"{env_id} {args.algo.upper()} NatureCNN {args.envs} envs x {args.nstep} steps",
                   "n_envs": args.envs, "n_steps": args.nstep, "n_epochs": args.epochs,
                   "batch_size": args.batch_size, "minibatches_per_epoch": -(-args.envs * args.nstep // args.batch_size),
                   "conv_math": conv_impl.math if conv_impl is not None else None,
                   "parallelism": f"dp{world} (env-sharded, RCCL grad all-reduce)" if world > 1 else "single GPU"},
    }
    # per iteration, rank 0: GPU stream time and host time of each phase (phases.py);
    # gae and episodes run inside collect
    out["phases_ms_per_step"] = phase_ms
    if kt:
        out["roofline"] = conv_roofline(prof_kernel, kt, totals, solo.get(prof_kernel))
        launch_rows = float(np.mean([a[2] for _, a in kt]))
        if out["roofline"].get("traffic") is not None and launch_rows != PMC_LAUNCH_ROWS:
            # the committed PMC passes ran launches of PMC_LAUNCH_ROWS rows (the 1-GPU
            # workload); a per-launch byte count of another size does not apply here
            out["roofline"]["traffic"] = None
            out["roofline"]["traffic_note"] = (f"PMC traffic was measured on {PMC_LAUNCH_ROWS}-row launches "
                                               f"(profiles/); these launches average {launch_rows:.0f} rows")
    if gae_ms:
        n_local = args.envs // world
        alg_bytes = (17 if gae_kernel == "ppox_gae" else 33) * args.nstep * n_local
        mean_ms = gae_ms
        ach = alg_bytes / (mean_ms * 1e-3) / 1e9
        out["gae_roofline"] = {"kernel": gae_kernel, "bound": "hbm", "achieved": round(ach, 1),
                               "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                               "mean_us": round(mean_ms * 1e3, 2), "alg_bytes_per_launch": alg_bytes,
                               "note": "config-size launch (graph replay of the rollout's own GAE call, "
                                       "kernel time only) is latency-bound; large_n: the same kernel on "
                                       "T=128 x N=1,048,576 synthetic streams, timed live here; "
                                       "tools/gae_sweep.py sweeps N"}
        large = gae_large_n(gae_kernel != "ppox_gae")
        if large:
            out["gae_roofline"]["large_n"] = large
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, ROOT)
        from oracle.baseline import atari_ppo_rate
        out["cpu_baseline"] = atari_ppo_rate(args.envs, args.nstep, args.epochs, args.batch_size,
                                             threads=args.cpu_threads or None)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        tdist.destroy_process_group()


FP64_VECTOR_PEAK_TFLOPS = 78.6  # AMD MI355X spec (FP64 vector); not listed in MI355X_MICROARCH.md


def bench_es(args, world, rank, tdist):
    """BASELINE.json config 5: ES-NSRA on Swimmer-v3 (synthetic SwimmerLike episodes of the
    Swimmer shape, 1000 steps), --population perturbations per generation, members sharded
    across ranks.  A step = one generation (noise, every member's episode, update, novelty
    bookkeeping); value = population x episode steps / s (all ranks)."""
    import numpy as np
    import torch
    import native
    import logger
    import evolution_strategies as ES
    np.random.seed(0)
    hidden = [int(x) for x in args.es_hidden.split(",")]
    es = ES.EvolutionStrategy("Swimmer-v3", hidden_sizes=hidden, population_size=args.population, seed=1)
    logger.configure("bench", "Swimmer-v3", quiet=True)
    native.enable_event_timing(["ppox_es_evaluate"])
    es.run(args.warmup, log_interval=10 ** 9)
    native.enable_event_timing(["ppox_es_evaluate"])
    torch.cuda.synchronize()
    if world > 1:
        tdist.barrier()
    t0 = time.perf_counter()
    es.run(args.steps, log_interval=10 ** 9)
    torch.cuda.synchronize()
    if world > 1:
        tdist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device="cuda", dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        dt = float(t.item())
    kt = [(ms, a) for ms, a in native.event_times_ms("ppox_es_evaluate") if a[3] > 1]  # population launches
    native.enable_event_timing([])
    steps = args.steps * args.population * es.T
    out = {"metric": "env-steps/sec (ES-NSRA: population episodes + update), Swimmer-v3 shape",
           "value": round(steps / dt, 1), "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 2), "higher_is_better": True,
           "scaling": "strong", "vs_baseline": None, "dtype": "f64",
           "data": "synthetic SwimmerLike episodes (oracle/es.py dynamics), Philox perturbations",
           "config": {"workload": f"Swimmer-v3 ES-NSRA, {args.population} perturbations/generation",
                      "population": args.population, "hidden": hidden, "episode_len": es.T,
                      "n_params": es.n_params, "parallelism": f"dp{world} (members sharded)" if world > 1 else
                      "single GPU"}}
    if kt:
        mean_ms = float(np.mean([t for t, _ in kt]))
        members = float(np.mean([a[3] for _, a in kt]))
        flops = 2.0 * members * es.T * es.n_params  # one FMA per weight per env step
        ach = flops / (mean_ms * 1e-3) / 1e12
        out["roofline"] = {"kernel": "ppox_es_evaluate (es_eval_kernel)", "bound": "valu-f64", "achieved": round(ach, 2),
                           "peak": FP64_VECTOR_PEAK_TFLOPS, "unit": "TFLOP/s",
                           "frac": round(ach / FP64_VECTOR_PEAK_TFLOPS, 4), "traffic": None,
                           "mean_us": round(mean_ms * 1e3, 1), "launches": len(kt),
                           "alg_flops_per_launch": flops}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
