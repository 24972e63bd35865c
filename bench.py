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


def pmc_traffic(pattern):
    """HBM bytes per launch of a kernel from the latest committed rocprofv3 --pmc summary
    (profiles/rNN_pmc_summary.json, made by tools/pmc_summary.py from separate FETCH_SIZE /
    WRITE_SIZE passes of this bench command, gfx950-corrected 2*FETCH + WRITE).  `pattern` is a
    regular expression over rocprof's kernel names (template arguments vary with the build's
    forms: Px<> wrappers, IDX flags), matched in full; the summary's first matching key wins."""
    import glob
    import re
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_summary.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        summary = json.load(f)
    d = summary.get(pattern)
    if d is None:
        rx = re.compile(pattern)
        d = next((v for k, v in summary.items() if rx.fullmatch(k)), None)
    return (None, None) if d is None else (d["hbm_bytes_per_launch_corrected"], os.path.relpath(files[-1], ROOT))


# The MFMA kernels of the NatureCNN training pass (K6 convs, K10 fc layer and the heads' hidden
# layer), keyed by their event-timing name (native.enable_event_timing).  Per row (sample) of a
# launch: MACs and algorithmic HBM bytes; `fixed` = bytes per launch independent of
# the row count (weights in, weight gradient out); `products` = f16 MFMA products per f32 MAC of
# the split-f16 form (2 when one operand is the exact u8 frame); `rows_arg` = the entry point's
# argument holding the row count; `rocprof` = a regular expression matching the kernel's rocprofv3
# name (PMC lookup; `PX` / `IDX` below absorb the template flags of the planes / rollout-row forms).
CONV_MAC = {1: 400 * 256 * 32, 2: 81 * 512 * 64, 3: 49 * 576 * 64}
ACT_B = {0: 28224, 1: 20 * 20 * 32 * 4, 2: 9 * 9 * 64 * 4, 3: 7 * 7 * 64 * 4}
BITMASK_B = {1: 400 * 4, 2: 81 * 4, 3: 49 * 4}   # a layer's ReLU bitmask (one u32 per pixel)
F16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense f16 / bf16 MFMA
FC_K, FC_N, HID = 3136, 512, 512


def _sg(prob, tail, raw=False):
    """rocprof name pattern of an sgemm_kernel instance, with or without the Px<> wrapper (PX operands);
    raw: `prob` is already a regular expression"""
    import re
    return r"sgemm_kernel<(Px<)?" + (prob if raw else re.escape(prob)) + r"(, \w+(, \w+)?>)?, " + tail + ">"


def _rows(k, n, mode, bits):
    """SgRows<K, N, MODE, G, BITS[, NB]> with any column-group size and tile width"""
    return _sg(f"SgRows<{k}, {n}, {mode}, \\d+, {bits}(, \\d+)?>", r"4, \d", raw=True)


IDX = r"(, \w+)*"  # trailing template flags


def _kernels():
    import re
    k = {}
    # conv1 in a training pass reads its rows through the rollout index (IDX form <..., true>); the
    # collect pass's forward of the same name without it runs at another row count
    roc = {("fwd", 1): r"fwd1_split_kernel<1, false, true>",
           ("fwd", 2): _sg("SgFwd<32, 20, 20, 4, 4, 2, 64, false>", "4, 2"),
           # (the planes forward: the direct form, csrc/dconv.hip, by default; the sg2 GEMM with PPOX_DCONV3=0;
           # a training pass writes the ReLU bitmask (BITS = true), the collect pass's 4,096-row forward does not)
           ("fwd", 3): r"(dconv_fwd_kernel<DcF3, true>|" + _sg("SgFwd<64, 9, 9, 3, 3, 1, 64, false>", "4, 2") + ")",
           # (PX g2: the direct class-wise form, csrc/dconv.hip, by default; PPOX_DDGRAD2=0: the col2im form)
           ("dgrad", 2): r"(ddgrad2_kernel|dgrad2_colp_kernel<true, false>)",
           # (the direct form, csrc/dconv.hip ddgrad3_kernel, from DDGRAD3_MIN rows; the sg2 GEMM below)
           ("dgrad", 3): r"(ddgrad3_kernel|" + _sg("SgDgradPM<64, 9, 9, 3, 3, 1, 64, true>", "4, 2") + ")",
           ("wgrad", 1): (re.escape("wgrad_split_kernel<4, 84, 84, 8, 8, 4, 32, true, 256, true, 1>")
                          if os.environ.get("PPOX_AB") == "1" and os.environ.get("PPOX_WGRAD1_IM2COL") == "1"
                          else r"wgrad1_frames_kernel<true>"),
           ("wgrad", 2): re.escape("wgrad_split_kernel<32, 20, 20, 4, 4, 2, 64, false, 128, false, 1>"),
           # (PX h2 / g3: the direct form, csrc/dconv.hip dwgrad3_kernel; else the im2col split form)
           ("wgrad", 3): r"(dwgrad3_kernel|" + re.escape("wgrad_split_kernel<64, 9, 9, 3, 3, 1, 64, false, 64, false, 1")
                         + IDX + ">)"}
    for op in ("fwd", "dgrad", "wgrad"):
        for layer in (1, 2, 3):
            if op == "dgrad" and layer == 1:
                continue
            for m in ("", "_split", "_split_idx"):
                if m == "_split_idx" and (op != "wgrad" or layer != 1):
                    continue
                split = m != ""
                # input + output (fwd); output grad + input grad + the input layer's ReLU mask
                # (dgrad: the split kernels read the forward's bitmask); input + output grad (wgrad)
                per = ACT_B[layer] + ACT_B[layer - 1]
                if op == "dgrad":
                    per += BITMASK_B[layer - 1] if split else ACT_B[layer - 1]
                k[f"ppox_nature_conv_{op}{m}:{layer}"] = dict(
                    rows_arg=2, macs=CONV_MAC[layer], bytes=per, fixed=0,
                    products=(2 if layer == 1 and op != "dgrad" else 3) if split else 0,
                    rocprof=roc.get((op, layer)) if split else None, label=f"conv{layer} {op}")
    # H1P (conv1's output as two f16 planes, the size of its f32 form): conv1 forward writing it,
    # conv2 forward and the direct conv2 weight gradient reading it
    k["ppox_nature_conv1_fwd_planes"] = dict(rows_arg=1, macs=CONV_MAC[1], bytes=ACT_B[0] + ACT_B[1], fixed=0,
                                             products=2, rocprof=r"fwd1_split_kernel<1, true, true>", label="conv1 fwd (H1P)")
    k["ppox_nature_conv2_fwd_planes"] = dict(rows_arg=2, macs=CONV_MAC[2], bytes=ACT_B[1] + ACT_B[2], fixed=0,
                                             products=3, rocprof=r"(dconv_fwd_kernel<DcF2, true>|" + _sg("SgFwd2P", "4, 2") + ")",
                                             label="conv2 fwd (H1P)")
    k["ppox_nature_conv2_wgrad_planes"] = dict(rows_arg=2, macs=CONV_MAC[2], bytes=ACT_B[1] + ACT_B[2], fixed=0,
                                               products=3, rocprof="wgrad2_planes_kernel",
                                               label="conv2 wgrad (H1P, direct)")
    w_fc = FC_K * FC_N * 4          # weights in as two fp16 planes (= f32 bytes) / dW out in f32
    k["ppox_nature_fc_fwd"] = dict(rows_arg=1, macs=FC_K * FC_N, bytes=ACT_B[3] + FC_N * 4, fixed=w_fc, products=3,
                                   rocprof=_rows(3136, 512, 0, "false"), label="fc fwd")
    k["ppox_nature_fc_fwd_splitk"] = dict(rows_arg=1, macs=FC_K * FC_N, bytes=ACT_B[3] + FC_N * 4, fixed=w_fc,
                                          products=3, rocprof=r"sgemm_kernel<(Px<)?SgRowsSK<3136, 512, \d+>(, \w+(, \w+)?>)?, 4, 3>",
                                          label="fc fwd split-K")
    k["ppox_nature_fc_dgrad"] = dict(rows_arg=1, macs=FC_K * FC_N, bytes=FC_N * 4 + ACT_B[3] + BITMASK_B[3],
                                     fixed=w_fc, products=3,
                                     # (the direct form, csrc/dconv.hip fcd_kernel, by default; PPOX_DFCD=0: sg2)
                                     rocprof=r"(fcd_kernel|" + _rows(512, 3136, 1, "true") + ")", label="fc dgrad")
    k["ppox_nature_fc_wgrad"] = dict(rows_arg=1, macs=FC_K * FC_N, bytes=FC_N * 4 + ACT_B[3], fixed=w_fc, products=3,
                                     # (PX df and h3: the direct form, csrc/conv.hip fcwg_kernel, round 6; else the
                                     # split wgrad form)
                                     rocprof=r"(fcwg_kernel|" + re.escape(
                                         "wgrad_split_kernel<512, 1, 1, 1, 1, 1, 64, false, 128, false, 49") + IDX + ">)",
                                     label="fc wgrad")
    w_h = HID * HID * 4
    k["ppox_head_hidden_fwd"] = dict(rows_arg=1, macs=HID * HID, bytes=2 * HID * 4, fixed=w_h, products=3,
                                     rocprof=_rows(512, 512, 0, "false"),
                                     label="head hidden fwd")
    # dgrad: de in, the heads' input grad read + written (accumulated in place), f read for the ReLU
    k["ppox_head_hidden_dgrad"] = dict(rows_arg=1, macs=HID * HID, bytes=4 * HID * 4, fixed=w_h, products=3,
                                       rocprof=_rows(512, 512, 2, "false"),
                                       label="head hidden dgrad")
    k["ppox_head_hidden_wgrad"] = dict(rows_arg=1, macs=HID * HID, bytes=2 * HID * 4, fixed=w_h, products=3,
                                       rocprof=re.escape("wgrad_split_kernel<512, 1, 1, 1, 1, 1, 64, false, 128, false, 8>"),
                                       label="head hidden wgrad")
    return k


KERNELS = _kernels()


def _launch_rows(key, args):
    return int(args[KERNELS[key]["rows_arg"]])


def kernel_roofline(key, kt):
    """Roofline of one MFMA kernel over its launches kt = [(ms, args)] of ONE row count:
    algorithmic FLOPs (2 x MACs x rows) and bytes per launch / mean HIP-event duration.
    The f32 kernels run v_mfma_f32_32x32x2_f32 (peak 157.3 TF/s); the split-f16 kernels issue
    `products` f16 MFMA products per f32 MAC, so their f32-equivalent peak is 2500 / products.
    The binding bound is the larger of the two lower bounds (MFMA work at its peak, the
    algorithmic bytes at the HBM peak)."""
    import numpy as np
    spec = KERNELS[key]
    rows = _launch_rows(key, kt[0][1])
    mean_ms = float(np.mean([t for t, _ in kt]))
    flops = 2.0 * spec["macs"] * rows
    alg_bytes = float(spec["bytes"] * rows + spec["fixed"])
    peak = F16_MFMA_PEAK_TFLOPS / spec["products"] if spec["products"] else FP32_MFMA_PEAK_TFLOPS
    t_mfma, t_hbm = flops / (peak * 1e12), alg_bytes / (HBM_PEAK_GBS * 1e9)
    tf = flops / (mean_ms * 1e-3) / 1e12
    gbs = alg_bytes / (mean_ms * 1e-3) / 1e9
    traffic, src = pmc_traffic(spec["rocprof"]) if spec["rocprof"] else (None, None)
    hbm = t_hbm > t_mfma
    return {"kernel": f"{spec['label']} ({key})" + (f" = {spec['rocprof']}" if spec["rocprof"] else ""),
            "bound": "hbm" if hbm else "mfma",
            "achieved": round(gbs, 1) if hbm else round(tf, 2), "peak": HBM_PEAK_GBS if hbm else round(peak, 1),
            "unit": "GB/s" if hbm else "TFLOP/s", "frac": round((gbs / HBM_PEAK_GBS) if hbm else (tf / peak), 4),
            "traffic": traffic, "traffic_source": src,
            "traffic_ratio": round(traffic / alg_bytes, 3) if traffic else None,
            "rows": rows, "launches": len(kt), "mean_us": round(mean_ms * 1e3, 1),
            "alg_bytes_per_launch": alg_bytes, "alg_flops_per_launch": flops,
            "mfma_achieved_tflops": round(tf, 2), "mfma_peak_tflops": round(peak, 1), "mfma_frac": round(tf / peak, 4),
            "alg_hbm_GBs": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4),
            "lower_bound_us": {"mfma": round(t_mfma * 1e6, 1), "hbm": round(t_hbm * 1e6, 1)},
            "peak_note": (f"f16 MFMA 2500 TF/s / {spec['products']} products per f32 MAC (split-f16, fp32-class "
                          "accuracy)") if spec["products"] else "f32 MFMA 157.3 TF/s"}


def same_size(key, kt):
    """The launches of the most frequent row count (a minibatch remainder is a different size)."""
    from collections import Counter
    if not kt:
        return []
    rows = Counter(_launch_rows(key, a) for _, a in kt).most_common(1)[0][0]
    return [(t, a) for t, a in kt if _launch_rows(key, a) == rows]


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
    p.add_argument("--force-dist", action="store_true",
                   help="one rank: run the world > 1 code paths (owned-row minibatches, every collective) over a "
                        "one-rank RCCL communicator — the per-rank program of an 8-GPU run on one GPU")
    p.add_argument("--launch-check", action="store_true",
                   help="launcher rehearsal without a GPU: every rank joins the process group (gloo), agrees on "
                        "the world size and rank 0 prints the line's identity fields with value null")
    return p.parse_args()


def _free_port():
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def launch_ranks(args):
    """`bench.py --gpus N` (N > 1) started as a plain process: run the N ranks through
    torch.distributed.run as a CHILD process (one rank per GPU, rendezvous on 127.0.0.1) and
    forward rank 0's JSON line and the child's exit code.  This process touches no GPU and never
    execs: the ranks initialise their own devices.  (reference step being sharded: ppo.py:241-244)"""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    p = subprocess.run(cmd, stdout=subprocess.PIPE, text=True)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode == 0 and len(lines) != 1:
        print(f"bench.py: expected one JSON line from rank 0, got {len(lines)}", file=sys.stderr)
        return 3
    for ln in lines:
        print(ln, flush=True)
    return p.returncode


def _world_guard(args, world):
    """A scaling run must measure the world it was asked for: --gpus N with WORLD_SIZE != N
    (a launcher that started the wrong number of ranks) fails instead of reporting a number."""
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report", file=sys.stderr)
        sys.exit(2)


def launch_check(args, json_out):
    """--launch-check: the multi-rank plumbing of main() without the workload (CPU, gloo)."""
    import torch
    import torch.distributed as tdist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    _world_guard(args, world)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        tdist.init_process_group("gloo")
        t = torch.tensor([1.0])
        tdist.all_reduce(t)
        assert int(t.item()) == world
    if rank == 0:
        print(json.dumps({"metric": "env-steps/sec (collect+GAE+PPO update), 4096 envs×128 steps @ 1/2/4/8 GPU",
                          "value": None, "unit": "env-steps/s", "n_gpus": world, "launch_check": True,
                          "config": {"parallelism": f"dp{world}" if world > 1 else "single GPU"}}),
              file=json_out, flush=True)
    if world > 1:
        tdist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    # stdout carries the one JSON line only: whatever else writes to fd 1 (RCCL prints its version
    # banner there when a communicator is created) goes to stderr
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    if args.launch_check:
        return launch_check(args, json_out)
    import numpy as np
    import torch
    import torch.distributed as tdist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    _world_guard(args, world)
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
    elif args.force_dist:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
        tdist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", local))
        sys.path.insert(0, os.path.join(ROOT, "ppo-exploration_amd"))
        import dist as _dist
        _dist.DistContext.enabled = property(lambda self: True)  # every world > 1 branch, one rank
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

    # The roofline kernel is picked the way rocprofv3's per-kernel totals rank them: from the
    # TRAINING launches of the first warmup iteration, run on ONE stream (with the backward's
    # weight gradients on a side stream, concurrent launches stretch each other's event
    # durations, so the pick would follow the overlap).  Collect is not timed there: in the
    # timed region it replays as a captured graph whose launches are a small share, while its
    # first, eager pass is host-bound and would inflate the forward kernels' event times.
    # The remaining warmup and the timed region run as configured; the timed region then
    # times the picked kernel on its own stream.
    import convs
    keys = list(KERNELS)
    streams = convs.BWD_STREAMS
    # The second warmup iteration (two streams, as the timed region runs) is event-timed too: its
    # largest kernel is the one rocprofv3's --stats ranks first ("roofline_rocprof"), whose event
    # durations include its sharing of the CUs with the other stream's kernels.
    solo, duo = {}, {}
    # (with --warmup 1 one more untimed iteration runs for the two-stream pick; the line says so)
    n_warm = max(args.warmup, 2 if streams else 1)
    for w in range(n_warm):
        convs.BWD_STREAMS = streams and w > 0
        if w == 0 or (w == 1 and streams):
            alg.collect_samples()
            native.enable_event_timing(keys)
            alg.train()
            times = {k: same_size(k, native.event_times_ms(k)) for k in keys}
            native.enable_event_timing([])
            if w == 0:
                solo = times
            else:
                duo = times
        else:
            iteration()
    convs.BWD_STREAMS = streams
    totals = {k: sum(t for t, _ in v) for k, v in solo.items()}
    duo_tot = {k: sum(t for t, _ in v) for k, v in duo.items()}
    solo_kernel = max(totals, key=totals.get) if any(totals.values()) else "ppox_nature_conv2_wgrad_planes"
    # the headline kernel: the largest in the pass as the timed region runs it (two streams: rocprofv3
    # --stats's ranking over the timed region), the one-stream pick beside it
    prof_kernel = max(duo_tot, key=duo_tot.get) if any(duo_tot.values()) else solo_kernel
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
        "warmup": args.warmup, "untimed_profiling_iterations": n_warm - args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 2), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (Philox uint8 4x84x84 frames, Bernoulli rewards/dones, device envs)",
        "config": {"workload": f"{env_id} {args.algo.upper()} NatureCNN {args.envs} envs x {args.nstep} steps",
                   "n_envs": args.envs, "n_steps": args.nstep, "n_epochs": args.epochs,
                   "batch_size": args.batch_size, "minibatches_per_epoch": -(-args.envs * args.nstep // args.batch_size),
                   "conv_math": conv_impl.math if conv_impl is not None else None,
                   "parallelism": f"dp{world} (env-sharded, {'RCCL' if backend == 'nccl' else backend} grad all-reduce)"
                   if world > 1 else
                   ("dp code paths forced on over a one-rank RCCL communicator" if args.force_dist else "single GPU")},
    }
    # per iteration, rank 0: GPU stream time and host time of each phase (phases.py);
    # gae and episodes run inside collect
    out["phases_ms_per_step"] = phase_ms
    kt = same_size(prof_kernel, kt)
    if kt:
        r = kernel_roofline(prof_kernel, kt)
        r["timing"] = ("HIP events on the kernel's launch stream around its timed-region launches of "
                       f"{r['rows']} rows; a launch beside side-stream kernels (convs.BWD_STREAMS) also counts "
                       "its sharing of the CUs with them")
        r["selection"] = (("largest total kernel time in a two-stream warmup iteration (rocprofv3 --stats's "
                           "ranking over the timed region; collect untimed)") if any(duo_tot.values()) else
                          "largest total kernel time in a one-stream warmup iteration (collect untimed)")
        if solo.get(prof_kernel):
            s_ = kernel_roofline(prof_kernel, solo[prof_kernel])
            r["solo"] = {k: s_[k] for k in ("mean_us", "launches", "rows", "frac", "mfma_frac", "hbm_frac")}
        if any(duo_tot.values()):
            r["share_of_mfma_kernel_time"] = round(duo_tot[prof_kernel] / sum(duo_tot.values()), 3)
        if r.get("traffic") is not None and r["rows"] != PMC_LAUNCH_ROWS:
            # the committed PMC passes ran launches of PMC_LAUNCH_ROWS rows (the 1-GPU workload);
            # a per-launch byte count of another size does not apply here
            r["traffic"] = r["traffic_ratio"] = None
            r["traffic_note"] = (f"PMC traffic was measured on {PMC_LAUNCH_ROWS}-row launches (profiles/); "
                                 f"these launches have {r['rows']} rows")
        out["roofline"] = r
    if solo.get(solo_kernel):
        q = kernel_roofline(solo_kernel, solo[solo_kernel])
        if q["traffic"] is not None and q["rows"] != PMC_LAUNCH_ROWS:
            q["traffic"] = q["traffic_ratio"] = None
        q["selection"] = ("largest total kernel time in a one-stream warmup iteration; mean over that "
                          "iteration's launches, each alone on the GPU")
        out["roofline_solo"] = q
    tot = sum(totals.values())
    if tot:
        top = []
        for k in sorted(totals, key=totals.get, reverse=True)[:5]:
            q = kernel_roofline(k, solo[k])
            if q["traffic"] is not None and q["rows"] != PMC_LAUNCH_ROWS:
                q["traffic"] = q["traffic_ratio"] = None
            top.append({"kernel": q["kernel"], "share_of_mfma_kernel_time": round(totals[k] / tot, 3),
                        "solo_mean_us": q["mean_us"], "rows": q["rows"], "bound": q["bound"], "frac": q["frac"],
                        "mfma_frac": q["mfma_frac"], "hbm_frac": q["hbm_frac"], "pmc_ratio": q["traffic_ratio"]})
        out["roofline_top"] = top
        # every training-pass MFMA kernel's one-stream mean (us) at its most frequent row count
        out["solo_us"] = {KERNELS[k]["label"]: round(float(np.mean([t for t, _ in solo[k]])) * 1e3, 1)
                          for k in sorted(totals, key=totals.get, reverse=True) if solo[k]}
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
        from oracle.baseline import atari_ppo_iteration_rate
        out["cpu_baseline"] = atari_ppo_iteration_rate(args.envs, args.nstep, args.epochs, args.batch_size,
                                                       threads=args.cpu_threads or None)
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    if world > 1 or args.force_dist:
        import dist as _dist
        _dist.shutdown()  # the native communicator first (csrc/dp.cpp), then torch's process group
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
        print(json.dumps(out), file=json_out, flush=True)
    if world > 1:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
