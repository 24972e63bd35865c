"""CPU baseline for bench.py: the oracle's restatement of the reference PPO
iteration (numpy step-major buffer + Python-loop GAE + per-minibatch torch-CPU
autograd and Adam, ppo.py:166-259) timed on the host cores, on a BOUNDED sample
of the benchmark workload: atari_ppo_iteration_rate times one complete iteration
(collect -> GAE -> n_epochs of minibatch updates) end to end at a reduced env count
(bench.py's leg); atari_ppo_rate is the earlier per-phase sample extrapolated per
env-step.

Test infrastructure only (see oracle/__init__.py): imported solely by
bench.py's cpu_baseline leg.  Kind "port" — the reference's Python cannot
travel to the GPU box.
"""
import os
import time

import numpy as np
import torch

from . import models as M
from .algos import OraclePPO
from .philox import SyntheticAtari


def atari_ppo_rate(n_envs, nstep, n_epochs, batch_size, sample_envs=512, sample_steps=64, sample_train=32768,
                   threads=None, budget_s=30.0, seed=0):
    """env-steps/s of the reference algorithm on the CPU for the (n_envs, nstep,
    n_epochs) workload, measured on a bounded sample:
      collect: sample_envs envs x sample_steps steps (NatureCNN act + env + storage)
      GAE:     the Python loop at the FULL (nstep, n_envs) shape
      train:   minibatches covering sample_train rows (fwd + bwd + clip + Adam)
    per env-step time = t_collect/step + t_gae/step + n_epochs * t_train/row."""
    if threads:
        torch.set_num_threads(threads)
    th = torch.get_num_threads()
    t_start = time.time()
    np.random.seed(seed)
    torch.manual_seed(seed)
    env = SyntheticAtari(sample_envs, seed)
    env.observation_space = type("Box", (), {"shape": (4, 84, 84)})()
    env.action_space = type("Discrete", (), {"n": 4})()
    net = M.NatureCNN(4, 4)
    bs = min(batch_size, sample_train)
    alg = OraclePPO(env, nstep=sample_steps, batch_size=bs, n_epochs=1, net=net)
    t0 = time.time()
    alg.collect()
    t_collect = (time.time() - t0) / (sample_envs * sample_steps)
    # GAE at the full shape (pure numpy)
    from .gae import gae_single
    rs = np.random.RandomState(1)
    r = rs.rand(nstep, n_envs).astype(np.float32)
    v = rs.randn(nstep, n_envs).astype(np.float32)
    d = rs.rand(nstep, n_envs) < 1e-3
    t0 = time.time()
    gae_single(r, v, d, v[-1], d[-1], 0.99, 0.95)
    t_gae = (time.time() - t0) / (nstep * n_envs)
    # train rows: restrict the minibatches to sample_train rows
    rows = 0
    t0 = time.time()
    for _idx, mb in alg.rollout.minibatches(bs):
        mbt = {k: torch.tensor(x) for k, x in mb.items()}
        vv, _, lp, ent = M.evaluate(alg.net, mbt["observations"], mbt["actions"])
        from .algos import ppo_loss
        loss, *_ = ppo_loss(vv, lp, ent, mbt, 0.2, 0.01, 1.0)
        alg.opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(alg.net.parameters(), 0.2)
        alg.opt.step()
        rows += mbt["observations"].shape[0]
        if rows >= sample_train or time.time() - t_start > budget_s:
            break
    t_train = (time.time() - t0) / rows
    per_step = t_collect + t_gae + n_epochs * t_train
    return {"value": 1.0 / per_step, "unit": "env-steps/s", "cores": th, "kind": "port",
            "sample": (f"oracle PPO (torch-CPU NatureCNN) on {th} threads: collect {sample_envs} envs x "
                       f"{sample_steps} steps ({t_collect*1e3:.2f} ms/env-step), numpy GAE at {nstep}x{n_envs} "
                       f"({t_gae*1e9:.0f} ns/elem), train {rows} rows in minibatches of {bs} "
                       f"({t_train*1e3:.2f} ms/row/epoch) x {n_epochs} epochs; extrapolated per env-step"),
            "wall_s": round(time.time() - t_start, 1)}


def atari_ppo_iteration_rate(n_envs, nstep, n_epochs, batch_size, sample_envs=64, threads=None, seed=0):
    """env-steps/s of ONE complete reference PPO iteration timed end to end on the CPU: collect
    sample_envs envs x nstep steps (NatureCNN act + env + storage; GAE in the rollout's finish),
    then n_epochs over the sample_envs * nstep rows in minibatches of min(batch_size, rows) (fwd +
    bwd + clip + Adam).  The workload's n_envs are scaled down to sample_envs: the per-env-step cost
    does not depend on the env count, and the minibatch is all the sample's rows when batch_size
    exceeds them."""
    if threads:
        torch.set_num_threads(threads)
    th = torch.get_num_threads()
    np.random.seed(seed)
    torch.manual_seed(seed)
    env = SyntheticAtari(sample_envs, seed)
    env.observation_space = type("Box", (), {"shape": (4, 84, 84)})()
    env.action_space = type("Discrete", (), {"n": 4})()
    rows = sample_envs * nstep
    bs = min(batch_size, rows)
    alg = OraclePPO(env, nstep=nstep, batch_size=bs, n_epochs=n_epochs, net=M.NatureCNN(4, 4))
    t0 = time.time()
    alg.collect()
    t1 = time.time()
    alg.train()
    t2 = time.time()
    return {"value": rows / (t2 - t0), "unit": "env-steps/s", "cores": th, "kind": "port",
            "sample": (f"one complete oracle PPO iteration (torch-CPU NatureCNN) timed end to end on {th} threads: "
                       f"collect {sample_envs} envs x {nstep} steps with GAE ({t1 - t0:.1f} s), {n_epochs} epochs "
                       f"over the {rows} rows in minibatches of {bs} ({t2 - t1:.1f} s); the workload's {n_envs} "
                       f"envs scaled down to {sample_envs} (batch {batch_size} > {rows} rows: one minibatch "
                       f"per epoch)"),
            "wall_s": round(t2 - t0, 1)}


if __name__ == "__main__":
    print(atari_ppo_rate(4096, 128, 10, 16384, threads=int(os.environ.get("THREADS", "0")) or None))
