"""Collect-phase host vs GPU time (dev tool): wall time of collect_samples(), the host time
to enqueue it, and the summed GPU time between events around each step's work.
Usage: python tools/collect_probe.py [envs]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-exploration_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ppo  # noqa: E402


def main():
    envs = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    np.random.seed(0)
    torch.manual_seed(0)
    alg = ppo.PPO(env_id="BreakoutNoFrameskip-v4", n_envs=envs, nstep=128, batch_size=envs * 4, n_epochs=1, seed=1,
                  quiet=True)
    mark = {}
    orig = alg.rollout.compute_returns_and_advantages

    def gae(*a, **k):  # end of the step loop: host clock + a GPU event
        mark["t"] = time.perf_counter()
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        mark["ev"] = ev
        return orig(*a, **k)

    alg.rollout.compute_returns_and_advantages = gae
    for it in range(3):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        alg.collect_samples()
        t1 = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"it {it}: collect wall {1e3 * (t2 - t0):.1f} ms, host enqueue {1e3 * (t1 - t0):.1f} ms, "
              f"gpu span {e0.elapsed_time(e1):.1f} ms | step loop: host {1e3 * (mark['t'] - t0):.1f} ms, "
              f"gpu {e0.elapsed_time(mark['ev']):.1f} ms", flush=True)
        alg.train()


if __name__ == "__main__":
    main()
