"""Host vs GPU time of one PPO iteration at a given shape (dev tool): wall time of
train(), host time to enqueue it (no sync), and GPU time (events around it).
Usage: python tools/host_overhead.py [envs] [batch]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-exploration_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ppo  # noqa: E402


def main():
    envs = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    bs = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    np.random.seed(0)
    torch.manual_seed(0)
    alg = ppo.PPO(env_id="BreakoutNoFrameskip-v4", n_envs=envs, nstep=128, batch_size=bs, n_epochs=10, seed=1, quiet=True)
    for it in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        alg.collect_samples()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        alg.train()
        t2 = time.perf_counter()
        e.record()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        print(f"it {it}: collect {1e3 * (t1 - t0):.1f} ms | train wall {1e3 * (t3 - t1):.1f} ms, "
              f"host enqueue {1e3 * (t2 - t1):.1f} ms, gpu {s.elapsed_time(e):.1f} ms", flush=True)


if __name__ == "__main__":
    main()
