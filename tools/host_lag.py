"""Host-vs-GPU progress inside one PPO train() (dev tool): at every optimizer step records
the host clock and a GPU event; a host that runs ahead of the GPU shows host time << GPU
time at the same step, a blocking sync shows them equal.  Usage: python tools/host_lag.py [envs] [batch]
[ppo|icm] [dist] ("dist": the data-parallel branches on over a one-rank RCCL communicator, as bench.py
--force-dist)"""
import os
os.environ.setdefault("PPOX_AB", "1")  # this tool switches kernel forms / gates (native.ab_env)
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-exploration_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ppo  # noqa: E402


def main():
    envs = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    bs = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    algo = sys.argv[3] if len(sys.argv) > 3 else "ppo"
    if len(sys.argv) > 4 and sys.argv[4] == "dist":
        import socket
        import torch.distributed as tdist
        import dist
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(sk.getsockname()[1]))
        sk.close()
        torch.cuda.set_device(0)
        tdist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        dist.DistContext.enabled = property(lambda self: True)
    np.random.seed(0)
    torch.manual_seed(0)
    cls = ppo.PPO_ICM if algo == "icm" else ppo.PPO
    alg = cls(env_id="BreakoutNoFrameskip-v4", n_envs=envs, nstep=128, batch_size=bs, n_epochs=10, seed=1, quiet=True)
    marks = []
    orig = alg.flat.adam_step

    def step(*a, **k):
        orig(*a, **k)
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        marks.append((time.perf_counter(), ev))

    alg.flat.adam_step = step
    for it in range(2):
        alg.collect_samples()
        torch.cuda.synchronize()
        marks.clear()
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        alg.train()
        torch.cuda.synchronize()
        n = len(marks)
        for k in sorted({0, 1, n // 4, n // 2, 3 * n // 4, n - 1}):
            h, ev = marks[k]
            print(f"it {it} step {k}: host {1e3 * (h - t0):8.1f} ms  gpu {e0.elapsed_time(ev):8.1f} ms", flush=True)


if __name__ == "__main__":
    main()
