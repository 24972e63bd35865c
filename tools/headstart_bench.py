"""bench.py with the GPU held back at the start of every train() (dev tool): a spin kernel of
PPOX_HEADSTART_MS (default 150 ms) is queued first, so the host enqueues the minibatches far ahead of
the GPU and a kernel trace of the early minibatches shows the GPU's own schedule — under rocprofv3
the per-launch host cost otherwise makes the host the bound at the per-rank shape, and the trace's
gaps are the profiler's.  Read it with tools/timeline.py TRACE -K (the K-th minibatch from the start).
Usage: rocprofv3 --kernel-trace ... -- python3 tools/headstart_bench.py [bench.py args]"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ppo-exploration_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
import ppo  # noqa: E402

_orig = ppo.PPO.train


def _train(self):
    # ~2.1e9 spin cycles per second (the shader clock under load)
    torch.cuda._sleep(int(float(os.environ.get("PPOX_HEADSTART_MS", "150")) * 2.1e6))
    return _orig(self)


ppo.PPO.train = _train

if __name__ == "__main__":
    bench.main()
