"""Eager launches vs one captured hipGraph of the same NatureCNN training minibatch (dev tool;
VERDICT r03 item 3: why did the round-3 epoch graph ADD GPU time?).  One minibatch = forward_train +
backward_train (two streams) + clip/Adam on a `B`-row batch of random frames, as PPO.train() runs it.
Prints the GPU time per minibatch (events around N back-to-back minibatches) and the host time to
issue them, for the eager loop and for N replays of one graph captured from the same code.
  python tools/probes/graph_probe.py [B] [N]            both variants, timed
  python tools/probes/graph_probe.py B N eager|graph    one variant only (for rocprofv3 --kernel-trace)"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "ppo-exploration_amd"))
import torch  # noqa: E402

import convs  # noqa: E402
import models  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    only = sys.argv[3] if len(sys.argv) > 3 else None
    torch.manual_seed(0)
    net = models.CnnActorCritic(4, 4)
    flat = models.FlatParams(net, "cuda")
    convs.attach(net, flat, "split")
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda")
    dout = torch.randn(B, 4, device="cuda") * 1e-3
    dv = torch.randn(B, device="cuda") * 1e-3

    def step():
        _, _, _, ctx = net.forward_train(x)
        net.backward_train(ctx, dout, dv)
        flat.adam_step(1e-6, 0.5)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    res = {}

    def timed(fn, name):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        t0 = time.perf_counter()
        for _ in range(N):
            fn()
        host = time.perf_counter() - t0
        e.record()
        torch.cuda.synchronize()
        res[name] = (s.elapsed_time(e) / N, host * 1e3 / N)
        print(f"{name}: {res[name][0] * 1e3:8.1f} us GPU per minibatch, host {res[name][1] * 1e3:8.1f} us", flush=True)

    if only in (None, "eager"):
        timed(step, "eager")
    if only in (None, "graph"):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        g.replay()
        torch.cuda.synchronize()
        timed(g.replay, "graph")


if __name__ == "__main__":
    main()
