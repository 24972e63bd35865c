"""What does a fork (event record on the main stream + wait on a side stream) cost the main stream
(dev tool)?  The same chain of N conv2-forward launches at 2,048 rows on one stream, timed with HIP
events, (a) back to back, (b) with an event recorded on the main stream after each launch, (c) with
that event also waited on by an idle side stream (convs.fork), (d) with a join after each launch
(record on the idle side stream, wait on the main stream).  Usage: python tools/probes/event_probe.py [N]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "ppo-exploration_amd"))
import torch  # noqa: E402

import convs  # noqa: E402
import models  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    torch.manual_seed(0)
    net = models.CnnActorCritic(4, 4)
    flat = models.FlatParams(net, "cuda")
    cv = convs.attach(net, flat, "split")
    B = 2048
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda")
    h1, h2, _, am = cv.forward_acts(x, train=True)
    cur = torch.cuda.current_stream()
    side = convs.side_stream(x.device)
    ev = torch.cuda.Event()

    def run(mode):
        for _ in range(N):
            cv.fwd(2, h1, B, cv.c2.bias, h2, am)
            if mode == "record":
                ev.record(cur)
            elif mode == "fork":
                convs.fork(side, cur)
            elif mode == "join":
                convs.join(side, cur)

    for mode in ("plain", "record", "fork", "join", "plain"):
        run(mode)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        run(mode)
        e.record()
        torch.cuda.synchronize()
        print(f"{mode:7s} {s.elapsed_time(e) * 1e3 / N:8.2f} us per launch", flush=True)


if __name__ == "__main__":
    main()
