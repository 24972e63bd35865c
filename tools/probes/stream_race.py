"""Two-stream vs one-stream backward at ragged per-rank row counts (dev probe, round 6: the 8-rank C4 corruption).

The same training pass (forward_train + backward_train of the NatureCNN actor-critic, split math) is run with the
backward's side stream (convs.BWD_STREAMS) on and off on the same weights and inputs; the gradients must agree
bitwise (the same kernels compute the same values; only the streams differ).  Row counts are drawn from the C4
run's per-rank range (1,990-2,110), the loss-gradient scale from 1e-30 .. 1e2; an Adam step after each pair so the
packing runs every iteration.  Prints one JSON line: pairs, mismatching pairs and, for each, the row count and the
parameters that differ.  Usage: python tools/probes/stream_race.py [PAIRS] [SEED]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "ppo-exploration_amd"))
sys.path.insert(0, ROOT)


def main():
    import convs
    import models
    pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    torch.manual_seed(seed)
    rng = np.random.default_rng(seed)
    net = models.CnnActorCritic(4, 6)
    flat = models.FlatParams(net, "cuda")
    convs.attach(net, flat, "split")
    names = [(n, p) for n, p in net.named_parameters()]
    g = torch.Generator(device="cuda").manual_seed(seed)
    bad = []
    # PPOX_RACE_EXTRA=k: k extra high-priority streams, each given a short matmul every iteration (more hardware
    # queues in use, as gloo's pooled copy streams add in the 8-rank run)
    extra = [torch.cuda.Stream(priority=-1) for _ in range(int(os.environ.get("PPOX_RACE_EXTRA", "0")))]
    ea = torch.randn(512, 512, device="cuda")
    for it in range(pairs):
        for s_ in extra:
            with torch.cuda.stream(s_):
                ea @ ea
        B = int(rng.integers(1990, 2111))
        s = float(10.0 ** rng.uniform(-30, 2))
        x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda", generator=g)
        dout = torch.randn(B, 6, device="cuda", generator=g) * s
        dv = torch.randn(B, device="cuda", generator=g) * s
        got = {}
        for mode in (True, False):
            convs.BWD_STREAMS = mode
            flat.zero_grad()
            _, _, _, ctx = net.forward_train(x)
            net.backward_train(ctx, dout, dv)
            got[mode] = flat.grad.clone()
        convs.BWD_STREAMS = True
        if not torch.equal(got[True], got[False]):
            torch.cuda.synchronize()
            diff = []
            for n, p in names:
                o = (p.data_ptr() - flat.data.data_ptr()) // 4
                a, b = got[True][o:o + p.numel()], got[False][o:o + p.numel()]
                if not torch.equal(a, b):
                    d = float((a - b).abs().max()) if bool(torch.isfinite(a).all()) else float("nan")
                    diff.append([n, d, float(b.abs().max())])
            bad.append({"pair": it, "rows": B, "scale": s, "params": diff})
        flat.grad.copy_(got[True])
        flat.adam_step(2.5e-4, 0.5)
    torch.cuda.synchronize()
    print(json.dumps({"pairs": pairs, "seed": seed, "mismatches": len(bad), "bad": bad[:20]}))


if __name__ == "__main__":
    main()
