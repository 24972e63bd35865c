"""Per-rank row counts through the explicit training pass (dev probe, round 6): for each batch B, one
forward_train + backward_train of a NatureCNN in split math and in exact-f32 math on the same random frames
and upstream grads; prints per parameter tensor the split pass's max |difference| over the f32 pass's max and
any NaN / Inf.  Usage: python tools/probes/rank_rows_sweep.py B [B ...]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "ppo-exploration_amd"))
import convs  # noqa: E402
import models  # noqa: E402


def grads(net, flat, math, x, dout, dv, reps):
    net.conv_impl = None
    convs.attach(net, flat, math)
    outs = []
    for _ in range(reps):
        flat.zero_grad()
        _, _, _, ctx = net.forward_train(x)
        net.backward_train(ctx, dout, dv)
        torch.cuda.synchronize()
        outs.append({n: p.grad.detach().clone() for n, p in net.named_parameters() if p.requires_grad})
    return outs


torch.manual_seed(3)
net = models.CnnActorCritic(4, 4)
flat = models.FlatParams(net, "cuda")
for B in [int(b) for b in sys.argv[1:]]:
    g = torch.Generator(device="cuda").manual_seed(B)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda", generator=g)
    dout = torch.randn(B, 4, device="cuda", generator=g) * 1e-3
    dv = torch.randn(B, device="cuda", generator=g) * 1e-3
    s = grads(net, flat, "split", x, dout, dv, 3)
    f = grads(net, flat, "f32", x, dout, dv, 1)[0]
    rep = {"B": B}
    for n in f:
        a, b = s[0][n], f[n]
        bad = int((~torch.isfinite(a)).sum())
        rel = float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
        same = all(torch.equal(s[0][n], s[k][n]) for k in range(1, len(s)))
        if bad or rel > 1e-3 or not same:
            rep[n] = {"nonfinite": bad, "rel": rel, "repeat_bitwise": same}
    print(json.dumps(rep), flush=True)
