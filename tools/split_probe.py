"""Accuracy + speed probe: split-bf16 conv kernels vs the f32-MFMA kernels vs fp64.

Accuracy: max |err| / max |ref| of each kernel against a float64 CPU reference on
a small batch (the f32-MFMA kernel's error is the yardstick: an exact f32 FMA
chain).  Speed: HIP-event time per launch at the training minibatch size.
Usage: python tools/split_probe.py [B] [path/to/libppox variant .so]
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-exploration_amd"))
import native  # noqa: E402

MAC = {1: 400 * 256 * 32, 2: 81 * 512 * 64, 3: 49 * 576 * 64}


def t_ms(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def weights(d):
    g = torch.Generator().manual_seed(0)
    w1 = torch.randn(32, 4, 8, 8, generator=g) * 0.05
    w2 = torch.randn(64, 32, 4, 4, generator=g) * 0.05
    w3 = torch.randn(64, 64, 3, 3, generator=g) * 0.05
    b1, b2, b3 = (torch.randn(c, generator=g) * 0.1 for c in (32, 64, 64))
    return [t.to(d) for t in (w1, w2, w3, b1, b2, b3)]


class Packs:
    def __init__(self, w1, w2, w3, d):
        self.wp = [torch.empty(n, device=d) for n in (256 * 32, 512 * 64, 576 * 64, 4 * 256 * 32, 576 * 64)]
        native.nature_pack_weights(w1, w2, w3, *self.wp)
        self.q = [torch.empty(native.nature_split_pack_elems(k), dtype=torch.int16, device=d) for k in (1, 2, 3, 12, 13)]
        native.nature_pack_split(w1, w2, w3, *self.q)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    if len(sys.argv) > 2:
        native.load(sys.argv[2])
        print(json.dumps({"lib": sys.argv[2]}))
    d = "cuda"
    w1, w2, w3, b1, b2, b3 = weights(d)
    pk = Packs(w1, w2, w3, d)
    # ---- accuracy at a small batch vs float64 CPU
    Bs = 48
    x = torch.randint(0, 256, (Bs, 4, 84, 84), dtype=torch.uint8, device=d)
    ref1 = F.relu(F.conv2d(x.double().cpu(), w1.double().cpu(), b1.double().cpu(), stride=4))  # NCHW
    ref1 = ref1.permute(0, 2, 3, 1).contiguous()
    h_f32 = torch.empty(Bs, 20, 20, 32, device=d)
    h_spl = torch.empty(Bs, 20, 20, 32, device=d)
    native.nature_conv_fwd(1, x, Bs, None, 0, 0, 28224, pk.wp[0], b1, h_f32)
    native.nature_conv_fwd_split(1, x, Bs, None, 0, 0, 28224, pk.q[0], b1, h_spl)
    scale = ref1.abs().max().item()
    for name, h in (("f32_mfma", h_f32), ("split_bf16", h_spl)):
        e = (h.cpu().double() - ref1).abs()
        print(json.dumps({"check": "fwd1", "kernel": name, "max_rel_err": e.max().item() / scale,
                          "mean_rel_err": e.mean().item() / scale}), flush=True)
    # ---- speed at B
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=d)
    h1 = torch.empty(B, 20, 20, 32, device=d)
    for name, fn in (("f32_mfma", lambda: native.nature_conv_fwd(1, x, B, None, 0, 0, 28224, pk.wp[0], b1, h1)),
                     ("split_bf16", lambda: native.nature_conv_fwd_split(1, x, B, None, 0, 0, 28224, pk.q[0], b1,
                                                                        h1))):
        ms = t_ms(fn)
        print(json.dumps({"kernel": name, "layer": 1, "op": "fwd", "B": B, "ms": round(ms, 4),
                          "alg_TF/s": round(2 * B * MAC[1] / ms / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
