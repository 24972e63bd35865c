"""Split-bf16 conv fwd2 / fwd3 / dgrad3 of the in-tree libppox vs a variant build (dev tool):
bitwise comparison and HIP-event times.  Usage: python tools/split_ab.py B variant.so"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-exploration_amd"))
import native  # noqa: E402


def t_ms(f, iters=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def run(lib, B, ws, xs):
    native._lib = None
    native.load(lib)
    w1, w2, w3 = ws
    h1, h2, g3 = xs
    n = [native.nature_split_pack_elems(L) for L in (1, 2, 3)]
    q = {L: torch.empty(n[L - 1], dtype=torch.int16, device="cuda") for L in (1, 2, 3)}
    qd3 = torch.empty(native.nature_split_pack_elems(13), dtype=torch.int16, device="cuda")
    native.nature_pack_split(w1, w2, w3, q[1], q[2], q[3], None, qd3)
    b2, b3 = torch.zeros(64, device="cuda"), torch.zeros(64, device="cuda")
    y2, y3, d2 = (torch.empty(B, 9, 9, 64, device="cuda"), torch.empty(B, 64, 7, 7, device="cuda"),
                  torch.empty(B, 9, 9, 64, device="cuda"))
    ops = {"fwd2": lambda: native.nature_conv_fwd_split(2, h1, B, None, 0, 0, 0, q[2], b2, y2),
           "fwd3": lambda: native.nature_conv_fwd_split(3, h2, B, None, 0, 0, 0, q[3], b3, y3),
           "dgrad3": lambda: native.nature_conv_dgrad_split(3, g3, B, qd3, h2, d2)}
    res = {k: t_ms(f) for k, f in ops.items()}
    for f in ops.values():
        f()
    torch.cuda.synchronize()
    return res, (y2.clone(), y3.clone(), d2.clone())


def main():
    B, var = int(sys.argv[1]), sys.argv[2]
    torch.manual_seed(0)
    ws = (torch.randn(32, 4, 8, 8, device="cuda") * 0.05, torch.randn(64, 32, 4, 4, device="cuda") * 0.05,
          torch.randn(64, 64, 3, 3, device="cuda") * 0.05)
    xs = (torch.randn(B, 20, 20, 32, device="cuda").relu(), torch.randn(B, 9, 9, 64, device="cuda").relu(),
          torch.randn(B, 7, 7, 64, device="cuda"))
    t0, o0 = run(native.LIB_PATH, B, ws, xs)
    t1, o1 = run(var, B, ws, xs)
    print(json.dumps({"B": B, "in_tree_ms": {k: round(v, 4) for k, v in t0.items()},
                      "variant_ms": {k: round(v, 4) for k, v in t1.items()},
                      "bitwise_equal": [bool(torch.equal(a, b)) for a, b in zip(o0, o1)]}))


if __name__ == "__main__":
    main()
