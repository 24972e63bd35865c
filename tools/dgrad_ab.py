"""conv2 f32 dgrad of the in-tree libppox vs variant builds (dev tool): bitwise
comparison of the outputs and HIP-event times.  Usage: python tools/dgrad_ab.py B lib1.so [lib2.so ...]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-exploration_amd"))
import native  # noqa: E402


def run(lib, B, w, g, h1):
    native._lib = None
    native.load(lib)
    wp = torch.empty(16 * 64 * 32, device="cuda")
    dummy = [torch.empty(n, device="cuda") for n in (4 * 64 * 32 * 8, 16 * 32 * 64, 9 * 64 * 64)]
    w1, w3 = torch.randn(32, 4, 8, 8, device="cuda"), torch.randn(64, 64, 3, 3, device="cuda")
    native.nature_pack_weights(w1, w, w3, dummy[0], dummy[1], dummy[2], wp, None)
    out = torch.empty(B, 20, 20, 32, device="cuda")
    f = lambda: native.nature_conv_dgrad(2, g, B, wp, h1, out)
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        f()
    e.record()
    torch.cuda.synchronize()
    return out.clone(), s.elapsed_time(e) / 20


def main():
    B = int(sys.argv[1])
    libs = [native.LIB_PATH] + sys.argv[2:]
    torch.manual_seed(0)
    w = torch.randn(64, 32, 4, 4, device="cuda") * 0.05
    g = torch.randn(B, 9, 9, 64, device="cuda")
    h1 = torch.randn(B, 20, 20, 32, device="cuda").relu()
    ref, t0 = run(libs[0], B, w, g, h1)
    print(json.dumps({"lib": "in-tree", "ms": round(t0, 4)}))
    for lib in libs[1:]:
        out, t = run(lib, B, w, g, h1)
        print(json.dumps({"lib": lib, "ms": round(t, 4), "bitwise_equal": bool(torch.equal(out, ref)),
                          "max_abs_diff": float((out - ref).abs().max())}))


if __name__ == "__main__":
    main()
