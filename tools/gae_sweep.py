"""K1 GAE roofline sweep: one-stream (17 B/elem) and two-stream (33 B/elem)
kernels over N envs at T = 128, HIP-event timed on the launch stream.  The
config-size launch (N = 4096) is latency-bound (8.9 MB ≈ 1.4 µs of HBM time),
so the HBM roofline claim is made on the large-N points."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-exploration_amd"))
import native  # noqa: E402

HBM_PEAK = 8000.0


def time_ms(fn, iters=20):
    """Kernel time per launch: `iters` launches captured in one graph and replayed, so
    the host's per-launch cost (ctypes + HIP API, ~10 us) is not in the measurement."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    if len(sys.argv) > 1:  # optional libppox variant (tools/build_variant.sh)
        native.load(sys.argv[1])
    T = 128
    rows = []
    for N in (1024, 4096, 16384, 65536, 131072, 262144, 1 << 20, 1 << 21, 1 << 22):
        f = lambda: torch.randn(T, N, device="cuda")
        r, v, ir, iv = f(), f(), f(), f()
        d = (torch.rand(T, N, device="cuda") < 0.01).to(torch.uint8)
        lv, liv = torch.randn(N, device="cuda"), torch.randn(N, device="cuda")
        ld = d[-1].contiguous()
        outs = [torch.empty(T, N, device="cuda") for _ in range(4)]
        ms1 = time_ms(lambda: native.gae(r, v, d, lv, ld, 0.99, 0.95, outs[0], outs[1]))
        ms2 = time_ms(lambda: native.gae_dual(r, v, d, lv, ld, ir, iv, liv, 0.99, 0.99, 0.95, *outs))
        for name, ms, bpe in (("ppox_gae", ms1, 17), ("ppox_gae_dual", ms2, 33)):
            gbs = bpe * T * N / (ms * 1e-3) / 1e9
            rows.append({"kernel": name, "T": T, "N": N, "us": round(ms * 1e3, 2), "GB/s": round(gbs, 1),
                         "frac_of_8TBs": round(gbs / HBM_PEAK, 3)})
            print(json.dumps(rows[-1]), flush=True)
        del r, v, ir, iv, d, outs


if __name__ == "__main__":
    main()
