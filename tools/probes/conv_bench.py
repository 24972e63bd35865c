"""Per-kernel timing of the NatureCNN conv kernels (fwd / dgrad / wgrad) at the
training minibatch size, HIP events on the launch stream, vs algorithmic FLOPs.
Usage: python tools/probes/conv_bench.py [B] [path/to/libppox variant .so]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "ppo-exploration_amd"))
import native  # noqa: E402

PEAK = 157.3
# split-f16: 2.5 PF/s of f16 MFMA / 3 products per f32 MAC (2 for conv1's uint8 frames)
SPLIT_PEAK = {1: 2500 / 2, 2: 2500 / 3, 3: 2500 / 3}
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


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    if len(sys.argv) > 2:
        native.load(sys.argv[2])
        print(json.dumps({"lib": sys.argv[2]}))
    d = "cuda"
    w1, w2, w3 = torch.randn(32, 4, 8, 8, device=d) * 0.05, torch.randn(64, 32, 4, 4, device=d) * 0.05, \
        torch.randn(64, 64, 3, 3, device=d) * 0.05
    b1, b2, b3 = torch.randn(32, device=d), torch.randn(64, device=d), torch.randn(64, device=d)
    wp1, wp2, wp3 = torch.empty(256 * 32, device=d), torch.empty(512 * 64, device=d), torch.empty(576 * 64, device=d)
    wpd2, wpd3 = torch.empty(4 * 256 * 32, device=d), torch.empty(576 * 64, device=d)
    native.nature_pack_weights(w1, w2, w3, wp1, wp2, wp3, wpd2, wpd3)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=d)
    h1 = torch.empty(B, 20, 20, 32, device=d)
    h2 = torch.empty(B, 9, 9, 64, device=d)
    h3 = torch.empty(B, 64, 7, 7, device=d)
    g1, g2, g3 = torch.randn_like(h1), torch.randn(B, 9, 9, 64, device=d), torch.randn(B, 7, 7, 64, device=d)
    dw = {1: torch.empty_like(w1), 2: torch.empty_like(w2), 3: torch.empty_like(w3)}
    db = {1: torch.empty_like(b1), 2: torch.empty_like(b2), 3: torch.empty_like(b3)}
    ws = {k: torch.empty(native.nature_wgrad_workspace_bytes(k, B), dtype=torch.uint8, device=d) for k in (1, 2, 3)}
    lib = native.lib()
    sp = native.stream_ptr()
    res = []

    def rec(name, layer, ms, mac):
        tf = 2 * B * mac / (ms * 1e-3) / 1e12
        peak = SPLIT_PEAK[layer] if "split" in name and not (name == "wgrad_split" and layer > 1) else PEAK
        if name == "wgrad_split":
            peak = SPLIT_PEAK[layer]
        res.append({"kernel": name, "layer": layer, "B": B, "ms": round(ms, 3), "TF/s": round(tf, 1),
                    "frac": round(tf / peak, 3), "peak": round(peak, 1)})
        print(json.dumps(res[-1]), flush=True)

    rec("fwd", 1, t_ms(lambda: native.nature_conv_fwd(1, x, B, None, 0, 0, 28224, wp1, b1, h1)), MAC[1])
    rec("fwd", 2, t_ms(lambda: native.nature_conv_fwd(2, h1, B, None, 0, 0, 0, wp2, b2, h2)), MAC[2])
    rec("fwd", 3, t_ms(lambda: native.nature_conv_fwd(3, h2, B, None, 0, 0, 0, wp3, b3, h3)), MAC[3])
    rec("dgrad", 3, t_ms(lambda: native.nature_conv_dgrad(3, g3, B, wpd3, h2, g2)), MAC[3])
    rec("dgrad", 2, t_ms(lambda: native.nature_conv_dgrad(2, g2, B, wpd2, h1, g1)), MAC[2])
    # split-f16 forms: operand amax rows recorded once (the product's producers record them in
    # their epilogues), so only the kernels are timed
    q = {k: torch.empty(native.nature_split_pack_elems(k), dtype=torch.int16, device=d) for k in (1, 2, 3, 12, 13)}
    native.nature_pack_split(w1, w2, w3, q[1], q[2], q[3], q[12], q[13])
    h3 = torch.empty(B, 7, 7, 64, device=d)
    am = native.amax_table(8, d)
    native.nature_conv_fwd_split(1, x, B, None, 0, 0, 28224, q[1], b1, h1, amax_y=am[0])
    native.nature_conv_fwd_split(2, h1, B, None, 0, 0, 0, q[2], b2, h2, amax_x=am[0], amax_y=am[1])
    for i, t in ((4, g3), (5, g2), (6, g1)):
        native.amax(t, am[i])
    rec("fwd_split", 1, t_ms(lambda: native.nature_conv_fwd_split(1, x, B, None, 0, 0, 28224, q[1], b1, h1)), MAC[1])
    rec("fwd_split", 2, t_ms(lambda: native.nature_conv_fwd_split(2, h1, B, None, 0, 0, 0, q[2], b2, h2,
                                                                  amax_x=am[0])), MAC[2])
    rec("fwd_split", 3, t_ms(lambda: native.nature_conv_fwd_split(3, h2, B, None, 0, 0, 0, q[3], b3, h3,
                                                                  amax_x=am[1])), MAC[3])
    g2o, g1o = torch.empty_like(g2), torch.empty_like(g1)
    rec("dgrad_split", 3, t_ms(lambda: native.nature_conv_dgrad_split(3, g3, B, q[13], h2, g2o, amax_g=am[4])), MAC[3])
    rec("dgrad_split", 2, t_ms(lambda: native.nature_conv_dgrad_split(2, g2, B, q[12], h1, g1o, amax_g=am[5])), MAC[2])
    for L, xin, g, stride, ax, ag in ((3, h2, g3, 0, am[1], am[4]), (2, h1, g2, 0, am[0], am[5]),
                                      (1, x, g1, 28224, None, am[6])):
        wsp = torch.empty(native.nature_wgrad_split_workspace_bytes(L, B), dtype=torch.uint8, device=d)
        rec("wgrad_split", L, t_ms(lambda: native.nature_conv_wgrad_split(L, xin, B, stride, g, wsp, dw[L], db[L],
                                                                          amax_x=ax, amax_g=ag)), MAC[L])
    for L, xin, g, stride in ((3, h2, g3, 0), (2, h1, g2, 0), (1, x, g1, 28224)):
        f = lambda: lib.ppox_nature_conv_wgrad(L, native._p(xin), B, None, 0, 0, stride, native._p(g),
                                               native._p(ws[L]), ws[L].numel(), sp)
        rec("wgrad", L, t_ms(f), MAC[L])
        rec("wgrad_reduce", L, t_ms(lambda: native.call("ppox_nature_wgrad_reduce", L, B, native._p(ws[L]),
                                                        native._p(dw[L]), native._p(db[L]), sp)), 0)
    # library reference (MIOpen) for the same shapes
    xf = x.float()
    import torch.nn.functional as F
    rec("miopen_fwd", 1, t_ms(lambda: F.conv2d(xf, w1, b1, stride=4), 5), MAC[1])
    tot = sum(r["ms"] for r in res if not r["kernel"].startswith("miopen") and "split" not in r["kernel"])
    print(json.dumps({"total_conv_ms_per_minibatch": round(tot, 3)}))


if __name__ == "__main__":
    main()
