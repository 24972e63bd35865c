"""Timing of the conv2 / conv3 forwards (H1P / h2 planes -> h2 / h3 planes), the direct form
(csrc/dconv.hip) against the im2col sg2 GEMM (PPOX_DCONV2=0 / PPOX_DCONV3=0), and of the conv2 dgrad: the
direct class-wise form on PX g2 (ddgrad2_kernel) against the col2im form on f32 g2 (dgrad2_colp_kernel),
and of the conv3 weight gradient: direct (dwgrad3_kernel) against im2col (wgrad_split_kernel), slab reduce included;
HIP events on the launch stream.  Usage: python tools/dconv_bench.py [B ...]"""
import json
import os
os.environ.setdefault("PPOX_AB", "1")  # this tool switches kernel forms / gates (native.ab_env)
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-exploration_amd"))
import native  # noqa: E402

if os.environ.get("PPOX_LIB"):
    native.load(os.environ["PPOX_LIB"])
import convs  # noqa: E402
import models  # noqa: E402

convs.PX_MIN_BATCH = 0


def t_ms(fn, iters=20):
    for _ in range(3):
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
    torch.manual_seed(0)
    net = models.CnnActorCritic(4, 4)
    cv = convs.attach(net, models.FlatParams(net, "cuda"), "split")
    for B in [int(a) for a in sys.argv[1:]] or [2048, 16384]:
        x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda")
        with torch.no_grad():
            _, h2, h3, am = cv.forward_acts(x, train=True)
        h1 = cv.empty_h1(B, "cuda")
        cv.fwd(1, x, B, cv.c1.bias, h1, am)
        for layer, xin, y, bias, P, K, pin in ((2, h1, h2, cv.c2.bias, 81, 512, 400 * 32),
                                               (3, h2, h3, cv.c3.bias, 49, 576, 81 * 64)):
            row = {"B": B, "layer": layer}
            for name, v in (("gemm", "0"), ("direct", "1")):
                os.environ["PPOX_DCONV%d" % layer] = v
                row[name + "_us"] = round(1e3 * t_ms(lambda: cv.fwd(layer, xin, B, bias, y, am)), 1)
            flop = 2 * P * K * 64 * B
            byt = B * (pin + P * 64) * 4
            for name in ("gemm", "direct"):
                t = row[name + "_us"] * 1e-6
                row[name + "_tf"] = round(flop / t / 1e12, 1)
                row[name + "_tbs"] = round(byt / t / 1e12, 2)
            print(json.dumps(row), flush=True)
        # conv2 dgrad: g2 (B, 9, 9, 64) -> g1 (B, 20, 20, 32) times conv1's ReLU mask
        g2 = torch.randn(B, 9, 9, 64, device="cuda")
        ag = native.amax_table(2, "cuda")
        native.amax(g2, ag[0])
        g2p = torch.empty(B, 9, 9, 128, dtype=torch.int16, device="cuda")
        e = torch.zeros(1, dtype=torch.int32, device="cuda")
        native.px_split(g2, ag[0], g2p, e)
        bits = am.bits[0]
        g1 = torch.empty(B, 20, 20, 32, device="cuda")
        q = cv.q[12]
        row = {"B": B, "op": "conv2 dgrad",
               "colp_us": round(1e3 * t_ms(lambda: native.nature_conv_dgrad_split(2, g2, B, q, None, g1, amax_g=ag[0],
                                                                                  amax_out=ag[1], relu_bits=bits)), 1),
               "direct_us": round(1e3 * t_ms(lambda: native.nature_conv_dgrad_split(2, g2p, B, q, None, g1, amax_out=ag[1],
                                                                                    relu_bits=bits, g_exp=e)), 1)}
        byt = B * (81 * 64 * 4 + 400 * 32 * 4 + 400 * 4)  # g2 in, g1 out, conv1's bitmask in
        for name in ("colp", "direct"):
            t = row[name + "_us"] * 1e-6
            row[name + "_tbs"] = round(byt / t / 1e12, 2)
            row[name + "_tf"] = round(2 * 81 * 512 * 64 * B / t / 1e12, 1)
        print(json.dumps(row), flush=True)
        # conv3 dgrad on g3 planes: f32 g2 out against PX g2 out (the planes the direct conv2 dgrad reads)
        g3 = torch.randn(B, 7, 7, 64, device="cuda")
        native.amax(g3, ag[0])
        os.environ["PPOX_DDGRAD3_MIN"] = "1"  # (the direct conv3 dgrad at every batch: px_out_us)
        g3p = torch.empty(B, 7, 7, 128, dtype=torch.int16, device="cuda")
        e3 = torch.zeros(1, dtype=torch.int32, device="cuda")
        native.px_split(g3, ag[0], g3p, e3)
        q3 = cv.q[13]
        bits2 = am.bits[1]
        row = {"B": B, "op": "conv3 dgrad",
               "f32_out_us": round(1e3 * t_ms(lambda: native.nature_conv_dgrad_split(
                   3, g3p, B, q3, None, g2, amax_g=ag[0], amax_out=ag[1], relu_bits=bits2, g_exp=e3)), 1),
               "px_out_us": round(1e3 * t_ms(lambda: native.nature_conv_dgrad_split(
                   3, g3p, B, q3, None, g2p, amax_g=ag[0], amax_out=ag[1], relu_bits=bits2, g_exp=e3, y_exp=e)), 1)}
        os.environ["PPOX_DDGRAD3"] = "0"  # the im2col sgemm with the PX output
        row["px_out_sgemm_us"] = round(1e3 * t_ms(lambda: native.nature_conv_dgrad_split(
            3, g3p, B, q3, None, g2p, amax_g=ag[0], amax_out=ag[1], relu_bits=bits2, g_exp=e3, y_exp=e)), 1)
        os.environ.pop("PPOX_DDGRAD3")
        print(json.dumps(row), flush=True)
        # conv3 weight gradient on PX h2 and PX g3: the direct form against the im2col split form
        h2p = torch.empty(B, 9, 9, 128, dtype=torch.int16, device="cuda")
        eh = torch.zeros(1, dtype=torch.int32, device="cuda")
        h2f = torch.relu(torch.randn(B, 9, 9, 64, device="cuda"))
        native.amax(h2f, ag[1])
        native.px_split(h2f, ag[1], h2p, eh)
        ws = torch.empty(native.nature_wgrad_split_workspace_bytes(3, B), dtype=torch.uint8, device="cuda")
        dw, db = torch.empty(64, 64, 3, 3, device="cuda"), torch.empty(64, device="cuda")
        row = {"B": B, "op": "conv3 wgrad"}
        for name, v in (("im2col", "0"), ("direct", "1")):
            os.environ["PPOX_DWGRAD3"] = v
            row[name + "_us"] = round(1e3 * t_ms(lambda: native.nature_conv_wgrad_split(
                3, h2p, B, 0, g3p, ws, dw, db, x_exp=eh, g_exp=e3)), 1)
            t = row[name + "_us"] * 1e-6
            row[name + "_tbs"] = round(B * (81 + 49) * 256 / t / 1e12, 2)
            row[name + "_tf"] = round(2 * 49 * 576 * 64 * B / t / 1e12, 1)
        os.environ.pop("PPOX_DWGRAD3")
        print(json.dumps(row), flush=True)
        # fc forward on PX h3: the 256 x 128 wide-tile form against the sg2 GEMM
        h3f = torch.relu(torch.randn(B, 7, 7, 64, device="cuda"))
        native.amax(h3f, ag[1])
        h3p = torch.empty(B, 7, 7, 128, dtype=torch.int16, device="cuda")
        e3h = torch.zeros(1, dtype=torch.int32, device="cuda")
        native.px_split(h3f, ag[1], h3p, e3h)
        f = torch.empty(B, 512, device="cuda")
        row = {"B": B, "op": "fc fwd"}
        os.environ["PPOX_FCW_MIN"] = "1"
        for name, v in (("sg2", "0"), ("wide", "1")):
            os.environ["PPOX_FCW"] = v
            row[name + "_us"] = round(1e3 * t_ms(lambda: native.nature_fc_fwd(h3p, B, cv.qfc[0], cv.fc.bias, f,
                                                                               amax_f=ag[0], h3_exp=e3h)), 1)
            row[name + "_tf"] = round(2 * 3136 * 512 * B / (row[name + "_us"] * 1e-6) / 1e12, 1)
        os.environ.pop("PPOX_FCW")
        os.environ.pop("PPOX_FCW_MIN")
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
