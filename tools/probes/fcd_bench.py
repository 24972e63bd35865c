"""Timing of the fc dgrad on df planes writing g3 planes: the direct form (PPOX_DFCD=1, csrc/dconv.hip
fcd_kernel) against the sg2 GEMM, HIP events on the launch stream.  Usage: python tools/probes/fcd_bench.py [B ...]"""
import json
import os
os.environ.setdefault("PPOX_AB", "1")  # this tool switches kernel forms / gates (native.ab_env)
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "ppo-exploration_amd"))
import native  # noqa: E402

if os.environ.get("PPOX_LIB"):
    native.load(os.environ["PPOX_LIB"])
import convs  # noqa: E402
import models  # noqa: E402


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
        cv.pack(B)
        df = torch.randn(B, 512, device="cuda")
        am = native.amax_table(convs.AM_ROWS, "cuda")
        native.amax(df, am[convs.AM_DF])
        e = torch.zeros(1, dtype=torch.int32, device="cuda")
        dfp = torch.empty(B, 1024, dtype=torch.int16, device="cuda")
        native.px_split(df, am[convs.AM_DF], dfp, e)
        bits = torch.randint(-2 ** 31, 2 ** 31 - 1, (B * 98,), dtype=torch.int32, device="cuda")
        g3 = torch.empty(B, 7, 7, 128, dtype=torch.int16, device="cuda")
        ex = torch.zeros(1, dtype=torch.int32, device="cuda")
        amg = native.amax_table(1, "cuda")
        row = {"B": B}
        for name, v in (("gemm", "0"), ("direct", "1")):
            os.environ["PPOX_DFCD"] = v
            row[name + "_us"] = round(1e3 * t_ms(lambda: native.nature_fc_dgrad(
                dfp, B, cv.qfc[1], None, g3, amax_df=am[convs.AM_DF], df_exp=e, relu_bits=bits, g3_exp=ex,
                amax_g3=amg[0])), 1)
        print(json.dumps(row), flush=True)

if __name__ == "__main__":
    main()
