"""Timing of the fc weight gradient on PX df / PX h3: the direct form (csrc/conv.hip fcwg_kernel) against the
split wgrad form (PPOX_FCWG=0), slab reduce included; HIP events on the launch stream, one JSON line per batch.
Usage: python tools/fcwg_bench.py [B ...]"""
import json
import os
os.environ.setdefault("PPOX_AB", "1")  # this tool switches kernel forms / gates (native.ab_env)
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo-exploration_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import native  # noqa: E402
from test_fcwg_gpu import _case  # noqa: E402


def timed(B, form, reps=20):
    dfp, h3p, _, _, e1, e2 = _case(B, 1)
    os.environ["PPOX_FCWG"] = "1" if form == "direct" else "0"
    ws = torch.empty(native.nature_fc_wgrad_workspace_bytes(B), dtype=torch.uint8, device="cuda")
    dw = torch.empty(512, 3136, device="cuda")
    for _ in range(3):
        native.nature_fc_wgrad(dfp, B, h3p, ws, dw, h3_exp=e2, df_exp=e1)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        native.nature_fc_wgrad(dfp, B, h3p, ws, dw, h3_exp=e2, df_exp=e1)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for B in [int(x) for x in sys.argv[1:]] or [2048, 16384]:
    d, sp = timed(B, "direct"), timed(B, "split")
    flops = 2.0 * B * 512 * 3136
    print(json.dumps({"B": B, "direct_us": round(d, 1), "split_us": round(sp, 1),
                      "direct_split_f16_frac": round(flops * 3 / (d * 1e-6) / 2.5e15, 3)}), flush=True)
