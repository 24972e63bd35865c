"""Timing of the conv1 forward writing H1P (fwd1_split_kernel<1, true>, the training pass's form without the
rollout index), HIP events on the launch stream.  Usage: python tools/probes/conv1_bench.py [B ...] (PPOX_LIB: a
variant build)"""
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
        x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda")
        with torch.no_grad():
            h1, _, _, am = cv.forward_acts(x, train=True)
        us = 1e3 * t_ms(lambda: cv.fwd(1, x, B, cv.c1.bias, h1, am))
        byt = B * (28224 + 400 * 128 + 400 * 4)
        torch.cuda.synchronize()
        ck = int((h1.view(torch.int16).to(torch.int64) * torch.arange(1, 65, device="cuda")).sum().item())
        bk = int(am.bits[0].to(torch.int64).sum().item()) if am.bits[0] is not None else 0
        print(json.dumps({"B": B, "conv1_fwd_us": round(us, 1), "TB/s": round(byt / us / 1e6, 2), "h1_checksum": ck,
                          "bits_checksum": bk}), flush=True)


if __name__ == "__main__":
    main()
