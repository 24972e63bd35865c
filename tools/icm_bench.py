"""Per-kernel timing of the K11 ICM kernels at one minibatch (dev tool).
Usage: [PPOX_LIB=variant.so] [ICM_BENCH_RANDOM=1] python tools/icm_bench.py [B]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-exploration_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import icm as icm_native  # noqa: E402
import native  # noqa: E402
from env import Discrete  # noqa: E402
from models import FlatParams, IntrinsicCuriosityModule  # noqa: E402
from util import ActionConverter  # noqa: E402


def t_us(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / iters * 1e3, 1)


B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
K, A = 4 * 84 * 84, 4
torch.manual_seed(0)
m = IntrinsicCuriosityModule(K, ActionConverter(Discrete(A)), 32)
flat = FlatParams(m, "cuda")
nat = icm_native.NativeIcm(m, flat, K)
if os.environ.get("ICM_BENCH_RANDOM"):  # minibatch rows gathered from a rollout twice their size (as in train)
    import convs
    T = 128
    frames = torch.randint(0, 256, (T, 2 * B // T + 1, 4, 84, 84), dtype=torch.uint8, device="cuda")
    x = convs.RolloutRows(frames, torch.randperm(frames.shape[0] * frames.shape[1], device="cuda")[:B])
    xw = frames  # the weight gradient reads the frame rows numbered by rowno
else:
    x = xw = torch.randint(0, 256, (B, K), dtype=torch.uint8, device="cuda")
acts = torch.randint(0, A, (B if xw is x else xw.shape[0] * xw.shape[1],), dtype=torch.int32, device="cuda")
pre1, phi, rowno = nat.encode(x, "mb", rowno=True)
partials = nat._buf("partials", (native.icm_partials_bytes(B, A) // 4,))
g1q = nat._buf("g1q", (native.icm_g1_pack_elems(B),), torch.int16)
dS, dN = torch.empty(B, 32, device="cuda"), torch.empty(B, 32, device="cuda")
acc = torch.zeros(1, dtype=torch.float64, device="cuda")
res = {"B": B}
res["pack_w1"] = t_us(lambda: native.icm_pack_w1(nat.w1.detach(), nat.q))
res["encode"] = t_us(lambda: nat.encode(x, "mb", rowno=True))
res["pair"] = t_us(lambda: native.icm_pair_backward(phi, B, acts, rowno, None, B - 1, B - 1, A, 0.2, nat.seg, dS, dN,
                                                    partials))
res["row"] = t_us(lambda: native.icm_row_backward(dS, dN, None, B, pre1, nat.seg, A, g1q, partials))
res["reduce"] = t_us(lambda: native.icm_grad_reduce(partials, B, B - 1, A, 0.2, B - 1, nat.gseg, acc))
res["wgrad"] = t_us(lambda: native.icm_enc_wgrad(xw, rowno, B, K, g1q, nat.w1_grad))


class One:
    enabled = False


res["minibatch"] = t_us(lambda: nat.train_minibatch(x, acts, None, B, 0.2, One(), acc))
print(json.dumps(res))
