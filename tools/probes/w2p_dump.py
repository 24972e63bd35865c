"""Dump the conv2 weight gradient from H1P planes (native.nature_conv2_wgrad_planes) on seeded inputs, for a
bitwise comparison of two library builds (PPOX_LIB).  Usage: python tools/probes/w2p_dump.py OUT.pt [B]"""
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

B = int(sys.argv[2]) if len(sys.argv) > 2 else 3001
torch.manual_seed(0)
net = models.CnnActorCritic(4, 4)
cv = convs.attach(net, models.FlatParams(net, "cuda"), "split")
x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda")
with torch.no_grad():
    _, h2, h3, am = cv.forward_acts(x, train=True)
h1 = cv.empty_h1(B, "cuda")
cv.fwd(1, x, B, cv.c1.bias, h1, am)
g2 = torch.randn(B, 81, 64, device="cuda") * (torch.rand(B, 81, 64, device="cuda") > 0.5)
amg = native.amax_table(1, "cuda")
native.amax(g2, amg[0])
ws = torch.empty(native.nature_conv2_wgrad_planes_workspace_bytes(B), dtype=torch.uint8, device="cuda")
dw = torch.empty(64, 32, 4, 4, device="cuda")
db = torch.empty(64, device="cuda")
native.nature_conv2_wgrad_planes(h1, cv.q[1], B, g2, ws, dw, db, amax_g=amg[0])
torch.cuda.synchronize()
torch.save({"dw": dw.cpu(), "db": db.cpu()}, sys.argv[1])
print("saved", sys.argv[1], float(dw.abs().max()))
