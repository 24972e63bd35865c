"""The direct conv3 weight gradient (csrc/dconv.hip dwgrad3_kernel, round 5): ppox_nature_conv_wgrad_split(3)
on PX h2 and PX g3 — per sample both images in LDS, the MFMA fragments read straight from them, one partial slab
per workgroup.  Its k order (each sample's 49 pixels in one accumulator per tile, the three split products
together) is not the im2col form's, so it is held to float64: no larger than twice the error of the same op in
f32 and of the im2col split form on the same planes (PPOX_DWGRAD3=0), bitwise run to run.
Reference layer: .ipynb_checkpoints/models-checkpoint.py:57 (Conv2d(64, 64, 3)), trained by ppo.py:241."""
import os

import numpy as np
import pytest
import torch

from test_ddgrad2_gpu import _fp64_check, _planes, _split_exp, _values

pytestmark = pytest.mark.gpu

SIZES = [1, 2, 5, 37, 255, 300, 2048, 9001, 16384]


def _operands(B, seed, scale_g=1.0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    h2 = torch.relu(torch.randn(B, 9, 9, 64, device="cuda", generator=g)) * 3
    g3 = torch.randn(B, 7, 7, 64, device="cuda", generator=g) * torch.rand(B, 7, 7, 64, device="cuda", generator=g)
    g3 = g3 * scale_g
    Eh, Eg = _split_exp(float(h2.abs().max())), _split_exp(float(g3.abs().max()))
    hp, gp = _planes(h2, Eh), _planes(g3, Eg)
    return hp, gp, _values(hp, Eh), _values(gp, Eg), Eh, Eg


def _wgrad(hp, gp, B, Eh, Eg, form):
    import native
    old = os.environ.get("PPOX_DWGRAD3")
    os.environ["PPOX_DWGRAD3"] = "1" if form == "direct" else "0"
    try:
        ws = torch.empty(native.nature_wgrad_split_workspace_bytes(3, B), dtype=torch.uint8, device="cuda")
        dw, db = torch.full((64, 64, 3, 3), 7.0, device="cuda"), torch.full((64,), 7.0, device="cuda")
        eh = torch.tensor([Eh], dtype=torch.int32, device="cuda")
        eg = torch.tensor([Eg], dtype=torch.int32, device="cuda")
        native.nature_conv_wgrad_split(3, hp, B, 0, gp, ws, dw, db, x_exp=eh, g_exp=eg)
        torch.cuda.synchronize()
        return dw, db
    finally:
        if old is None:
            os.environ.pop("PPOX_DWGRAD3", None)
        else:
            os.environ["PPOX_DWGRAD3"] = old


@pytest.mark.parametrize("B", SIZES)
def test_direct_conv3_wgrad_vs_fp64(B):
    hp, gp, h2, g3, Eh, Eg = _operands(B, B)
    dw, db = _wgrad(hp, gp, B, Eh, Eg, "direct")
    dw_i, db_i = _wgrad(hp, gp, B, Eh, Eg, "im2col")
    xn, gn = h2.permute(0, 3, 1, 2), g3.permute(0, 3, 1, 2)
    ref = lambda dt: torch.nn.grad.conv2d_weight(xn.to(dt), (64, 64, 3, 3), gn.to(dt))
    _fp64_check(dw, ref(torch.float64), ref(torch.float32), "direct conv3 wgrad", also=dw_i)
    rb = lambda dt: gn.to(dt).sum((0, 2, 3))
    _fp64_check(db, rb(torch.float64), rb(torch.float32), "direct conv3 bias grad", also=db_i)


@pytest.mark.parametrize("B", [3, 2048])
def test_direct_conv3_wgrad_is_deterministic(B):
    hp, gp, _, _, Eh, Eg = _operands(B, 100 + B)
    a = _wgrad(hp, gp, B, Eh, Eg, "direct")
    b = _wgrad(hp, gp, B, Eh, Eg, "direct")
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


def test_direct_conv3_wgrad_taps_and_pixels():
    """Every tap sees exactly its h2 window: h2 = one-hot pixel images, g3 one nonzero output pixel per
    sample (each of the 49 in turn) — dW3[:, :, ky, kx] is nonzero exactly where the output pixel's tap
    (ky, kx) lands on the hot input pixel, compared elementwise with float64 (tight: every sum has a
    single nonzero term per sample)."""
    B = 49
    h2 = torch.zeros(B, 9, 9, 64, device="cuda")
    g3 = torch.zeros(B, 7, 7, 64, device="cuda")
    for n in range(B):
        oy, ox = divmod(n, 7)
        g3[n, oy, ox] = torch.linspace(0.25, 1.0, 64, device="cuda")
        iy, ix = (n * 5) % 9, (n * 7) % 9
        h2[n, iy, ix] = torch.linspace(1.0, 2.0, 64, device="cuda")
    Eh, Eg = _split_exp(2.0), _split_exp(1.0)
    hp, gp = _planes(h2, Eh), _planes(g3, Eg)
    dw, db = _wgrad(hp, gp, B, Eh, Eg, "direct")
    ref = torch.nn.grad.conv2d_weight(_values(hp, Eh).permute(0, 3, 1, 2).double(), (64, 64, 3, 3),
                                      _values(gp, Eg).permute(0, 3, 1, 2).double())
    assert bool(((dw != 0) <= (ref != 0)).all()), "a nonzero gradient where no pixel pair contributes"
    assert float((dw.double() - ref).abs().max()) <= 1e-6 * float(ref.abs().max())
    assert torch.allclose(db.double(), _values(gp, Eg).double().sum((0, 1, 2)), rtol=1e-6, atol=0)


def test_direct_conv3_wgrad_extreme_exponents():
    """tiny g3 values (exponents far from zero) keep their relative accuracy: the unscale is exact"""
    B = 64
    hp, gp, h2, g3, Eh, Eg = _operands(B, 7, scale_g=1e-20)
    dw, db = _wgrad(hp, gp, B, Eh, Eg, "direct")
    xn, gn = h2.permute(0, 3, 1, 2), g3.permute(0, 3, 1, 2)
    ref = lambda dt: torch.nn.grad.conv2d_weight(xn.to(dt), (64, 64, 3, 3), gn.to(dt))
    _fp64_check(dw, ref(torch.float64), ref(torch.float32), "direct conv3 wgrad (tiny g3)")
    assert float(np.abs(db.cpu().numpy()).max()) < 1e-15
