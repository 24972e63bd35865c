"""The direct conv3 dgrad (csrc/dconv.hip ddgrad3_kernel, round 5): ppox_nature_conv_dgrad_split(3) on PX g3
writing PX g2 — each h2 pixel's 9 taps x 64 channels in its accumulators, taps off the 7 x 7 g3 image reading
a zero pixel.  The k order is not the im2col sgemm's (PPOX_DDGRAD3=0), so the values are held to float64: no
larger than twice the error of the same op in f32 and of the sgemm form; the planes' exponent is the same bound
as the sgemm form's (bitwise), the recorded amax is the output's, run to run bitwise, nothing written past
the batch.  Reference layer: .ipynb_checkpoints/models-checkpoint.py:57 (Conv2d(64, 64, 3)), ppo.py:241."""
import os

import numpy as np
import pytest
import torch

from test_ddgrad2_gpu import _bits, _fp64_check, _packed, _planes, _split_exp, _values

pytestmark = pytest.mark.gpu

SIZES = [1, 2, 5, 37, 255, 300, 2048, 9001, 16384]


def _dgrad3(g3p, Eg, B, q13, bits2, am_g3, form):
    import native
    old = os.environ.get("PPOX_DDGRAD3")
    os.environ["PPOX_DDGRAD3"] = "1" if form == "direct" else "0"
    os.environ["PPOX_DDGRAD3_MIN"] = "1"  # (the direct form at every batch here)
    try:
        y = torch.full((B + 1, 9, 9, 128), -7, dtype=torch.int16, device="cuda")
        e = torch.zeros(1, dtype=torch.int32, device="cuda")
        am = native.amax_table(1, "cuda")[0]
        native.nature_conv_dgrad_split(3, g3p, B, q13, None, y, amax_g=am_g3, amax_out=am, relu_bits=bits2,
                                       g_exp=torch.tensor([Eg], dtype=torch.int32, device="cuda"), y_exp=e)
        torch.cuda.synchronize()
        return y, int(e.item()), float(am.cpu().numpy().view(np.float32).max())
    finally:
        os.environ.pop("PPOX_DDGRAD3_MIN", None)
        if old is None:
            os.environ.pop("PPOX_DDGRAD3", None)
        else:
            os.environ["PPOX_DDGRAD3"] = old


def _operands(B, seed):
    import native
    (_, _, w3), q = _packed(seed)
    g = torch.Generator(device="cuda").manual_seed(seed + 1)
    g3f = torch.randn(B, 7, 7, 64, device="cuda", generator=g) * torch.rand(B, 7, 7, 64, device="cuda", generator=g)
    Eg = _split_exp(float(g3f.abs().max()))
    g3p = _planes(g3f, Eg)
    h2 = torch.relu(torch.randn(B, 9, 9, 64, device="cuda", generator=g))
    am_g3 = native.amax_table(1, "cuda")[0]
    native.amax(_values(g3p, Eg).contiguous(), am_g3)
    return w3, q, g3p, Eg, _values(g3p, Eg), h2, _bits(h2), am_g3


@pytest.mark.parametrize("B", SIZES)
def test_direct_conv3_dgrad_vs_fp64(B):
    w3, q, g3p, Eg, g3, h2, bits2, am_g3 = _operands(B, B)
    yd, Ed, amd = _dgrad3(g3p, Eg, B, q[13], bits2, am_g3, "direct")
    ys, Es, ams = _dgrad3(g3p, Eg, B, q[13], bits2, am_g3, "sgemm")
    assert Ed == Es, "the same bound, the same exponent"
    assert bool((yd[B] == -7).all()), "nothing written past the batch"
    got, sg = _values(yd[:B], Ed), _values(ys[:B], Es)
    # the recorded amax is the largest f32 value before its split into planes (hi + lo: within 2^-21)
    assert abs(amd - float(got.abs().max())) <= 2.0 ** -20 * amd
    mask = (h2.permute(0, 3, 1, 2) > 0)
    ref = lambda dt: (torch.nn.grad.conv2d_input((B, 64, 9, 9), w3.to(dt), g3.permute(0, 3, 1, 2).to(dt)) * mask
                      ).permute(0, 2, 3, 1)
    _fp64_check(got, ref(torch.float64), ref(torch.float32), "direct conv3 dgrad", also=sg)
    assert bool(((got != 0) <= (h2 > 0)).all()), "a nonzero gradient under a dead ReLU"


@pytest.mark.parametrize("B", [3, 2048])
def test_direct_conv3_dgrad_is_deterministic(B):
    _, q, g3p, Eg, _, _, bits2, am_g3 = _operands(B, 50 + B)
    a = _dgrad3(g3p, Eg, B, q[13], bits2, am_g3, "direct")
    b = _dgrad3(g3p, Eg, B, q[13], bits2, am_g3, "direct")
    assert torch.equal(a[0], b[0]) and a[1:] == b[1:]


def test_direct_conv3_dgrad_taps_off_the_image():
    """each h2 pixel gets exactly its taps: a g3 with one nonzero output pixel per sample (each of the 49 in
    turn) gives g2 = that pixel's 3 x 3 window of W3 and zeros elsewhere (no tap reads a neighbouring sample)"""
    import native
    (_, _, w3), q = _packed(11)
    B = 49
    g3f = torch.zeros(B, 7, 7, 64, device="cuda")
    for n in range(B):
        g3f[n, n // 7, n % 7] = torch.linspace(0.5, 1.5, 64, device="cuda")
    Eg = _split_exp(1.5)
    g3p = _planes(g3f, Eg)
    am_g3 = native.amax_table(1, "cuda")[0]
    native.amax(_values(g3p, Eg).contiguous(), am_g3)
    bits = torch.full((B * 81 * 2,), -1, dtype=torch.int32, device="cuda")
    y, E, _ = _dgrad3(g3p, Eg, B, q[13], bits, am_g3, "direct")
    got = _values(y[:B], E)
    ref = torch.nn.grad.conv2d_input((B, 64, 9, 9), w3.double(), _values(g3p, Eg).permute(0, 3, 1, 2).double()
                                     ).permute(0, 2, 3, 1)
    assert bool(((got != 0) <= (ref.abs() > 0)).all()), "a nonzero output where no tap contributes"
    assert float((got.double() - ref).abs().max()) <= 1e-6 * float(ref.abs().max())
