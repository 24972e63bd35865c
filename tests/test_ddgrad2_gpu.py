"""PX g2 and the direct class-wise conv2 dgrad (round 5).

* The conv3 dgrad writes g2 as its PX planes (ppox_nature_conv_dgrad_split(3, y_exp_out)): the planes
  are the exact split of the f32 dgrad's values at the stored exponent, which comes from the bound
  amax(g3) x the conv3 dgrad matrix's column l1-norms (so it never overflows).
* The direct conv2 dgrad (csrc/dconv.hip ddgrad2_kernel, ppox_nature_conv_dgrad_split(2, g_exp)) sums
  each input pixel's 4 taps x 64 channels in its accumulators (the col2im form adds taps into an LDS
  image): a different k order, so it is held to float64 — no larger than the error of the same op in
  f32 (x2) and than the col2im kernel's on the same g2 values — bitwise run to run, nothing written
  past the batch.
* The conv2 weight gradient reading the planes (ppox_nature_conv2_wgrad_planes(g_exp)) likewise.
Reference layer: .ipynb_checkpoints/models-checkpoint.py:55 (Conv2d(32, 64, 4, stride 2)), trained by
ppo.py:241."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SIZES = [1, 5, 37, 300, 2048, 9001, 16384]


def _packed(seed):
    import native
    g = torch.Generator(device="cuda").manual_seed(seed)
    w1 = torch.randn(32, 4, 8, 8, device="cuda", generator=g) * 0.02
    w2 = torch.randn(64, 32, 4, 4, device="cuda", generator=g) * 0.05
    w3 = torch.randn(64, 64, 3, 3, device="cuda", generator=g) * 0.05
    b1, b2, b3 = (torch.randn(64 if i else 32, device="cuda", generator=g) * 0.1 for i in range(3))
    q = {k: torch.empty(native.nature_split_pack_elems(k), dtype=torch.int16, device="cuda") for k in (1, 2, 3, 12, 13)}
    native.nature_pack_all(w1, w2, w3, None, None, q[1], q[2], q[3], q[12], q[13], None, None, b1=b1, b2=b2, b3=b3)
    return (w1, w2, w3), q


def _planes(v, E):
    """PX planes (int16, last dim doubled) of an f32 tensor whose last dim is a multiple of 32, at 2^E:
    per 32-element group the 32 high f16 then the 32 low f16 (round to nearest, as the kernels)"""
    x = v.reshape(-1, v.shape[-1] // 32, 32) * (2.0 ** E)
    h = x.half()
    lo = (x - h.float()).half()
    return torch.stack([h, lo], dim=2).reshape(v.shape[:-1] + (2 * v.shape[-1],)).view(torch.int16)


def _values(p, E):
    """the f32 values (hi + lo) / 2^E of PX planes"""
    x = p.view(torch.float16).reshape(p.shape[:-1] + (p.shape[-1] // 64, 2, 32)).float()
    return ((x[..., 0, :] + x[..., 1, :]) * (2.0 ** -E)).reshape(p.shape[:-1] + (p.shape[-1] // 2,))


def _split_exp(amax):
    """the split scale exponent of an amax (conv_common.h split_scale_exp)"""
    e = int(np.float32(amax).view(np.uint32)) >> 23
    return 141 - min(max(e, 15), 254)


def _bits(h):
    """ReLU bitmask (one int32 per 32 channels, bit c = channel c > 0) of an NHWC tensor"""
    w = ((h > 0).reshape(-1, 32).long() << torch.arange(32, device=h.device)).sum(1)
    return torch.where(w >= 2 ** 31, w - 2 ** 32, w).to(torch.int32)


def _fp64_check(got, r64, r32, what, also=None):
    """normwise error vs float64 no larger than the same op in f32 (x2 headroom) — and than `also`'s"""
    scale = r64.abs().max()
    e_s = float((got.double() - r64).abs().max() / scale)
    e_f = float((r32.double() - r64).abs().max() / scale)
    e_a = float((also.double() - r64).abs().max() / scale) if also is not None else e_f
    assert torch.isfinite(got).all(), what
    assert e_s <= 2 * max(e_f, e_a) + 1e-7, (what, e_s, e_f, e_a)
    return e_s, e_f, e_a


@pytest.mark.parametrize("B", [1, 37, 2048, 16384])
def test_conv3_dgrad_px_output_is_the_split_of_f32(B):
    import native
    _, q = _packed(B)
    g = torch.Generator(device="cuda").manual_seed(B + 1)
    g3 = torch.randn(B, 7, 7, 64, device="cuda", generator=g) * torch.rand(B, 7, 7, 64, device="cuda", generator=g)
    h2 = torch.relu(torch.randn(B, 9, 9, 64, device="cuda", generator=g))
    bits2 = _bits(h2)
    am = native.amax_table(2, "cuda")
    native.amax(g3, am[0])
    y32 = torch.empty(B, 9, 9, 64, device="cuda")
    native.nature_conv_dgrad_split(3, g3, B, q[13], None, y32, amax_g=am[0], relu_bits=bits2)
    yp = torch.full((B, 9, 9, 128), -1, dtype=torch.int16, device="cuda")
    e = torch.zeros(1, dtype=torch.int32, device="cuda")
    # (f32 g3: the sgemm form; the direct form on PX g3 is tests/test_ddgrad3_gpu.py's)
    native.nature_conv_dgrad_split(3, g3, B, q[13], None, yp, amax_g=am[0], amax_out=am[1], relu_bits=bits2, y_exp=e)
    torch.cuda.synchronize()
    E = int(e.item())
    amax = float(y32.abs().max())
    assert E <= _split_exp(amax)  # the bound is above the true amax: no overflow
    assert torch.equal(yp, _planes(y32, E)), "the planes are the split of the f32 values"
    assert float(am[1].cpu().numpy().view(np.float32).max()) == amax
    assert (y32 != 0).any()


@pytest.mark.parametrize("B", SIZES)
def test_direct_conv2_dgrad_vs_fp64(B):
    import native
    (_, w2, _), q = _packed(B + 7)
    g = torch.Generator(device="cuda").manual_seed(B)
    g2f = torch.randn(B, 9, 9, 64, device="cuda", generator=g) * torch.rand(B, 9, 9, 64, device="cuda", generator=g) ** 2
    E = _split_exp(float(g2f.abs().max()))
    g2p = _planes(g2f, E)
    g2 = _values(g2p, E)  # the f32 values the planes hold
    h1 = torch.relu(torch.randn(B, 20, 20, 32, device="cuda", generator=g))
    bits = _bits(h1)
    e = torch.tensor([E], dtype=torch.int32, device="cuda")
    outs, ams = [], []
    for _ in range(2):
        o = torch.full((B + 1, 20, 20, 32), 7.0, device="cuda")
        am = native.amax_table(1, "cuda")[0]
        native.nature_conv_dgrad_split(2, g2p, B, q[12], None, o, amax_out=am, relu_bits=bits, g_exp=e)
        outs.append(o)
        ams.append(am)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]) and bool((outs[0][B] == 7.0).all())
    got = outs[0][:B]
    assert float(ams[0].cpu().numpy().view(np.float32).max()) == float(got.abs().max())
    colp = torch.empty(B, 20, 20, 32, device="cuda")
    native.nature_conv_dgrad_split(2, g2, B, q[12], None, colp, relu_bits=bits)
    gn, mask = g2.permute(0, 3, 1, 2), (h1.permute(0, 3, 1, 2) > 0)
    ref = lambda dt: (torch.nn.grad.conv2d_input((B, 32, 20, 20), w2.to(dt), gn.to(dt), stride=2) * mask).permute(
        0, 2, 3, 1)
    _fp64_check(got, ref(torch.float64), ref(torch.float32), "direct conv2 dgrad", also=colp)


def test_direct_conv2_dgrad_taps_off_the_image():
    """Every input pixel of a sample gets exactly its taps: a g2 with one nonzero output pixel (each of
    the 81 in turn, all 64 channels) gives g1 = that pixel's 4 x 4 window of W2 and zeros elsewhere —
    the border pixels' missing taps read zeros, no tap reads a neighbouring sample."""
    import native
    (_, w2, _), q = _packed(3)
    B = 81
    g2f = torch.zeros(B, 9, 9, 64, device="cuda")
    for n in range(81):
        g2f[n, n // 9, n % 9] = torch.linspace(0.5, 1.5, 64, device="cuda")
    E = _split_exp(1.5)
    g2p = _planes(g2f, E)
    bits = torch.full((B * 400,), -1, dtype=torch.int32, device="cuda")
    o = torch.empty(B, 20, 20, 32, device="cuda")
    native.nature_conv_dgrad_split(2, g2p, B, q[12], None, o, relu_bits=bits, g_exp=torch.tensor([E], dtype=torch.int32,
                                                                                                   device="cuda"))
    ref = torch.nn.grad.conv2d_input((B, 32, 20, 20), w2.double(), _values(g2p, E).permute(0, 3, 1, 2).double(),
                                     stride=2).permute(0, 2, 3, 1)
    nz = ref.abs() > 0
    assert bool(((o != 0) <= nz).all()), "a nonzero output where no tap contributes"
    assert float((o.double() - ref).abs().max()) <= 1e-6 * float(ref.abs().max())


@pytest.mark.parametrize("B", [1, 37, 2048, 16384])
def test_conv2_wgrad_planes_g2_vs_fp64(B):
    """the conv2 weight gradient reading PX g2: within 2x of f32 math's error against float64 (weights and
    bias), and close to the f32-g2 form on the same values"""
    import native
    _, q = _packed(B + 3)
    tail = q[1][native.nature_split_pack_elems(1) - 2 * native.PACK_TAIL32:].view(torch.int32)
    E1 = int(tail[native.AMAX_SLOTS + 1])
    g = torch.Generator(device="cuda").manual_seed(B)
    h1 = torch.relu(torch.randn(B, 20, 20, 32, device="cuda", generator=g)) * 4
    h1p = _planes(h1, E1)
    h1v = _values(h1p, E1)
    g2f = torch.randn(B, 9, 9, 64, device="cuda", generator=g) * torch.rand(B, 9, 9, 64, device="cuda", generator=g)
    E = _split_exp(float(g2f.abs().max()))
    g2p = _planes(g2f, E)
    g2 = _values(g2p, E)
    ws = torch.empty(native.nature_conv2_wgrad_planes_workspace_bytes(B), dtype=torch.uint8, device="cuda")
    e = torch.tensor([E], dtype=torch.int32, device="cuda")
    dw_p, db_p = torch.empty(64, 32, 4, 4, device="cuda"), torch.empty(64, device="cuda")
    native.nature_conv2_wgrad_planes(h1p, q[1], B, g2p, ws, dw_p, db_p, g_exp=e)
    dw_f, db_f = torch.empty(64, 32, 4, 4, device="cuda"), torch.empty(64, device="cuda")
    native.nature_conv2_wgrad_planes(h1p, q[1], B, g2, ws, dw_f, db_f)
    torch.cuda.synchronize()
    xn, gn = h1v.permute(0, 3, 1, 2), g2.permute(0, 3, 1, 2)
    ref = lambda dt: torch.nn.grad.conv2d_weight(xn.to(dt), (64, 32, 4, 4), gn.to(dt), stride=2)
    _fp64_check(dw_p, ref(torch.float64), ref(torch.float32), "wgrad2 (PX g2)", also=dw_f)
    rb = lambda dt: gn.to(dt).sum((0, 2, 3))
    _fp64_check(db_p, rb(torch.float64), rb(torch.float32), "bias grad (PX g2)", also=db_f)
