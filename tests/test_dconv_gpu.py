"""The direct conv2 / conv3 forwards (round 4, csrc/dconv.hip: weights in registers, input images in
LDS) are bitwise the im2col sg2 GEMMs they replace (PPOX_DCONV2=0 / PPOX_DCONV3=0): the same MFMA
sequence per output element, so the output's planes, its ReLU bitmask, its amax slots' maximum and its
exponent must all be equal.  Reference layers: .ipynb_checkpoints/models-checkpoint.py:55-57
(Conv2d(32, 64, 4, stride 2) and Conv2d(64, 64, 3, stride 1), each + ReLU)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _px_at_every_batch(monkeypatch):
    import convs
    monkeypatch.setattr(convs, "PX_MIN_BATCH", 0)
    yield
    os.environ.pop("PPOX_DCONV2", None)
    os.environ.pop("PPOX_DCONV3", None)


def _trunk(seed):
    import convs
    import models
    torch.manual_seed(seed)
    net = models.CnnActorCritic(4, 4)
    flat = models.FlatParams(net, "cuda")
    return convs.attach(net, flat, "split")


def _forward(cv, x, layer, direct):
    import convs
    os.environ["PPOX_DCONV%d" % layer] = "1" if direct else "0"
    with torch.no_grad(), torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        _, h2, h3, am = cv.forward_acts(x, train=True)
        torch.cuda.synchronize()
    names = " ".join(e.name for e in prof.events())
    assert ("DcF%d" % layer in names) == direct, names[:2000]
    assert am.px[0] and am.px[1], am.px  # h2 and h3 ran as planes
    y = h2 if layer == 2 else h3
    amax = am[convs.AM_H1 + layer - 1].cpu().numpy().view(np.uint32).max()
    bits = am.bits[layer - 1]
    return y.clone(), (bits.clone() if bits is not None else None), amax, \
        int(am[convs.AM_EXP].cpu()[convs.EX_H2 + layer - 2])


@pytest.mark.parametrize("layer", [2, 3])
@pytest.mark.parametrize("B", [1, 5, 37, 300, 2048, 9001, 16384])
def test_direct_conv_forward_is_the_gemm_bitwise(B, layer):
    cv = _trunk(B)
    g = torch.Generator(device="cuda").manual_seed(B)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda", generator=g)
    ya, ba, ma, ea = _forward(cv, x, layer, False)
    yb, bb, mb, eb = _forward(cv, x, layer, True)
    assert ea == eb and ma == mb, (ea, eb, ma, mb)
    assert torch.equal(ya, yb), (ya != yb).nonzero()[:8]
    assert (ba is None) == (bb is None)
    if ba is not None:
        assert torch.equal(ba, bb), (ba != bb).nonzero()[:8]
    assert (ya.view(torch.int16) != 0).any()  # not a vacuous comparison


@pytest.mark.parametrize("B", [1, 37, 2048, 9001, 16384])
def test_direct_fc_dgrad_is_the_gemm_bitwise(B):
    """The fc dgrad's direct form (PPOX_DFCD=1, csrc/dconv.hip fcd_kernel: weights in AGPRs, df planes
    streamed through LDS) against the sg2 GEMM on the same df planes: g3's planes, amax and exponent equal.
    Reference: .ipynb_checkpoints/models-checkpoint.py:58-59 (Linear(3136, 512)) backward."""
    import convs
    import native
    cv = _trunk(B)
    cv.pack(B)
    g = torch.Generator(device="cuda").manual_seed(B)
    df = torch.randn(B, 512, device="cuda", generator=g) * torch.rand(B, 512, device="cuda", generator=g) ** 2
    am = native.amax_table(convs.AM_ROWS, "cuda")
    native.amax(df, am[convs.AM_DF])
    e = torch.zeros(1, dtype=torch.int32, device="cuda")
    dfp = torch.empty(B, 1024, dtype=torch.int16, device="cuda")
    native.px_split(df, am[convs.AM_DF], dfp, e)
    bits = torch.randint(-2 ** 31, 2 ** 31 - 1, (B * 98,), dtype=torch.int32, device="cuda", generator=g)
    outs = []
    for direct in (False, True):
        os.environ["PPOX_DFCD"] = "1" if direct else "0"
        g3 = torch.empty(B, 7, 7, 128, dtype=torch.int16, device="cuda")
        ex = torch.zeros(1, dtype=torch.int32, device="cuda")
        amg = native.amax_table(1, "cuda")
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
            native.nature_fc_dgrad(dfp, B, cv.qfc[1], None, g3, amax_df=am[convs.AM_DF], df_exp=e, relu_bits=bits,
                                   g3_exp=ex, amax_g3=amg[0])
            torch.cuda.synchronize()
        names = " ".join(ev.name for ev in prof.events())
        assert ("fcd_kernel" in names) == direct, names[:2000]
        outs.append((g3, int(ex.item()), amg[0].cpu().numpy().view(np.uint32).max()))
    os.environ.pop("PPOX_DFCD", None)
    (ga, ea, ma), (gb, eb, mb) = outs
    assert ea == eb and ma == mb, (ea, eb, ma, mb)
    assert torch.equal(ga, gb), (ga != gb).nonzero()[:8]
    assert (ga != 0).any()
