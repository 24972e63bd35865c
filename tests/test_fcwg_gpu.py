"""The fc weight gradient, direct (round 6, csrc/conv.hip fcwg_kernel): dW = df^T h3 on PX df
and PX h3 — 256 outputs x 2 pixels per workgroup over a fifth of the rows, 5 split-K slabs — in Flatten order.
Its k order and tiling are not the split wgrad form's (PPOX_FCWG=0: wgrad_split_kernel<GFc> on the same planes),
so it is held to float64: no larger than twice the error of torch's f32 GEMM and of the split wgrad form on the
same plane values (normwise), per element within the f32 dot-product bound plus the split floor, bitwise run to
run, and the whole gradient written at every batch (ragged and tiny ones included).
Reference layer: .ipynb_checkpoints/models-checkpoint.py:60 Linear(3136, 512), trained by ppo.py:241."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _split_exp(amax):
    e = int(np.float32(amax).view(np.uint32)) >> 23
    return 141 - min(max(e, 15), 254)


def _planes(v, E):
    """PX planes of an f32 tensor (last dim a multiple of 32) at 2^E, and the f32 values they hold"""
    x = v.reshape(-1, v.shape[-1] // 32, 32) * (2.0 ** E)
    h = x.half()
    lo = (x - h.float()).half()
    p = torch.stack([h, lo], dim=2).reshape(v.shape[:-1] + (2 * v.shape[-1],)).view(torch.int16)
    vals = ((h.float() + lo.float()) * 2.0 ** -E).reshape(v.shape)
    return p, vals


def _run(dfp, h3p, B, e_df, e_h3, form):
    import native
    old = os.environ.get("PPOX_FCWG")
    os.environ["PPOX_FCWG"] = "1" if form == "direct" else "0"
    try:
        ws = torch.empty(max(native.nature_fc_wgrad_workspace_bytes(B), 16), dtype=torch.uint8, device="cuda")
        dw = torch.full((512, 3136), float("nan"), device="cuda")
        native.nature_fc_wgrad(dfp, B, h3p, ws, dw, h3_exp=e_h3, df_exp=e_df)
        torch.cuda.synchronize()
        return dw
    finally:
        if old is None:
            os.environ.pop("PPOX_FCWG", None)
        else:
            os.environ["PPOX_FCWG"] = old


def _case(B, seed, wide=False):
    g = torch.Generator(device="cuda").manual_seed(seed)
    df = torch.randn(B, 512, device="cuda", generator=g) * (torch.rand(B, 512, device="cuda", generator=g) > 0.4)
    if wide:
        df = df * torch.exp(3.0 * torch.randn(B, 512, device="cuda", generator=g))
    h3 = torch.relu(torch.randn(B, 7, 7, 64, device="cuda", generator=g))
    E1, E2 = _split_exp(float(df.abs().max()) or 1.0), _split_exp(float(h3.abs().max()) or 1.0)
    dfp, dfv = _planes(df, E1)
    h3p, h3v = _planes(h3, E2)
    e1 = torch.tensor([E1], dtype=torch.int32, device="cuda")
    e2 = torch.tensor([E2], dtype=torch.int32, device="cuda")
    return dfp, h3p, dfv, h3v, e1, e2


@pytest.mark.parametrize("B,wide", [(1, False), (17, False), (300, True), (2048, False), (2049, True),
                                    (16384, False), (16384, True)])
def test_fc_wgrad_direct_vs_fp64(B, wide):
    dfp, h3p, dfv, h3v, e1, e2 = _case(B, B + 3 * wide, wide)
    d1 = _run(dfp, h3p, B, e1, e2, "direct")
    d2 = _run(dfp, h3p, B, e1, e2, "direct")
    ds = _run(dfp, h3p, B, e1, e2, "split")
    assert torch.isfinite(d1).all(), "every element written"
    assert torch.equal(d1, d2), "bitwise run to run"
    if B >= 300:
        assert not torch.equal(d1, ds), "PPOX_FCWG selects the form (a different k order rounds differently)"
    # Flatten order: feature c * 49 + p of the NHWC h3[p][c]
    hf = lambda dt: h3v.to(dt).permute(0, 3, 1, 2).reshape(B, 3136)
    r64 = dfv.double().t() @ hf(torch.float64)
    r32 = dfv.t() @ hf(torch.float32)
    scale = float(r64.abs().max())
    err = lambda x: float((x.double() - r64).abs().max()) / scale
    e_d, e_f, e_s = err(d1), err(r32), err(ds)
    assert e_d <= 2 * max(e_f, e_s) + 1e-7, (e_d, e_f, e_s)
    # per element: the f32 dot-product bound (q: torch f32's own worst multiple of it) + twice the split floor
    S = (dfv.double().abs().t() @ hf(torch.float64).abs()) * 2.0 ** -24
    floor = 2.0 ** -39 * (dfv.double().abs().max() * hf(torch.float64).abs().sum(0)[None, :] +
                          hf(torch.float64).abs().max() * dfv.double().abs().sum(0)[:, None])
    q = float(((r32.double() - r64).abs() / S.clamp_min(1e-300)).max())
    excess = (d1.double() - r64).abs() - (2 * q + 4) * S - 2 * floor
    assert float(excess.max()) <= 0, (float(excess.max()), q)
