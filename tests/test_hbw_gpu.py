"""The heads' backward to the fc output in one launch (csrc/dconv.hip hbw_kernel, round 5:
ppox_head_backward): de = (e > 0) dv w_critic — bitwise ppox_head_dgrad_outer's — and df = (f > 0) (dout W_actor
+ de W_hidden), held to float64 (no larger than twice the error of the same math in f32 and of the two-launch
form ppox_head_dgrad_outer + ppox_head_hidden_dgrad), the amax slots the outputs', bitwise run to run, nothing
written past the rows.  Reference: .ipynb_checkpoints/models-checkpoint.py:72, 80-85 backward (ppo.py:241)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _case(B, A, seed, wc_off=0):
    """wc_off: w_critic at that float offset of a buffer (the flat parameter buffer puts it at 513 A mod 4)"""
    import native
    g = torch.Generator(device="cuda").manual_seed(seed)
    W = torch.randn(512, 512, device="cuda", generator=g) * 0.04
    wa = torch.randn(A, 512, device="cuda", generator=g) * 0.05
    wc = (torch.randn(1, 512 + wc_off, device="cuda", generator=g) * 0.05)[:, wc_off:]
    f = torch.relu(torch.randn(B, 512, device="cuda", generator=g))
    e = torch.relu(torch.randn(B, 512, device="cuda", generator=g))
    dout = torch.randn(B, A, device="cuda", generator=g) * 1e-3
    dv = torch.randn(B, device="cuda", generator=g) * 1e-3
    n = native.head_hidden_pack_elems()
    qf, qd = torch.empty(n, dtype=torch.int16, device="cuda"), torch.empty(n, dtype=torch.int16, device="cuda")
    w1, w2, w3 = torch.randn(32, 4, 8, 8, device="cuda"), torch.randn(64, 32, 4, 4, device="cuda"), \
        torch.randn(64, 64, 3, 3, device="cuda")
    native.nature_pack_all(w1, w2, w3, None, None, None, None, None, None, None, None, None, W, qf, qd)
    return W, wa, wc, f, e, dout, dv, qd


def _fused(B, A, case):
    import native
    W, wa, wc, f, e, dout, dv, qd = case
    df = torch.full((B + 1, 512), 7.0, device="cuda")
    de = torch.full((B + 1, 512), 7.0, device="cuda")
    am = native.amax_table(2, "cuda")
    native.head_backward(dout, wa, dv, wc, e, f, qd, df[:B], de[:B], am[0], am[1])
    torch.cuda.synchronize()
    return df, de, am


@pytest.mark.parametrize("B,A,wc_off", [(1, 4, 0), (31, 4, 0), (33, 4, 0), (2048, 4, 0), (2049, 6, 2), (16384, 4, 0),
                                        (4096, 1, 1), (4096, 8, 0), (600, 3, 3), (600, 7, 3)])
def test_head_backward_vs_fp64(B, A, wc_off):
    """(w_critic misaligned as the flat buffer leaves it for A mod 4 != 0 — read by dwords)"""
    import native
    case = _case(B, A, B * 10 + A, wc_off)
    W, wa, wc, f, e, dout, dv, qd = case
    df, de, am = _fused(B, A, case)
    assert bool((df[B] == 7.0).all()) and bool((de[B] == 7.0).all()), "nothing written past the rows"
    df, de = df[:B], de[:B]
    # the two-launch form
    df2, de2 = native.head_dgrad_outer(dout, wa, dv, wc, e, amax_de=native.amax_table(1, "cuda")[0])
    assert torch.equal(de, de2), "de is head_dgrad_outer's, bitwise"
    native.head_hidden_dgrad(de2, qd, f, df2)
    ref = lambda dt: (dout.to(dt) @ wa.to(dt) + ((e > 0) * dv[:, None] * wc).to(dt) @ W.to(dt)) * (f > 0)
    r64 = ref(torch.float64)
    scale = r64.abs().max()
    err = lambda x: float((x.double() - r64).abs().max() / scale)
    assert err(df) <= 2 * max(err(ref(torch.float32)), err(df2)) + 1e-7, (err(df), err(ref(torch.float32)), err(df2))
    assert float(am[0].cpu().numpy().view(np.float32).max()) == float(de.abs().max())
    assert float(am[1].cpu().numpy().view(np.float32).max()) == float(df.abs().max())
    assert bool(((df != 0) <= (f > 0)).all())


def test_head_backward_is_deterministic():
    case = _case(4096, 4, 5)
    a, b = _fused(4096, 4, case), _fused(4096, 4, case)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
