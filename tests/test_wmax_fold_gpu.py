"""The weight packing's amax pass folded into the Adam step (round 6; convs.WmaxLink).

ppox_adam_step_wmax must update parameters and moments bitwise as ppox_adam_step and record, per weight tensor,
partials whose maximum is max |w| of the new weights; ppox_nature_pack_all_wmax fed those partials must write
every packed form — planes, exponents, PX norms and bias bounds, the H1P exponent — bitwise as the packing
with its own amax pass (the tails' amax partials, read only by the packer, by their maximum); and a training run through FlatParams.adam_step and the
packing must end on bitwise the same weights with the fold on and off (PPOX_WMAX_FOLD=0).
Reference: ppo.py:241-244 (clip_grad_norm_ + Adam.step), the packing is the product's own (include/ppox.h)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,offs", [(4099, (0, 8, 777, 1001, 3000)), (2_000_003, (3, 70_000, 900_001, 1_200_000, 1_990_000))])
def test_adam_step_wmax_matches_adam_step(n, offs):
    import native
    g = torch.Generator(device="cuda").manual_seed(n)
    p = torch.randn(n, device="cuda", generator=g)
    gr = torch.randn(n, device="cuda", generator=g)
    m = torch.randn(n, device="cuda", generator=g) * 0.1
    v = torch.rand(n, device="cuda", generator=g) * 0.01
    cnts = [min(1000 + 37 * i, n - o) for i, o in enumerate(offs)]
    cnts[2] = 0 if n < 10_000 else cnts[2]  # an empty tensor range
    ranges = torch.tensor(list(offs) + cnts, dtype=torch.int64)
    parts = torch.zeros(native.NORM_PARTIALS, dtype=torch.float64, device="cuda")
    native.grad_sumsq(gr, parts)
    a = [t.clone() for t in (p, gr, m, v)]
    b = [t.clone() for t in (p, gr, m, v)]
    amax = torch.zeros(native.WMAX_TENSORS * native.WMAX_SLOTS, dtype=torch.int32, device="cuda")
    native.adam_step(*a, parts, 0.5, 2.5e-4, 0.9, 0.999, 1e-8, 3)
    native.adam_step_wmax(*b, parts, 0.5, 2.5e-4, 0.9, 0.999, 1e-8, 3, ranges, amax)
    torch.cuda.synchronize()
    for x, y in zip(a, b):
        assert torch.equal(x, y), "params / grads / moments bitwise ppox_adam_step's"
    slots = amax.view(native.WMAX_TENSORS, native.WMAX_SLOTS).cpu().numpy().view(np.uint32)
    for t, (o, c) in enumerate(zip(offs, cnts)):
        want = float(b[0][o:o + c].abs().max()) if c else 0.0
        got = float(np.uint32(slots[t].max()).view(np.float32))
        assert got == want, (t, got, want)


def _net(seed, fold, monkeypatch):
    import convs
    import models
    monkeypatch.setenv("PPOX_WMAX_FOLD", "1" if fold else "0")
    torch.manual_seed(seed)
    net = models.CnnActorCritic(4, 6)
    flat = models.FlatParams(net, "cuda")
    cv = convs.attach(net, flat, "split")
    assert (cv._wmax is not None) == fold and flat.wmax is cv._wmax
    return net, flat, cv


def _packed(cv):
    bufs = [cv.q[k] for k in sorted(cv.q)] + list(cv.qfc) + list(cv.qh) + [cv.wpd2]
    return [b.clone() for b in bufs]


TAIL16 = 2 * (2 * 256 + 8)  # a packed form's tail (PACK_TAIL32 uint32) in int16 elements; its first 256 words are
# the tensor's amax partials, which only the packer reads (as their maximum): the Adam step's partition of the
# weights into slots is not the amax pass's, so they are compared by their maximum


def _same(x, y):
    if x.dtype != torch.int16:
        return torch.equal(x, y)
    t0 = x.numel() - TAIL16
    if not (torch.equal(x[:t0], y[:t0]) and torch.equal(x[t0 + 512:], y[t0 + 512:])):
        return False
    mx = lambda t: int(t[t0:t0 + 512].view(torch.int32).max())  # non-negative float bits: int order
    return mx(x) == mx(y)


def test_pack_from_adam_amax_bitwise(monkeypatch):
    """a step, then the one-launch packing from the step's partials == the packing with its own amax pass"""
    net, flat, cv = _net(5, True, monkeypatch)
    B = 2048
    cv.pack(B)
    flat.grad.copy_(torch.randn_like(flat.grad) * 1e-2)
    flat.adam_step(2.5e-4, 0.5)
    lk = cv._wmax
    assert lk.valid is not None and lk.valid[0][0] == flat.step_count
    idx = lk.valid[1]
    cv.pack(B)  # fold: amax_in = the step's partials
    torch.cuda.synchronize()
    assert lk.nxt == idx ^ 1 and lk.zeroed[idx ^ 1]
    folded = _packed(cv)
    assert int(lk.bufs[idx ^ 1].abs().sum()) == 0, "the next step's buffer zeroed by the packing"
    cv.invalidate()
    cv.pack(B)  # the amax pass (the link invalidated)
    torch.cuda.synchronize()
    own = _packed(cv)
    for i, (x, y) in enumerate(zip(folded, own)):
        assert _same(x, y), f"packed buffer {i} differs"


def test_training_steps_fold_on_off_bitwise(monkeypatch):
    """four optimizer steps of the explicit training pass (forward_train / backward_train / adam_step): the same
    weights bitwise with the fold on and off"""
    B = 600
    g = torch.Generator(device="cuda").manual_seed(11)
    xs = [torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda", generator=g) for _ in range(4)]
    douts = [torch.randn(B, 6, device="cuda", generator=g) * 0.01 for _ in range(4)]
    dvs = [torch.randn(B, device="cuda", generator=g) * 0.01 for _ in range(4)]
    finals = []
    for fold in (True, False):
        net, flat, cv = _net(9, fold, monkeypatch)
        for x, dout, dv in zip(xs, douts, dvs):
            flat.zero_grad()
            _, _, _, ctx = net.forward_train(x)
            net.backward_train(ctx, dout, dv)
            flat.adam_step(2.5e-4, 0.5)
        torch.cuda.synchronize()
        if fold:
            assert cv._wmax.folds >= 3, "the packings of steps 2-4 read the previous step's partials"
        finals.append(flat.data.clone())
    assert torch.equal(finals[0], finals[1])


@pytest.mark.parametrize("how", ["parameter", "flat_view"])
def test_weights_written_after_the_step_pack_with_their_own_amax(monkeypatch, how):
    """weights overwritten in place between the step and the packing (a torch op on the flat buffer or a view of
    it: load_state_dict, teacher forcing in test_c4_gpu.py) must not be packed from the step's stale partials"""
    net, flat, cv = _net(6, True, monkeypatch)
    B = 2048
    cv.pack(B)
    flat.grad.copy_(torch.randn_like(flat.grad) * 1e-2)
    flat.adam_step(2.5e-4, 0.5)
    with torch.no_grad():  # the fc weight's max moves: stale partials would pack wrong
        if how == "parameter":
            net.feature_extractor[7].weight.mul_(3.0)
        else:
            w = net.feature_extractor[7].weight
            o = (w.data_ptr() - flat.data.data_ptr()) // 4
            flat.data[o:o + w.numel()].mul_(3.0)
    folds = cv._wmax.folds
    cv.pack(B)
    torch.cuda.synchronize()
    assert cv._wmax.folds == folds and cv._wmax.valid is None, "a version counter moved: its own amax pass"
    got = _packed(cv)
    cv.invalidate()
    cv.pack(B)
    torch.cuda.synchronize()
    for i, (x, y) in enumerate(zip(got, _packed(cv))):
        assert _same(x, y), f"packed buffer {i} differs"
