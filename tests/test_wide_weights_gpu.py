"""Weights spanning >= 30 binades through the split-f16 training pass.

A weight below 2^-17 of its tensor's largest has a subnormal low f16 plane, below ~2^-28 a subnormal high
plane too.  The split math keeps such a weight to an absolute 2^-25 2^-E (2^-39 of the tensor's
max per value) only while every kernel keeps its planes: a packer, loader or conversion that flushes
subnormal f16 values loses them, and the tests of earlier rounds, whose weights all sat within 17 binades,
could not see that.  (The matrix core itself keeps subnormal x subnormal products: tools/probes/
subnormal_mfma_probe.hip, profiles/r06g/subnormal_probe.txt — so round 5's subnormal-frame conv1 forward,
435f9b3, was exact and passes here.)  tools/build_mutant.sh flushlo1 — conv1's packed weights with their
subnormal low planes zeroed — must fail this file (tools/gpu.sh xfail:flushlo1:test_wide_weights_gpu.py).

Here every weighted layer of the NatureCNN (conv1-3, fc, the heads' hidden layer) gets weights W[o][i] =
randn * e^{N(0,1)} * a[o] * b[i], a and b log-uniform over 17 binades each (so whole output channels — and,
for the dgrads, whole input channels — are 2^-10 .. 2^-34 of the tensor's max), zero biases, and the pass's
outputs are held per element to the f32 dot-product bound plus the split floor, as the weight-gradient tests
(test_kernels_gpu.py test_h1p_conv2_fwd_and_wgrad_vs_fp64):
    |y - y64| <= (2 q + 4) 2^-24 sum_k |x_k||w_k| + 2 * 2^-39 (max|w| sum_k |x_k| + max|x| sum_k |w_k|)
              (+ 2^-24 |y| + 2^-25 2^-E for an output stored as planes at exponent E)
with q the torch f32 computation's own worst multiple of 2^-24 sum |x||w|.  Each op is checked on the inputs
the device consumed (planes decoded exactly), so errors do not compound.  The backward's weight-operand ops
(fc dgrad, conv3 dgrad, conv2 dgrad) and every parameter gradient are held per output channel against a
float64 autograd that applies the pass's own ReLU decisions (tests/f64_pass.py), within 2x the error of the
exact-f32-MFMA kernels (PPOX_CONV_MATH=f32) on the same weights plus the split floor of that channel.
Reference layers: .ipynb_checkpoints/models-checkpoint.py:53-56, 60, 80-85."""
import numpy as np
import pytest
import torch

import f64_pass

pytestmark = pytest.mark.gpu


def _wide(shape, gen, binades=17):
    o, i = shape[0], int(np.prod(shape[1:])) // (shape[2] * shape[3] if len(shape) == 4 else 1)
    a = torch.exp2(-binades * torch.rand(o, generator=gen, dtype=torch.float64))
    b = torch.exp2(-binades * torch.rand(i, generator=gen, dtype=torch.float64))
    a[0], b[0] = 1.0, 1.0  # the tensor's max sits near 1
    s = (a[:, None] * b[None, :])
    if len(shape) == 4:
        s = s[:, :, None, None]
    w = torch.randn(shape, generator=gen, dtype=torch.float64) * torch.exp(torch.randn(shape, generator=gen,
                                                                                         dtype=torch.float64))
    return (w * s * 0.05).float()


def _setup(seed, A=4):
    import convs
    import models
    torch.manual_seed(seed)
    net = models.CnnActorCritic(4, A)
    gen = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for mod in (net.feature_extractor[0], net.feature_extractor[2], net.feature_extractor[4],
                    net.feature_extractor[7], net.extra_layer[0]):
            mod.weight.copy_(_wide(tuple(mod.weight.shape), gen))
            mod.bias.zero_()
    span = np.log2(float(net.feature_extractor[7].weight.abs().max()) /
                   float(net.feature_extractor[7].weight.abs()[net.feature_extractor[7].weight != 0].min()))
    assert span >= 30, span
    ref = models.CnnActorCritic(4, A)
    ref.load_state_dict(net.state_dict())
    flat = models.FlatParams(net, "cuda")
    return net, flat, ref


def _bound_check(y, x64, w64, y32, what, planes_exp=None, relu=True):
    """y (rows, n) device output, x64 (rows, K) the inputs it consumed, w64 (n, K): per element against the
    dot-product bound + the split floor (module docstring)"""
    pre = x64 @ w64.t()
    r64 = pre.relu() if relu else pre
    S = (x64.abs() @ w64.abs().t()) * 2.0 ** -24
    floor = 2.0 ** -39 * (w64.abs().max() * x64.abs().sum(1, keepdim=True) +
                          x64.abs().max() * w64.abs().sum(1)[None, :])
    q = float(((y32.double() - r64).abs() / S.clamp_min(1e-300)).max())
    allow = (2 * q + 4) * S + 2 * floor
    if planes_exp is not None:
        allow = allow + 2.0 ** -24 * r64.abs() + 2.0 ** (-25 - planes_exp)
    excess = (y.double() - r64).abs() - allow
    worst = float(excess.max())
    assert torch.isfinite(y).all(), what
    assert worst <= 0, (what, worst, q)
    return q


def _h1_values(h1p, E):
    return (h1p[..., :32].contiguous().view(torch.float16).double() +
            h1p[..., 32:].contiguous().view(torch.float16).double()) * 2.0 ** -E


def _px_values(p, E):
    x = p.view(torch.float16).reshape(p.shape[:-1] + (p.shape[-1] // 64, 2, 32)).double()
    return ((x[..., 0, :] + x[..., 1, :]) * 2.0 ** -E).reshape(p.shape[:-1] + (p.shape[-1] // 2,))


@pytest.mark.parametrize("B", [37, 600, 8192])
def test_forward_wide_range_weights_per_element(B):
    """conv1 (u8 frames -> H1P), conv2 (H1P -> h2), conv3 (h2 -> h3), the fc layer (h3 -> f) and the heads'
    hidden layer (f -> e), each on the input the device consumed, per element (module docstring)."""
    import convs
    F = torch.nn.functional
    net, flat, _ = _setup(B)
    cv = convs.attach(net, flat, "split")
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda")
    with torch.no_grad():
        h1, h2, h3, am = cv.forward_acts(x, train=True)
        f = cv.fc_forward(h3, am)
        _, _, _, e, _ = net._heads(f, am)
    torch.cuda.synchronize()
    fe = net.feature_extractor
    exps = am[convs.AM_EXP].cpu().numpy()
    unf = lambda t, k, s: F.unfold(t, k, stride=s).transpose(1, 2).reshape(-1, t.shape[1] * k * k)
    # conv1: frames exact; output H1P at the weights' bound exponent
    E1 = cv.h1p_exponent()
    y1 = _h1_values(h1, E1).reshape(-1, 32)
    x1 = unf(x.double(), 8, 4)
    w1 = fe[0].weight.detach().double().reshape(32, -1)
    _bound_check(y1, x1, w1, (unf(x.float(), 8, 4) @ w1.float().t()).relu(), "conv1 fwd", planes_exp=E1)
    # conv2 on the H1P values
    h1v = _h1_values(h1, E1).permute(0, 3, 1, 2)
    y2 = _px_values(h2, int(exps[convs.EX_H2])) if am.px[convs.EX_H2] else h2.double()
    x2 = unf(h1v, 4, 2)
    w2 = fe[2].weight.detach().double().reshape(64, -1)
    _bound_check(y2.reshape(-1, 64), x2, w2, (x2.float() @ w2.float().t()).relu(), "conv2 fwd",
                 planes_exp=int(exps[convs.EX_H2]) if am.px[convs.EX_H2] else None)
    # conv3 on h2 as consumed
    x3 = unf(y2.permute(0, 3, 1, 2), 3, 1)
    w3 = fe[4].weight.detach().double().reshape(64, -1)
    y3 = _px_values(h3, int(exps[convs.EX_H3])) if am.px[convs.EX_H3] else h3.double()
    _bound_check(y3.reshape(-1, 64), x3, w3, (x3.float() @ w3.float().t()).relu(), "conv3 fwd",
                 planes_exp=int(exps[convs.EX_H3]) if am.px[convs.EX_H3] else None)
    # fc on h3 as consumed (NHWC rows; the weight in Flatten order c * 49 + p)
    xf = y3.permute(0, 3, 1, 2).reshape(B, -1)
    wf = fe[7].weight.detach().double()
    _bound_check(f, xf, wf, (xf.float() @ wf.float().t()).relu(), "fc fwd")
    # the heads' hidden layer on f
    wh = net.extra_layer[0].weight.detach().double()
    fd = f.double()
    _bound_check(e, fd, wh, (f @ wh.float().t()).relu(), "hidden fwd")


def _pass(net, flat, x, dout, dv, math):
    import convs
    net.conv_impl = None
    cv = convs.attach(net, flat, math)
    flat.zero_grad()
    out, v, _, ctx = net.forward_train(x)
    net.backward_train(ctx, dout, dv)
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().clone() for n, p in net.named_parameters() if p.requires_grad}
    masks = [m.clone() for m in f64_pass.pass_masks(ctx)]
    return grads, masks, cv


def _fp64_grads(ref, x, dout, dv, masks):
    """float64 autograd of the reference layers with the pass's ReLU decisions (CPU), and per weight element
    the sum of its gradient's terms' magnitudes, S = sum over the reduction of |input| |output grad|, with the
    reduction length K (the scale of an f32 sum's rounding)"""
    F = torch.nn.functional
    fe = ref.feature_extractor
    for p in ref.parameters():
        p.grad = None
    act = lambda z, m: z * m.cpu().double()
    h0 = x.double().cpu()
    z1 = fe[0](h0)
    h1 = act(z1, masks[0])
    z2 = fe[2](h1)
    h2 = act(z2, masks[1])
    z3 = fe[4](h2)
    h3 = act(z3, masks[2]).flatten(1)
    zf = fe[7](h3)
    f = act(zf, masks[3])
    out = ref.actor(f)
    ze = ref.extra_layer[0](f)
    e = act(ze, masks[4])
    v = ref.critic_ext(e).squeeze(-1)
    for z in (z1, z2, z3, zf, ze):
        z.retain_grad()
    ((out * dout.double().cpu()).sum() + (v * dv.double().cpu()).sum()).backward()
    grads = {n: p.grad.clone() for n, p in ref.named_parameters()}
    cw = torch.nn.grad.conv2d_weight
    B = x.shape[0]
    do, dvv = dout.double().cpu().abs(), dv.double().cpu().abs()[:, None]
    mags = {
        "feature_extractor.0.weight": (cw(h0.abs(), fe[0].weight.shape, z1.grad.abs(), stride=4), B * 400),
        "feature_extractor.2.weight": (cw(h1.abs(), fe[2].weight.shape, z2.grad.abs(), stride=2), B * 81),
        "feature_extractor.4.weight": (cw(h2.abs(), fe[4].weight.shape, z3.grad.abs(), stride=1), B * 49),
        "feature_extractor.7.weight": (zf.grad.abs().t() @ h3.abs(), B),
        "extra_layer.0.weight": (ze.grad.abs().t() @ f.abs(), B),
        "actor.0.weight": (do.t() @ f.abs(), B),
        "critic_ext.weight": (dvv.t() @ e.abs(), B),
    }
    return grads, mags


@pytest.mark.parametrize("B", [37, 600])
def test_training_pass_wide_range_weights_per_channel(B):
    """Every parameter gradient of the split training pass (all its dgrads and weight gradients) per output
    channel against float64 with the pass's own ReLU decisions.  A weight gradient element is a sum of K terms
    (K = the batch's pixels), so its f32 rounding scales with sqrt(K) 2^-24 S, S = the sum of the terms'
    magnitudes (computed in float64 with the same decisions): each element within 2x the exact-f32-MFMA pass's
    error of that channel (against float64 with its own decisions) or 4 sqrt(K) 2^-24 S, whichever is larger,
    plus the split floor, 2^-30 of the tensor's largest gradient (the operands' 2^-39 floors carried through the
    chain, with margin), + 1e-6 of the channel's largest entry; a bias (one sum per channel over every pixel,
    with cancellation) within 2x the f32 pass's error + 1e-5 of its largest entry."""
    net, flat, ref = _setup(1000 + B)
    ref = ref.double()
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(B)
    dout = torch.randn(B, 4, device="cuda", generator=g)
    dv = torch.randn(B, device="cuda", generator=g)
    g_s, m_s, cv = _pass(net, flat, x, dout, dv, "split")
    assert cv.math == "split"
    g_f, m_f, _ = _pass(net, flat, x, dout, dv, "f32")
    (r_s, mag), (r_f, _) = _fp64_grads(ref, x, dout, dv, m_s), _fp64_grads(ref, x, dout, dv, m_f)
    for name in r_s:
        rs, rf = r_s[name], r_f[name]
        a, b = g_s[name].cpu().double(), g_f[name].cpu().double()
        if rs.dim() == 1:  # a bias: one sum per channel over every pixel of the batch, with cancellation —
            # held as a tensor, 1e-5 of its largest entry (its terms' magnitudes are not carried here)
            es, ef = float((a - rs).abs().max()), float((b - rf).abs().max())
            assert es <= 2 * ef + 1e-5 * float(rs.abs().max()), (name, es, ef)
            continue
        rows = lambda t: t.reshape(t.shape[0], -1)
        err = rows((a - rs).abs())
        ef = rows((b - rf).abs()).max(1).values
        S, K = mag[name]
        tol = torch.maximum(2 * ef[:, None], 4 * K ** 0.5 * 2.0 ** -24 * rows(S))
        tol = tol + 2.0 ** -30 * float(rs.abs().max()) + 1e-6 * rows(rs.abs()).max(1).values[:, None]
        bad = err > tol
        assert not bool(bad.any()), (name, int(bad.sum()), float((err - tol).max()), float(err.max()),
                                     float(ef.max()), float(rows(S).max()))
