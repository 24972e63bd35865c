"""PX (round 4): the NatureCNN trunk's split-f16 operands h2, h3 and g3 written as their two f16
planes by their producers (conv2 forward, conv3 forward, fc dgrad) at exponents derived from
bounds, and read as they lie by their consumers (include/ppox.h "PX"); the fc layer's df split
into its planes once (ppox_px_split) for the fc dgrad and weight gradient.  The explicit training
forward / backward with PX on must stay fp32-class: within 2x the error of the same pass with PX
off (f32 operands split in the consumers, the round-3 path pinned by the reference fixtures)
against a float64 CPU autograd of the same network."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _px_at_every_batch(monkeypatch):
    """the PX machinery at every batch size (the product turns it on from convs.PX_MIN_BATCH rows),
    df's planes included (convs.PX_DF, off in the product)"""
    import convs
    monkeypatch.setattr(convs, "PX_MIN_BATCH", 0)
    monkeypatch.setattr(convs, "PX_DF", True)


def _setup(seed, A=4, intrinsic=False):
    import convs
    import models
    torch.manual_seed(seed)
    net = models.CnnActorCritic(4, A, intrinsic=intrinsic)
    ref = models.CnnActorCritic(4, A, intrinsic=intrinsic)
    ref.load_state_dict(net.state_dict())
    flat = models.FlatParams(net, "cuda")
    cv = convs.attach(net, flat, "split")
    return net, ref.double(), flat, cv


def _fp64(ref, x, dout, dv):
    """outputs and parameter gradients of the reference architecture in float64 (CPU autograd)"""
    F = torch.nn.functional
    fe = ref.feature_extractor
    for p in ref.parameters():
        p.grad = None
    h = F.relu(fe[0](x.double().cpu()))
    h = F.relu(fe[2](h))
    h = F.relu(fe[4](h))
    f = F.relu(fe[7](h.flatten(1)))
    out = ref.actor(f)
    v = ref.critic_ext(ref.extra_layer(f)).squeeze(-1)
    ((out * dout.double().cpu()).sum() + (v * dv.double().cpu()).sum()).backward()
    return out.detach(), v.detach(), {n: p.grad.clone() for n, p in ref.named_parameters()}


def _pass(net, flat, cv, x, dout, dv, px, masks=None):
    cv.px = px
    flat.zero_grad()
    out, v, _, ctx = net.forward_train(x)
    am = ctx[-1]
    net.backward_train(ctx, dout, dv)
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().clone() for n, p in net.named_parameters() if p.requires_grad}
    if masks is not None:
        masks.extend(_relu_masks(ctx))
    return out.detach().clone(), v.detach().clone(), grads, am


def _relu_masks(ctx):
    """the pass's own ReLU decisions (CPU bool, NCHW / rows): conv1-3 from the bitmasks its forwards wrote, the
    fc output f and the critic's hidden layer e from their f32 values"""
    x, _, _, _, f, e, _, am = ctx
    B = x.shape[0]

    def unpack(words, P, C, H, W):  # one int32 per 32 channels of a pixel, bit c = channel c > 0
        w = words.view(B, P, C // 32).long() & 0xFFFFFFFF
        bits = (w.unsqueeze(-1) >> torch.arange(32, device=w.device)) & 1
        return bits.reshape(B, H, W, C).permute(0, 3, 1, 2).bool().cpu()

    geo = ((400, 32, 20, 20), (81, 64, 9, 9), (49, 64, 7, 7))
    convm = [unpack(am.bits[i], *geo[i]) if am.bits[i] is not None else None for i in range(3)]
    return convm + [(f > 0).cpu(), (e > 0).cpu()]


def _fp64_masked(ref, x, dout, dv, masks):
    """_fp64 with the device pass's ReLU decisions (masks from _relu_masks): a pre-activation within a few f32
    roundings of 0 may round to the other side on the device; that flips one ReLU and moves the downstream
    gradients by a whole term, which is a sign decision, not the split math's error — so each pass is held
    against float64 with its own masks (a mask of None: the float64 ReLU)"""
    F = torch.nn.functional
    fe = ref.feature_extractor
    for p in ref.parameters():
        p.grad = None
    act = lambda z, m: F.relu(z) if m is None else z * m.double()
    h = act(fe[0](x.double().cpu()), masks[0])
    h = act(fe[2](h), masks[1])
    h = act(fe[4](h), masks[2])
    f = act(fe[7](h.flatten(1)), masks[3])
    out = ref.actor(f)
    v = ref.critic_ext(act(ref.extra_layer[0](f), masks[4])).squeeze(-1)
    ((out * dout.double().cpu()).sum() + (v * dv.double().cpu()).sum()).backward()
    return out.detach(), v.detach(), {n: p.grad.clone() for n, p in ref.named_parameters()}


@pytest.mark.parametrize("B", [37, 600, 2048])
def test_px_training_pass_is_fp32_class(B):
    import convs
    net, ref, flat, cv = _setup(B)
    assert cv.px, "PX is the default in split math"
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(B + 1)
    dout = torch.randn(B, 4, device="cuda", generator=g)
    dv = torch.randn(B, device="cuda", generator=g)
    m_off, m_on = [], []
    o_off, v_off, g_off, _ = _pass(net, flat, cv, x, dout, dv, False, m_off)
    o_on, v_on, g_on, am = _pass(net, flat, cv, x, dout, dv, True, m_on)
    assert am.px == [True, True, True, True, True], am.px  # h2, h3, g3, df, g2 all ran as planes
    # each pass against float64 with its own ReLU decisions (round 5: at 2,048 rows the wide fc forward's
    # rounding put one critic hidden unit of one row on the other side of 0 than the f32-operand pass)
    r_on, r_off = _fp64_masked(ref, x, dout, dv, m_on), _fp64_masked(ref, x, dout, dv, m_off)
    worst = []
    for name, r in list(r_on[2].items()) + [("out", r_on[0]), ("v", r_on[1])]:
        a = o_on if name == "out" else v_on if name == "v" else g_on[name]
        b = o_off if name == "out" else v_off if name == "v" else g_off[name]
        rb = r_off[0] if name == "out" else r_off[1] if name == "v" else r_off[2][name]
        scale = r.abs().max().item() + 1e-30
        e_on = (a.cpu().double() - r).abs().max().item() / scale
        e_off = (b.cpu().double() - rb).abs().max().item() / scale
        worst.append((e_on / max(e_off, 1e-9), name, e_on, e_off))
        assert e_on <= 2 * e_off + 2e-7, (name, e_on, e_off)
    print("PX/off error ratios (worst 3):", sorted(worst, reverse=True)[:3])


@pytest.mark.parametrize("A", [1, 3, 6, 7, 18])
def test_training_pass_any_action_count(A):
    """the training pass through FlatParams at action counts whose flat-buffer offsets leave
    critic_ext.weight off 16 B (513 A mod 4 != 0: Pong / SpaceInvaders have A = 6) — the fused heads' backward
    (A <= 8) reads it by dwords; A = 18 takes the two-launch form.  Every gradient within 2x the error of the
    PX-off pass against float64 with the pass's own ReLU decisions, as test_px_training_pass_is_fp32_class."""
    import models
    B = 300
    net, ref, flat, cv = _setup(100 + A, A=A)
    off = (net.critic_ext.weight.data_ptr() - flat.data.data_ptr()) // 4
    assert off % 4 == (513 * A) % 4
    assert models.HEAD_BWD_FUSED and cv.split_head_bwd(B)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(A)
    dout = torch.randn(B, A, device="cuda", generator=g)
    dv = torch.randn(B, device="cuda", generator=g)
    m_off, m_on = [], []
    o_off, v_off, g_off, _ = _pass(net, flat, cv, x, dout, dv, False, m_off)
    o_on, v_on, g_on, _ = _pass(net, flat, cv, x, dout, dv, True, m_on)
    r_on, r_off = _fp64_masked(ref, x, dout, dv, m_on), _fp64_masked(ref, x, dout, dv, m_off)
    for name, r in r_on[2].items():
        scale = r.abs().max().item() + 1e-30
        e_on = (g_on[name].cpu().double() - r).abs().max().item() / scale
        e_off = (g_off[name].cpu().double() - r_off[2][name]).abs().max().item() / scale
        assert e_on <= 2 * e_off + 2e-7, (name, e_on, e_off)
        assert e_on <= 1e-4, (name, e_on)


@pytest.mark.parametrize("B", [8192, 9001])
def test_px_training_pass_big_batch_matches_f32_operands(B):
    """From 8,192 rows (the sg2 fc forward and the split hidden head): PX on vs off, no fp64 (too
    slow on the CPU at this size) — the two fp32-class passes agree to a few f32 roundings."""
    net, _, flat, cv = _setup(7)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(11)
    dout = torch.randn(B, 4, device="cuda", generator=g)
    dv = torch.randn(B, device="cuda", generator=g)
    o_off, v_off, g_off, _ = _pass(net, flat, cv, x, dout, dv, False)
    o_on, v_on, g_on, am = _pass(net, flat, cv, x, dout, dv, True)
    assert am.px == [True, True, True, True, True], am.px
    for name in g_off:
        a, b = g_on[name], g_off[name]
        scale = b.abs().max().item() + 1e-30
        assert (a - b).abs().max().item() <= 2e-5 * scale, name
    for a, b in ((o_on, o_off), (v_on, v_off)):
        assert (a - b).abs().max().item() <= 1e-5 * (b.abs().max().item() + 1e-30)


def _bound_exp(amax, norm, bmax):
    """conv_common.h bound_exp in numpy f32"""
    b = np.float32(np.float32(amax) * np.float32(norm)) + np.float32(bmax)
    b = np.float32(b * np.float32(1.0 + 1.0 / 1024.0))
    e = int(np.array(b, dtype=np.float32).view(np.uint32)) >> 23
    return 141 - min(254, max(15, e))


def _amax(am_row):
    return float(am_row.cpu().numpy().view(np.uint32).max().view(np.float32))


def _from_planes(p, E):
    """f32 values of a PX tensor (..., 2C) int16: per 32-group hi then lo f16, times 2^-E"""
    q = p.reshape(-1, 64)
    hi = q[:, :32].contiguous().view(torch.float16).float()
    lo = q[:, 32:].contiguous().view(torch.float16).float()
    return ((hi + lo) * 2.0 ** -E).reshape(p.shape[:-1] + (p.shape[-1] // 2,))


@pytest.mark.parametrize("B", [5, 300])
def test_px_exponents_and_planes(B):
    """The exponents are the documented bounds (amax of the input x max column l1-norm of the packed
    weights + max |bias|, 2^-10 margin), every value lies below 2^15 in planes, and h2's planes
    are the split of the same conv2 sums the f32 epilogue writes (|decode - f32| <= 2^-22 |v| +
    the low plane's floor)."""
    import convs
    net, _, flat, cv = _setup(B)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda")
    with torch.no_grad():
        cv.px = False
        _, h2f, h3f, _ = cv.forward_acts(x, train=True)
        cv.px = True
        _, h2p, h3p, am = cv.forward_acts(x, train=True)
    torch.cuda.synchronize()
    exps = am[convs.AM_EXP].cpu().numpy()
    fe = net.feature_extractor
    w2, b2 = fe[2].weight.detach().cpu(), fe[2].bias.detach().cpu()
    w3, b3 = fe[4].weight.detach().cpu(), fe[4].bias.detach().cpu()
    n2 = w2.abs().reshape(64, -1).sum(1).max().item()
    n3 = w3.abs().reshape(64, -1).sum(1).max().item()
    e2 = _bound_exp(_amax(am[convs.AM_H1]), n2, b2.abs().max().item())
    e3 = _bound_exp(_amax(am[convs.AM_H2]), n3, b3.abs().max().item())
    # (the kernel's f32 column sums may differ from torch's in the last bits: the exponent only
    # changes when the bound sits within that of a power of two)
    assert abs(int(exps[convs.EX_H2]) - e2) <= 1, (exps[:3], e2)
    assert abs(int(exps[convs.EX_H3]) - e3) <= 1, (exps[:3], e3)
    E2 = int(exps[convs.EX_H2])
    d2 = _from_planes(h2p, E2)
    floor = 2.0 ** (-25 - E2)
    assert ((d2 - h2f).abs() <= 2.0 ** -22 * h2f.abs() + floor).all()
    assert (h2p.reshape(-1, 64)[:, :32].contiguous().view(torch.float16).float().abs().max() < 2 ** 15).item()
    d3 = _from_planes(h3p, int(exps[convs.EX_H3]))
    assert (d3 - h3f).abs().max().item() <= 1e-5 * h3f.abs().max().item()
    assert _amax(am[convs.AM_H2]) == h2f.abs().max().item()  # the PX producer records its true amax


@pytest.mark.parametrize("B", [64, 2048])
def test_px_df_planes_are_the_consumers_split(B):
    """ppox_px_split writes the planes a split GEMM makes of an f32 operand in registers (same
    exponent, same rounding): hi + lo = df 2^E to the split's 2^-24, and the fc dgrad (g3 f32 and
    PX g3) and the fc weight gradient on the planes are bitwise the same as on f32 df."""
    import convs
    import native
    net, _, flat, cv = _setup(3)
    cv.pack(B)
    g = torch.Generator(device="cuda").manual_seed(B)
    df = torch.randn(B, 512, device="cuda", generator=g) * torch.rand(B, 512, device="cuda", generator=g) ** 4
    am = native.amax_table(convs.AM_ROWS, "cuda")
    native.amax(df, am[convs.AM_DF])
    e = torch.zeros(1, dtype=torch.int32, device="cuda")
    dfp = torch.empty(B, 1024, dtype=torch.int16, device="cuda")
    native.px_split(df, am[convs.AM_DF], dfp, e)
    torch.cuda.synchronize()
    E = int(e.item())
    dec = _from_planes(dfp, E)
    assert ((dec - df).abs() <= 2.0 ** -23 * df.abs() + 2.0 ** (-25 - E)).all()
    amax = df.abs().max().item()
    assert 2 ** 14 <= amax * 2.0 ** E < 2 ** 15
    h3 = torch.relu(torch.randn(B, 7, 7, 64, device="cuda", generator=g))
    a = torch.empty(B, 7, 7, 64, device="cuda")
    b = torch.empty(B, 7, 7, 64, device="cuda")
    native.nature_fc_dgrad(df, B, cv.qfc[1], h3, a, amax_df=am[convs.AM_DF])
    native.nature_fc_dgrad(dfp, B, cv.qfc[1], h3, b, amax_df=am[convs.AM_DF], df_exp=e)
    assert torch.equal(a, b)
    ws = torch.empty(native.nature_fc_wgrad_workspace_bytes(B), dtype=torch.uint8, device="cuda")
    w1 = torch.empty(512, 3136, device="cuda")
    w2 = torch.empty(512, 3136, device="cuda")
    native.nature_fc_wgrad(df, B, h3, ws, w1, amax_df=am[convs.AM_DF])
    native.nature_fc_wgrad(dfp, B, h3, ws, w2, df_exp=e)
    assert torch.equal(w1, w2)


def test_px_output_refuses_a_form_packed_without_bias():
    """q2 / q3 packed by ppox_nature_pack_split (no biases) carry a NaN PX bias bound; an
    entry point asked for a PX output on such a form fails loudly instead of writing NaN activations,
    and the same forms packed by pack_all with their biases are accepted."""
    import native
    torch.manual_seed(5)
    w1 = torch.randn(32, 4, 8, 8, device="cuda") * 0.05
    w2 = torch.randn(64, 32, 4, 4, device="cuda") * 0.05
    w3 = torch.randn(64, 64, 3, 3, device="cuda") * 0.05
    b1, b2, b3 = (torch.randn(c, device="cuda") * 0.1 for c in (32, 64, 64))
    q = {k: torch.empty(native.nature_split_pack_elems(k), dtype=torch.int16, device="cuda") for k in (1, 2, 3)}
    native.nature_pack_split(w1, w2, w3, q[1], q[2], q[3])
    B = 3
    h2p = torch.zeros(B, 9, 9, 64, device="cuda")      # h2 as planes (f32-sized), exponent 0
    x_exp = torch.zeros(1, dtype=torch.int32, device="cuda")
    y = torch.empty(B, 7, 7, 64, device="cuda")
    y_exp = torch.zeros(1, dtype=torch.int32, device="cuda")
    amax = native.amax_table(1, "cuda")[0]
    bits = torch.zeros(B * 98, dtype=torch.int32, device="cuda")
    with pytest.raises(native.NativeError, match="packed with its bias"):
        native.nature_conv_fwd_split(3, h2p, B, None, 0, 0, 0, q[3], b3, y, amax_x=amax, relu_bits=bits,
                                     x_exp=x_exp, y_exp=y_exp)
    torch.cuda.synchronize()
    native.nature_pack_all(w1, w2, w3, None, None, q[1], q[2], q[3], None, None, None, None, b1=b1, b2=b2, b3=b3)
    native.nature_conv_fwd_split(3, h2p, B, None, 0, 0, 0, q[3], b3, y, amax_x=amax, relu_bits=bits,
                                 x_exp=x_exp, y_exp=y_exp)
    torch.cuda.synchronize()
    assert torch.isfinite(y).all()


@pytest.mark.parametrize("B,A", [(1, 4), (300, 6), (2048, 4), (16384, 18)])
def test_head_grads_writes_df_planes_bitwise(B, A):
    """Round 6: the heads' column-reduction pass writes df's PX planes in the same pass (ppox_head_grads
    df_planes) — bitwise ppox_px_split's planes and exponent, and the same head gradients as without them."""
    import native
    g = torch.Generator(device="cuda").manual_seed(B + A)
    f = torch.relu(torch.randn(B, 512, device="cuda", generator=g))
    e = torch.relu(torch.randn(B, 512, device="cuda", generator=g))
    dout = torch.randn(B, A, device="cuda", generator=g)
    dv = torch.randn(B, device="cuda", generator=g)
    de = torch.randn(B, 512, device="cuda", generator=g) * (e > 0)
    df = torch.randn(B, 512, device="cuda", generator=g) * (f > 0) * torch.rand(B, 512, device="cuda", generator=g) ** 3
    am = native.amax_table(1, "cuda")
    native.amax(df, am[0])
    ws = torch.empty(native.head_grads_workspace_bytes(B, 512, A, False), dtype=torch.uint8, device="cuda")

    def run(planes):
        outs = [torch.full((A, 512), float("nan"), device="cuda"), torch.full((A,), float("nan"), device="cuda"),
                torch.full((1, 512), float("nan"), device="cuda"), torch.full((1,), float("nan"), device="cuda"),
                torch.full((512,), float("nan"), device="cuda"), torch.full((512,), float("nan"), device="cuda")]
        p = torch.full((B, 1024), -1, dtype=torch.int16, device="cuda") if planes else None
        ex = torch.zeros(1, dtype=torch.int32, device="cuda") if planes else None
        native.head_grads(f, e, dout, dv.view(B, 1), de, df, ws, *outs, df_planes=p, df_planes_amax=am[0] if planes else None,
                          df_planes_exp=ex)
        torch.cuda.synchronize()
        return outs, p, ex
    o1, p1, e1 = run(True)
    o0, _, _ = run(False)
    for a, b in zip(o1, o0):
        assert torch.equal(a, b)
    p2 = torch.empty(B, 1024, dtype=torch.int16, device="cuda")
    e2 = torch.zeros(1, dtype=torch.int32, device="cuda")
    native.px_split(df, am[0], p2, e2)
    torch.cuda.synchronize()
    assert int(e1) == int(e2) and torch.equal(p1, p2)
