"""libppox kernels vs the CPU oracle through the C ABI (GPU box only)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import algos as OA
from oracle import philox as PH
from oracle import rms as RM

pytestmark = pytest.mark.gpu


def dev(a, dtype=None):
    t = torch.as_tensor(np.ascontiguousarray(a))
    return (t.to(dtype) if dtype is not None else t).cuda()


# ----------------------------------------------------------------- K4 loss
def _oracle_loss(logits, values, acts, old_lp, old_v, adv, ret, clip, ent_coef, vf_coef,
                 iv=None, old_iv=None, iadv=None, iret=None, int_vf_coef=0.5, scale=1.0):
    """torch-CPU autograd of ppo.py:216-238 (+ RND terms :431-460)."""
    z = torch.tensor(logits, requires_grad=True)
    v = torch.tensor(values, requires_grad=True)
    d = torch.distributions.Categorical(torch.softmax(z, dim=-1))
    lp = d.log_prob(torch.tensor(acts, dtype=torch.float64).flatten()).unsqueeze(1)
    ent = d.entropy()
    a = OA.normalized(torch.tensor(adv).reshape(-1, 1))
    if iv is not None:
        a = a + OA.normalized(torch.tensor(iadv).reshape(-1, 1))
    pl = OA.surrogate(a, torch.exp(lp - torch.tensor(old_lp).reshape(-1, 1)), clip)
    vl = OA.clipped_value_loss(torch.tensor(ret), v, torch.tensor(old_v), clip)
    el = -torch.mean(ent)
    loss = pl + ent_coef * el + vf_coef * vl
    ivt = None
    if iv is not None:
        ivt = torch.tensor(iv, requires_grad=True)
        ivl = OA.clipped_value_loss(torch.tensor(iret), ivt, torch.tensor(old_iv), clip)
        loss = loss + int_vf_coef * ivl
    (scale * loss).backward()
    out = {"dz": z.grad.numpy(), "dv": v.grad.numpy(), "pl": pl.item(), "vl": vl.item(), "el": el.item(),
           "loss": loss.item()}
    if ivt is not None:
        out["div"] = ivt.grad.numpy()
        out["ivl"] = ivl.item()
    return out


@pytest.mark.parametrize("A,B,dual,sat", [(4, 333, False, False), (2, 64, False, True), (18, 1000, False, False),
                                          (4, 517, True, False), (6, 2048, True, True)])
def test_ppo_loss_fwd_bwd_vs_torch(A, B, dual, sat):
    import native
    rs = np.random.RandomState(A * 1000 + B)
    T, N = 32, 64
    total = T * N
    clip, ent_coef, vf_coef, ivf = 0.2, 0.01, 0.5, 0.5
    roll = {"actions": rs.randint(0, A, (T, N)).astype(np.int32),
            "log_probs": (np.log(rs.dirichlet(np.ones(A), (T, N))).max(-1) - rs.rand(T, N)).astype(np.float32),
            "values": rs.randn(T, N).astype(np.float32), "advantages": rs.randn(T, N).astype(np.float32) * 2,
            "returns": rs.randn(T, N).astype(np.float32), "int_values": rs.randn(T, N).astype(np.float32),
            "int_advantages": rs.randn(T, N).astype(np.float32), "int_returns": rs.randn(T, N).astype(np.float32)}
    perm = rs.permutation(total)[:B]
    t_of, n_of = perm % T, perm // T
    logits = rs.randn(B, A).astype(np.float32) * (40.0 if sat else 1.5)
    values = (roll["values"][t_of, n_of] + rs.randn(B).astype(np.float32) * 0.3).astype(np.float32)
    ivals = (roll["int_values"][t_of, n_of] + rs.randn(B).astype(np.float32) * 0.3).astype(np.float32)
    g = {k: v[t_of, n_of] for k, v in roll.items()}
    ref = _oracle_loss(logits, values, g["actions"], g["log_probs"], g["values"], g["advantages"], g["returns"], clip,
                       ent_coef, vf_coef, ivals if dual else None, g["int_values"], g["int_advantages"],
                       g["int_returns"], ivf, scale=0.7)
    droll = {k: dev(v) for k, v in roll.items()}
    idx = dev(perm.astype(np.int64))
    stats = torch.empty(1, 4, dtype=torch.float64, device="cuda")
    native.minibatch_adv_stats(droll["advantages"], droll["int_advantages"] if dual else None, idx, B, B, T, N, stats)
    partials = torch.zeros(native.LOSS_PARTIALS * 8, dtype=torch.float64, device="cuda")
    accum = torch.zeros(8, dtype=torch.float64, device="cuda")
    z, v, iv = dev(logits), dev(values), dev(ivals) if dual else None
    native.ppo_loss_partials(z, v, iv, B, A, idx, T, N, droll, stats[0], clip, partials)
    dz, dv = torch.empty_like(z), torch.empty_like(v)
    div = torch.empty_like(iv) if dual else None
    native.ppo_loss_backward(z, v, iv, B, A, idx, T, N, droll, stats[0], clip, partials, B, ent_coef, vf_coef, ivf,
                             0.7, dz, dv, div, accum)
    torch.cuda.synchronize()
    acc = accum.cpu().numpy()
    np.testing.assert_allclose(acc[0], ref["pl"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(acc[1], ref["vl"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(acc[2], ref["el"], rtol=1e-5, atol=1e-7)
    scale_g = max(np.abs(ref["dz"]).max(), 1e-30)
    np.testing.assert_allclose(dz.cpu().numpy(), ref["dz"], rtol=1e-4, atol=1e-5 * scale_g)
    np.testing.assert_allclose(dv.cpu().numpy(), ref["dv"], rtol=1e-5, atol=1e-8)
    if dual:
        np.testing.assert_allclose(acc[4], ref["ivl"], rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(div.cpu().numpy(), ref["div"], rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("D,B,dual", [(2, 512, False), (3, 777, True), (6, 2048, False), (1, 1, False)])
def test_box_loss_fwd_bwd_vs_torch(D, B, dual):
    """Normal head (models.py:66-71) + per-dimension surrogate (ppo.py:216-238) vs torch-CPU
    autograd with the reference's dtypes: f64 actions (buffer.py:156) => f64 log_prob, ratio,
    surrogate; f32 entropy / values.  Tolerance: 1e-5 rel on losses, 1e-4 rel on grads."""
    import native
    rs = np.random.RandomState(D * 1000 + B)
    T, N = 32, 64
    clip, ent_coef, vf_coef, ivf, scale = 0.2, 0.01, 0.5, 0.5, 0.7
    roll = {"actions": (np.tanh(rs.randn(T, N, D)) + 0.5 * rs.randn(T, N, D)).astype(np.float32),
            "log_probs": (-1.0 - 0.5 * rs.rand(T, N, D)).astype(np.float32),
            "values": rs.randn(T, N).astype(np.float32), "advantages": rs.randn(T, N).astype(np.float32) * 2,
            "returns": rs.randn(T, N).astype(np.float32), "int_values": rs.randn(T, N).astype(np.float32),
            "int_advantages": rs.randn(T, N).astype(np.float32), "int_returns": rs.randn(T, N).astype(np.float32)}
    perm = rs.permutation(T * N)[:B]
    t_of, n_of = perm % T, perm // T
    g = {k: v[t_of, n_of] for k, v in roll.items()}
    mu = rs.randn(B, D).astype(np.float32)
    log_std = (0.3 * rs.randn(D)).astype(np.float32)
    values = (g["values"] + rs.randn(B).astype(np.float32) * 0.3).astype(np.float32)
    ivals = (g["int_values"] + rs.randn(B).astype(np.float32) * 0.3).astype(np.float32)
    # torch reference, op by op as the reference builds it
    mu_t = torch.tensor(mu, requires_grad=True)
    ls_t = torch.tensor(log_std.reshape(1, D), requires_grad=True)
    v_t = torch.tensor(values, requires_grad=True)
    iv_t = torch.tensor(ivals, requires_grad=True)
    mean = mu_t.tanh()
    dist = torch.distributions.Normal(mean, torch.exp(ls_t.expand_as(mean)))
    lp = dist.log_prob(torch.tensor(g["actions"]).double())
    assert lp.dtype == torch.float64

    def norm(x):
        x = torch.tensor(x).unsqueeze(1)
        return (x - x.mean()) / (x.std() + 1e-8)
    adv = norm(g["advantages"]) + (norm(g["int_advantages"]) if dual else 0)
    ratio = torch.exp(lp - torch.tensor(g["log_probs"]))
    pl = -torch.min(adv * ratio, adv * torch.clamp(ratio, 1 - clip, 1 + clip)).mean()

    def vloss(v, ov, ret):
        ov, ret = torch.tensor(ov), torch.tensor(ret)
        vc = ov + (v - ov).clamp(-clip, clip)
        return torch.max(F.mse_loss(ret, v), F.mse_loss(ret, vc))
    vl = vloss(v_t, g["values"], g["returns"])
    el = -torch.mean(dist.entropy())
    loss = pl + ent_coef * el + vf_coef * vl
    if dual:
        ivl = vloss(iv_t, g["int_values"], g["int_returns"])
        loss = loss + ivf * ivl
    (scale * loss).backward()
    # device
    droll = {k: dev(v) for k, v in roll.items()}
    idx = dev(perm.astype(np.int64))
    stats = torch.empty(1, 4, dtype=torch.float64, device="cuda")
    native.minibatch_adv_stats(droll["advantages"], droll["int_advantages"] if dual else None, idx, B, B, T, N, stats)
    partials = torch.zeros(native.LOSS_PARTIALS * 8, dtype=torch.float64, device="cuda")
    accum = torch.zeros(8, dtype=torch.float64, device="cuda")
    z, ls, v, iv = dev(mu), dev(log_std), dev(values), dev(ivals) if dual else None
    native.ppo_box_loss_partials(z, ls, v, iv, B, D, idx, T, N, droll, stats[0], clip, partials)
    dz, dv = torch.empty_like(z), torch.empty_like(v)
    div = torch.empty_like(iv) if dual else None
    dlsp = torch.empty(native.LOSS_PARTIALS * D, dtype=torch.float64, device="cuda")
    dls = torch.empty(D, device="cuda")
    native.ppo_box_loss_backward(z, ls, v, iv, B, D, idx, T, N, droll, stats[0], clip, partials, B, ent_coef,
                                 vf_coef, ivf, scale, dz, dlsp, dls, dv, div, accum)
    torch.cuda.synchronize()
    acc = accum.cpu().numpy()
    if B > 1:
        np.testing.assert_allclose(acc[0], pl.item(), rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(acc[1], vl.item(), rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(acc[2], el.item(), rtol=1e-5, atol=1e-7)
        sg = max(np.abs(mu_t.grad.numpy()).max(), 1e-30)
        np.testing.assert_allclose(dz.cpu().numpy(), mu_t.grad.numpy(), rtol=1e-4, atol=1e-5 * sg)
        np.testing.assert_allclose(dls.cpu().numpy(), ls_t.grad.numpy()[0], rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(dv.cpu().numpy(), v_t.grad.numpy(), rtol=1e-5, atol=1e-8)
        if dual:
            np.testing.assert_allclose(div.cpu().numpy(), iv_t.grad.numpy(), rtol=1e-5, atol=1e-8)
    else:  # one row: unbiased std is nan, as in torch — everything downstream of the surrogate is nan
        assert np.isnan(acc[0]) and np.isnan(pl.item())
        np.testing.assert_allclose(acc[1], vl.item(), rtol=1e-5, atol=1e-7)


def test_normal_sample_moments_and_logprob():
    """Collect-time Normal head: Philox Box-Muller samples have the head's mean / std, and
    log_prob matches torch's Normal.log_prob of the sampled (f32) action."""
    import native
    N, D = 100000, 3
    mu = torch.tensor([[0.3, -1.2, 2.0]], device="cuda").repeat(N, 1)
    ls = torch.tensor([-0.5, 0.0, 0.4], device="cuda")
    a = torch.empty(N, D, device="cuda")
    lp = torch.empty(N, D, device="cuda")
    native.normal_sample(mu, ls, N, D, 0, 99, 5, a, lp)
    loc, sc = torch.tanh(mu[0]).cpu(), torch.exp(ls).cpu()
    ac = a.cpu()
    np.testing.assert_allclose(ac.mean(0).numpy(), loc.numpy(), atol=4 * sc.numpy().max() / np.sqrt(N) * 3)
    np.testing.assert_allclose(ac.std(0).numpy(), sc.numpy(), rtol=2e-2)
    ref = torch.distributions.Normal(loc, sc).log_prob(ac)
    np.testing.assert_allclose(lp.cpu().numpy(), ref.numpy(), rtol=1e-5, atol=1e-5)


def test_adv_stats_remainder_and_singleton():
    """Minibatch slices incl. a remainder of 1 (unbiased std of one sample -> nan, as torch)."""
    import native
    T, N, B = 8, 5, 13
    rs = np.random.RandomState(3)
    adv = rs.randn(T, N).astype(np.float32)
    perm = rs.permutation(T * N)  # 40 = 3*13 + 1
    stats = torch.empty(4, 4, dtype=torch.float64, device="cuda")
    native.minibatch_adv_stats(dev(adv), None, dev(perm.astype(np.int64)), T * N, B, T, N, stats)
    st = stats.cpu().numpy()
    for k in range(4):
        sl = perm[k * B:(k + 1) * B]
        x = torch.tensor(adv[sl % T, sl // T])
        np.testing.assert_allclose(st[k, 0], x.double().mean().item(), rtol=1e-12)
        if len(sl) > 1:
            np.testing.assert_allclose(st[k, 1], x.double().std().item(), rtol=1e-10)
        else:
            assert np.isnan(st[k, 1])


def test_categorical_sample_distribution():
    import native
    N, A = 200000, 4
    logits = torch.tensor([[0.0, 1.0, 2.0, -1.0]], device="cuda").repeat(N, 1)
    acts = torch.empty(N, dtype=torch.int32, device="cuda")
    lp = torch.empty(N, device="cuda")
    native.categorical_sample(logits, N, A, 0, 1234, 7, acts, lp)
    p = torch.softmax(logits[0].cpu(), -1).numpy()
    freq = np.bincount(acts.cpu().numpy(), minlength=A) / N
    np.testing.assert_allclose(freq, p, atol=4e-3)
    np.testing.assert_allclose(lp.cpu().numpy(), np.log(p)[acts.cpu().numpy()], rtol=1e-5)


# ----------------------------------------------------------------- envs
def test_atari_env_matches_numpy_twin():
    import native
    N, off, seed = 6, 100, 0xDEADBEEF12345
    twin = PH.SyntheticAtari(N, seed, p_reward=0.3, p_done=0.2, env_offset=off)
    o0 = twin.reset()
    obs = torch.empty((N, 4, 84, 84), dtype=torch.uint8, device="cuda")
    native.atari_env_reset(obs, N, off, seed)
    assert np.array_equal(obs.cpu().numpy(), o0)
    rs = np.random.RandomState(0)
    nxt = torch.empty_like(obs)
    rew = torch.empty(N, device="cuda")
    done = torch.empty(N, dtype=torch.uint8, device="cuda")
    for k in range(1, 12):
        a = rs.randint(0, 4, N).astype(np.int32)
        o, r, d, _ = twin.step(a)
        native.atari_env_step(obs, nxt, dev(a), N, off, seed, k, 0.3, 0.2, rew, done)
        assert np.array_equal(nxt.cpu().numpy(), o), k
        assert np.array_equal(rew.cpu().numpy(), r)
        assert np.array_equal(done.cpu().numpy().astype(bool), d)
        obs, nxt = nxt, obs


def test_atari_env_in_place_and_sharding():
    """Stepping in place equals stepping out of place; a shard equals the slice of the full run."""
    import native
    N, seed = 8, 77
    full = torch.empty((N, 4, 84, 84), dtype=torch.uint8, device="cuda")
    native.atari_env_reset(full, N, 0, seed)
    shard = full[4:].clone()
    acts = torch.arange(N, dtype=torch.int32, device="cuda") % 4
    rew = torch.empty(N, device="cuda")
    done = torch.empty(N, dtype=torch.uint8, device="cuda")
    out = torch.empty_like(full)
    native.atari_env_step(full, out, acts, N, 0, seed, 1, 0.5, 0.5, rew, done)
    native.atari_env_step(full, full, acts, N, 0, seed, 1, 0.5, 0.5, rew, done)
    assert torch.equal(out, full)
    srew = torch.empty(4, device="cuda")
    sdone = torch.empty(4, dtype=torch.uint8, device="cuda")
    native.atari_env_step(shard, shard, acts[4:].contiguous(), 4, 4, seed, 1, 0.5, 0.5, srew, sdone)
    assert torch.equal(shard, full[4:])


# ----------------------------------------------------------------- RMS
def test_rms_u8_vs_numpy():
    import native
    rs = np.random.RandomState(1)
    rm = RM.RunningMoments()
    mean = torch.zeros(7056, dtype=torch.float64, device="cuda")
    var = torch.ones(7056, dtype=torch.float64, device="cuda")
    count = 1e-4
    for n in (100, 1, 257):
        x = rs.randint(0, 256, (n, 4, 84, 84)).astype(np.uint8)
        last = x[:, 3].reshape(n, -1)
        rm.update(last)
        xd = dev(x)
        view = xd[:, 3].reshape(n, -1)
        ws = torch.empty(native.rms_u8_workspace_bytes(n, 7056), dtype=torch.uint8, device="cuda")
        native.rms_update_u8(view, n, 7056, view.stride(0), mean, var, count, ws)
        count += n
        np.testing.assert_array_equal(mean.cpu().numpy(), rm.mean)
        np.testing.assert_allclose(var.cpu().numpy(), rm.var, rtol=1e-12)


def test_rms_f32_and_scalar_bitexact(golden):
    import native
    f = golden("rms")
    mean = torch.zeros(6, dtype=torch.float64, device="cuda")
    var = torch.ones(6, dtype=torch.float64, device="cuda")
    count = 1e-4
    for i in range(int(f["f32_n"])):
        b = f[f"f32_b{i}"]
        native.rms_update_f32(dev(b), b.shape[0], 6, 6, mean, var, count)
        count += b.shape[0]
        np.testing.assert_array_equal(mean.cpu().numpy(), f[f"f32_mean{i}"])
        np.testing.assert_array_equal(var.cpu().numpy(), f[f"f32_var{i}"])
    m1 = torch.zeros((), dtype=torch.float64, device="cuda")
    v1 = torch.ones((), dtype=torch.float64, device="cuda")
    count = 1e-4
    for i in range(int(f["sc_n"])):
        b = f[f"sc_b{i}"]
        native.rms_update_f32(dev(b), b.shape[0], 1, 1, m1, v1, count)
        count += b.shape[0]
        np.testing.assert_array_equal(m1.cpu().numpy(), f[f"sc_mean{i}"])
        np.testing.assert_array_equal(v1.cpu().numpy(), f[f"sc_var{i}"])


@pytest.mark.parametrize("n", [1, 7, 8, 100, 129, 1024, 4096, 5000])
def test_int_reward_scaling_bitexact(n):
    """ppo.py:396-398: int_rew_rms.update + in-place scaling, incl. numpy pairwise order."""
    import native
    rs = np.random.RandomState(n)
    rm = RM.RunningMoments()
    mean = torch.zeros((), dtype=torch.float64, device="cuda")
    var = torch.ones((), dtype=torch.float64, device="cuda")
    count = 1e-4
    for it in range(3):
        ir = (np.abs(rs.randn(n)) * (it + 1) * 1e3).astype(np.float32)
        exp = ir.copy()
        rm.update(exp)
        exp /= (np.sqrt(rm.var) + 1e-08)
        d = dev(ir)
        native.rms_scale_int_rewards(d, mean, var, count)
        count += n
        np.testing.assert_array_equal(mean.cpu().numpy(), rm.mean)
        np.testing.assert_array_equal(var.cpu().numpy(), rm.var)
        np.testing.assert_array_equal(d.cpu().numpy(), exp)


def test_normalize_obs_bitexact(golden):
    import native
    f = golden("rms")
    x = f["norm_in"]
    out = torch.empty(x.shape, device="cuda")
    native.normalize_obs(dev(x), x.shape[0], x.shape[1], x.shape[1], dev(f["norm_mean"]), dev(f["norm_var"]), out)
    np.testing.assert_array_equal(out.cpu().numpy(), f["norm_out"].astype(np.float32))
    # u8 frames
    rs = np.random.RandomState(2)
    u = rs.randint(0, 256, (5, 7056)).astype(np.uint8)
    m, v = rs.rand(7056) * 255, rs.rand(7056) * 5000 + 1
    out = torch.empty(u.shape, device="cuda")
    native.normalize_obs(dev(u), 5, 7056, 7056, dev(m), dev(v), out)
    np.testing.assert_array_equal(out.cpu().numpy(), RM.normalize_obs(u, m, v).astype(np.float32))


# ----------------------------------------------------------------- gather + Adam
def test_gather_rows_env_major():
    import native
    T, N, F = 16, 12, 4 * 84 * 84
    rs = np.random.RandomState(4)
    obs = rs.randint(0, 256, (T, N, F)).astype(np.uint8)
    idx = rs.permutation(T * N)[:50]
    out = torch.empty((50, F), dtype=torch.uint8, device="cuda")
    native.gather_rows(dev(obs), T, N, F, F, dev(idx.astype(np.int64)), 50, out)
    assert np.array_equal(out.cpu().numpy(), obs[idx % T, idx // T])


@pytest.mark.parametrize("max_norm", [0.2, 1e9, 0.0])
def test_adam_clip_vs_torch(max_norm):
    import native
    rs = np.random.RandomState(5)
    sizes = [(64, 33), (33,), (7, 5, 3)]
    ps = [torch.tensor(rs.randn(*s).astype(np.float32), requires_grad=True) for s in sizes]
    opt = torch.optim.Adam(ps, lr=3e-4)
    n = sum(p.numel() for p in ps)
    npad = (n + 63) // 64 * 64
    flat = torch.zeros(npad, device="cuda")
    flat[:n] = torch.cat([p.detach().reshape(-1) for p in ps]).cuda()
    m = torch.zeros_like(flat)
    v = torch.zeros_like(flat)
    g = torch.zeros_like(flat)
    part = torch.zeros(native.NORM_PARTIALS, dtype=torch.float64, device="cuda")
    for step in range(1, 4):
        grads = [rs.randn(*s).astype(np.float32) for s in sizes]
        for p, gg in zip(ps, grads):
            p.grad = torch.tensor(gg)
        if max_norm > 0:
            torch.nn.utils.clip_grad_norm_(ps, max_norm)
        opt.step()
        g.zero_()
        g[:n] = torch.cat([torch.tensor(gg).reshape(-1) for gg in grads]).cuda()
        if max_norm > 0:
            native.grad_sumsq(g, part)
        native.adam_step(flat, g, m, v, part, max_norm, 3e-4, 0.9, 0.999, 1e-8, step)
    ref = torch.cat([p.detach().reshape(-1) for p in ps]).numpy()
    np.testing.assert_allclose(flat[:n].cpu().numpy(), ref, rtol=1e-6, atol=1e-7)


# ----------------------------------------------------------------- K6 convs
def _h1p_exponent(w1, b1):
    """E of H1P (csrc/conv.hip h1p_exp_kernel): the bound 255 max_c sum_k |W1[c][k]| + |b1[c]|
    (uint8 frames) with a 2^-10 margin, scaled into [2^14, 2^15)."""
    bound = (255.0 * w1.double().abs().reshape(32, -1).sum(1) + b1.double().abs()).max().item()
    m = np.float32(bound * (1.0 + 1.0 / 1024.0))
    e = int(m.view(np.uint32)) >> 23
    return 141 - min(254, max(15, e))


def _h1_planes(h1, E):
    """H1P of an f32 NHWC h1 at exponent E with the kernels' rounding: hi = rn16(h1 2^E),
    lo = rn16(h1 2^E - hi) (the residual is exact in f32)."""
    v = h1 * 2.0 ** E
    hi = v.half()
    lo = (v - hi.float()).half()
    return torch.cat([hi.view(torch.int16), lo.view(torch.int16)], dim=-1).contiguous()


def _h1_from_planes(h1p, E):
    """(hi + lo) 2^-E: exact in f32 (two 11-bit significands 11 bits apart)."""
    return (h1p[..., :32].contiguous().view(torch.float16).float() +
            h1p[..., 32:].contiguous().view(torch.float16).float()) * 2.0 ** -E


def _relu_bits(h):
    """int32 ReLU bitmask words (bit c of word p: channel c of pixel p > 0) of a 32-channel NHWC h."""
    w = ((h > 0).reshape(-1, 32).long() << torch.arange(32, device=h.device)).sum(1)
    return torch.where(w >= 2 ** 31, w - 2 ** 32, w).to(torch.int32)

@pytest.mark.parametrize("math", ["split", "split_all", "f32"])
@pytest.mark.parametrize("B", [1, 3, 37, 256])
def test_nature_conv_fwd_vs_torch_fp32(B, math):
    """MFMA implicit-GEMM conv trunk vs torch fp32 convs (tolerance: fp32 re-association)."""
    import models
    import convs
    torch.manual_seed(B)
    net = models.CnnActorCritic(4, 4)
    ref = models.CnnActorCritic(4, 4)
    ref.load_state_dict(net.state_dict())
    flat = models.FlatParams(net, "cuda")
    ref = ref.cuda()
    convs.attach(net, flat, math)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda")
    with torch.no_grad():
        h = net.conv_impl(x)
        fe = ref.feature_extractor
        e = torch.relu(fe[4](torch.relu(fe[2](torch.relu(fe[0](x.float()))))))
    err = (h - e).abs().max().item()
    assert err <= 2e-5 * e.abs().max().item() + 1e-4, err


@pytest.mark.parametrize("math", ["split", "split_all", "f32"])
def test_nature_trunk_backward_vs_torch(math):
    import models
    import convs
    torch.manual_seed(0)
    net = models.CnnActorCritic(4, 4)
    ref = models.CnnActorCritic(4, 4)
    ref.load_state_dict(net.state_dict())
    flat = models.FlatParams(net, "cuda")
    ref = ref.cuda()
    convs.attach(net, flat, math)
    x = torch.randint(0, 256, (50, 4, 84, 84), dtype=torch.uint8, device="cuda")
    g = torch.randn(50, 64, 7, 7, device="cuda")
    flat.zero_grad()
    net.conv_impl(x).backward(g)
    fe = ref.feature_extractor
    torch.relu(fe[4](torch.relu(fe[2](torch.relu(fe[0](x.float())))))).backward(g)
    for mine, theirs in ((fe[0], net.feature_extractor[0]), (fe[2], net.feature_extractor[2]),
                         (fe[4], net.feature_extractor[4])):
        for a, b in ((theirs.weight.grad, mine.weight.grad), (theirs.bias.grad, mine.bias.grad)):
            scale = b.abs().max().item()
            assert (a - b).abs().max().item() <= 1e-4 * scale + 1e-6


def _conv_ops_fp64(B, seed):
    """Every NatureCNN conv op (fwd, dgrad, wgrad per layer) through both math modes
    and float64 CPU autograd on the same inputs: {(op, layer): (split, f32, fp64)}."""
    import models
    import convs
    import native
    torch.manual_seed(seed)
    net = models.CnnActorCritic(4, 4)
    flat = models.FlatParams(net, "cuda")
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda")
    out = {}
    for math in ("split_all", "f32"):
        net.conv_impl = None
        cv = convs.attach(net, flat, math)
        hs = {}
        cv.pack()
        h1 = cv.empty_h1(B, "cuda")  # H1P (conv1's output as f16 planes) in split math
        h2 = torch.empty(B, 9, 9, 64, device="cuda")
        h3 = torch.empty((B, 7, 7, 64) if cv.nhwc3 else (B, 64, 7, 7), device="cuda")
        am = native.amax_table(convs.AM_ROWS, "cuda")  # each forward records its output's amax
        cv.fwd(1, x, B, cv.c1.bias, h1, am)
        cv.fwd(2, h1, B, cv.c2.bias, h2, am)
        cv.fwd(3, h2, B, cv.c3.bias, h3, am)
        if cv.nhwc3:  # split math writes conv3's output NHWC
            h3 = h3.permute(0, 3, 1, 2)
        if cv.h1p:
            h1 = _h1_from_planes(h1, cv.h1p_exponent())
        hs.update({("fwd", 1): h1, ("fwd", 2): h2, ("fwd", 3): h3})
        out[math] = hs
    # backward ops on shared inputs (f32-mode activations as ReLU masks, random output grads)
    gen = torch.Generator(device="cuda").manual_seed(seed + 100)
    g3 = torch.randn(B, 7, 7, 64, device="cuda", generator=gen)
    g2r = torch.randn(B, 9, 9, 64, device="cuda", generator=gen)
    h1f, h2f = out["f32"][("fwd", 1)], out["f32"][("fwd", 2)]

    def amax_rows(**rows):  # a fresh amax table holding the given operands' rows
        am = native.amax_table(convs.AM_ROWS, "cuda")
        for name, t in rows.items():
            native.amax(t, am[getattr(convs, "AM_" + name)])
        return am
    for math in ("split_all", "f32"):
        net.conv_impl = None
        cv = convs.attach(net, flat, math)
        cv.pack()
        d2 = torch.empty(B, 9, 9, 64, device="cuda")
        d1 = torch.empty(B, 20, 20, 32, device="cuda")
        cv.dgrad(3, g3, B, h2f, d2, amax_rows(G3=g3))
        if cv.h1p:  # conv1's ReLU mask as the forward's bitmask (H1P is no f32 mask)
            cv.dgrad(2, g2r, B, None, d1, convs.PassState(amax_rows(G2=g2r), (_relu_bits(h1f), None, None)))
        else:
            cv.dgrad(2, g2r, B, h1f, d1, amax_rows(G2=g2r))
        out[math].update({("dgrad", 3): d2, ("dgrad", 2): d1})
        g1r = torch.randn(B, 20, 20, 32, device="cuda", generator=torch.Generator(device="cuda").manual_seed(seed + 7))
        am = amax_rows(G1=g1r, G2=g2r, G3=g3, H1=h1f, H2=h2f)
        for L, xin, gg in ((1, x, g1r), (2, _h1_planes(h1f, cv.h1p_exponent()) if cv.h1p else h1f, g2r), (3, h2f, g3)):
            wl = (cv.c1, cv.c2, cv.c3)[L - 1]
            dw, db = torch.empty_like(wl.weight), torch.empty_like(wl.bias)
            cv.wgrad(L, xin, B, gg, dw, db, am)
            out[math].update({("wgrad", L): dw, ("wgrad_bias", L): db})
    # fp64 reference (CPU autograd, same weights)
    fe = net.feature_extractor
    w = [fe[i].weight.detach().double().cpu() for i in (0, 2, 4)]
    b = [fe[i].bias.detach().double().cpu() for i in (0, 2, 4)]
    F = torch.nn.functional
    r1 = F.relu(F.conv2d(x.double().cpu(), w[0], b[0], stride=4))
    r2 = F.relu(F.conv2d(r1, w[1], b[1], stride=2))
    r3 = F.relu(F.conv2d(r2, w[2], b[2], stride=1))
    ref = {("fwd", 1): r1.permute(0, 2, 3, 1), ("fwd", 2): r2.permute(0, 2, 3, 1), ("fwd", 3): r3}
    nchw = lambda t: t.double().cpu().permute(0, 3, 1, 2)
    ci3 = torch.nn.grad.conv2d_input((B, 64, 9, 9), w[2], nchw(g3), stride=1)
    ci2 = torch.nn.grad.conv2d_input((B, 32, 20, 20), w[1], nchw(g2r), stride=2)
    ref[("dgrad", 3)] = (ci3 * (nchw(h2f) > 0)).permute(0, 2, 3, 1)
    ref[("dgrad", 2)] = (ci2 * (nchw(h1f) > 0)).permute(0, 2, 3, 1)
    g1r = torch.randn(B, 20, 20, 32, device="cuda", generator=torch.Generator(device="cuda").manual_seed(seed + 7))
    for L, xin, gg, st in ((1, x.double().cpu(), g1r, 4), (2, nchw(h1f), g2r, 2), (3, nchw(h2f), g3, 1)):
        ref[("wgrad", L)] = torch.nn.grad.conv2d_weight(xin, w[L - 1].shape, nchw(gg), stride=st)
        ref[("wgrad_bias", L)] = nchw(gg).sum(dim=(0, 2, 3))
    return {k: (out["split_all"][k], out["f32"][k], ref[k]) for k in ref}


@pytest.mark.parametrize("seed", [0, 1])
def test_split_conv_accuracy_is_fp32_class(seed):
    """Split-f16 kernels vs fp64: error no larger than the exact-f32-FMA kernels' own error
    (x2 headroom), for every op that has a split kernel.  Forward ops take each layer's
    input from the same mode, so errors compound as in the product path."""
    import convs
    res = _conv_ops_fp64(24, seed)
    for key, (spl, f32, ref) in res.items():
        op = ("wgrad", key[1]) if key[0] == "wgrad_bias" else key
        if op not in convs.SPLIT_OPS and op not in convs.SPLIT_SLOWER and not key[0].startswith("planes"):
            continue
        scale = ref.abs().max().item()
        e_s = (spl.cpu().double() - ref).abs().max().item() / scale
        e_f = (f32.cpu().double() - ref).abs().max().item() / scale
        assert e_s <= 2 * e_f + 1e-7, (key, e_s, e_f)


@pytest.mark.parametrize("T,N,B", [(5, 7, 33), (128, 16, 1000), (3, 2, 1)])
def test_conv1_split_reads_rollout_rows(T, N, B):
    """conv1 split forward and weight gradient reading the minibatch rows in place
    (convs.RolloutRows: idx into the step-major rollout frames) == the same kernels on the
    gathered rows (ppox_gather_rows), bitwise."""
    import convs
    import native
    torch.manual_seed(T * 100 + B)
    frames = torch.randint(0, 256, (T, N, 4, 84, 84), dtype=torch.uint8, device="cuda")
    idx = torch.randperm(T * N, device="cuda")[:B].to(torch.int64) if B <= T * N else \
        torch.randint(0, T * N, (B,), device="cuda")
    rows = torch.empty(B, 4, 84, 84, dtype=torch.uint8, device="cuda")
    native.gather_rows(frames, T, N, 28224, 28224, idx, B, rows)
    w1 = torch.randn(32, 4, 8, 8, device="cuda") * 0.05
    w2, w3 = torch.randn(64, 32, 4, 4, device="cuda"), torch.randn(64, 64, 3, 3, device="cuda")
    q = [torch.empty(native.nature_split_pack_elems(k), dtype=torch.int16, device="cuda") for k in (1, 2, 3, 12, 13)]
    native.nature_pack_split(w1, w2, w3, *q)
    b1 = torch.randn(32, device="cuda")
    y_rows, y_idx = (torch.empty(B, 20, 20, 32, device="cuda") for _ in range(2))
    native.nature_conv_fwd_split(1, rows, B, None, 0, 0, 28224, q[0], b1, y_rows)
    rr = convs.RolloutRows(frames, idx)
    native.nature_conv_fwd_split(1, rr.frames, B, rr.idx, rr.T, rr.N, 0, q[0], b1, y_idx)
    g1 = torch.randn(B, 20, 20, 32, device="cuda")
    ws = torch.empty(native.nature_wgrad_split_workspace_bytes(1, B), dtype=torch.uint8, device="cuda")
    dw_rows, dw_idx = torch.empty_like(w1), torch.empty_like(w1)
    db_rows, db_idx = torch.empty_like(b1), torch.empty_like(b1)
    native.nature_conv_wgrad_split(1, rows, B, 28224, g1, ws, dw_rows, db_rows)
    native.nature_conv_wgrad_split_idx(1, frames, B, idx, T, N, g1, ws, dw_idx, db_idx)
    torch.cuda.synchronize()
    assert torch.equal(y_rows, y_idx)
    assert torch.equal(dw_rows, dw_idx) and torch.equal(db_rows, db_idx)


@pytest.mark.parametrize("B", [1, 2, 4, 7, 301, 2311])
def test_conv2_split_dgrad_col2im_ragged(B):
    """conv2 split dgrad (col2im form: 3 samples per workgroup, four parity-class passes)
    at batches that leave a partial last workgroup, vs float64 CPU: error no larger than the
    exact-f32-FMA kernel's (x2 headroom), rows outside the batch untouched, deterministic."""
    import native
    torch.manual_seed(B)
    w2 = torch.randn(64, 32, 4, 4, device="cuda") * 0.05
    w3 = torch.randn(64, 64, 3, 3, device="cuda") * 0.05
    w1 = torch.randn(32, 4, 8, 8, device="cuda") * 0.05
    q1, q2, q3, qd2, qd3 = (torch.empty(native.nature_split_pack_elems(k), dtype=torch.int16, device="cuda")
                            for k in (1, 2, 3, 12, 13))
    native.nature_pack_split(w1, w2, w3, q1, q2, q3, qd2, qd3)
    wp = [torch.empty(n, device="cuda") for n in (256 * 32, 512 * 64, 576 * 64, 4 * 256 * 32, 576 * 64)]
    native.nature_pack_weights(w1, w2, w3, *wp)
    g = torch.randn(B, 9, 9, 64, device="cuda")
    h1 = torch.relu(torch.randn(B, 20, 20, 32, device="cuda"))
    out = torch.full((B + 1, 20, 20, 32), 7.0, device="cuda")
    out2 = torch.empty(B, 20, 20, 32, device="cuda")
    f32 = torch.empty(B, 20, 20, 32, device="cuda")
    native.nature_conv_dgrad_split(2, g, B, qd2, h1, out)
    native.nature_conv_dgrad_split(2, g, B, qd2, h1, out2)
    native.nature_conv_dgrad(2, g, B, wp[3], h1, f32)
    torch.cuda.synchronize()
    assert torch.equal(out[:B], out2), "run-to-run"
    assert bool((out[B] == 7.0).all()), "wrote past the batch"
    ref = torch.nn.grad.conv2d_input((B, 32, 20, 20), w2.double().cpu(), g.double().cpu().permute(0, 3, 1, 2),
                                     stride=2) * (h1.double().cpu().permute(0, 3, 1, 2) > 0)
    ref = ref.permute(0, 2, 3, 1)
    scale = ref.abs().max().item()
    e_s = (out[:B].double().cpu() - ref).abs().max().item() / scale
    e_f = (f32.double().cpu() - ref).abs().max().item() / scale
    assert e_s <= 2 * e_f + 1e-7, (e_s, e_f)


@pytest.mark.parametrize("B", [1, 5, 301])
def test_conv1_relu_bits_drive_conv2_dgrad(B):
    """The conv1 split forward's ReLU bitmask (bit c of word p: channel c of pixel p > 0) equals
    h1 > 0, and the conv2 split dgrad reading it equals the one reading h1, bitwise."""
    import native
    torch.manual_seed(B)
    w1 = torch.randn(32, 4, 8, 8, device="cuda") * 0.02
    w2 = torch.randn(64, 32, 4, 4, device="cuda") * 0.05
    w3 = torch.randn(64, 64, 3, 3, device="cuda") * 0.05
    q = {k: torch.empty(native.nature_split_pack_elems(k), dtype=torch.int16, device="cuda") for k in (1, 2, 3, 12, 13)}
    native.nature_pack_split(w1, w2, w3, q[1], q[2], q[3], q[12], q[13])
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda")
    b1 = torch.randn(32, device="cuda")
    h1 = torch.empty(B, 20, 20, 32, device="cuda")
    bits = torch.full((B * 400 + 1,), 12345, dtype=torch.int32, device="cuda")
    native.nature_conv_fwd_split(1, x, B, None, 0, 0, 28224, q[1], b1, h1, relu_bits=bits)
    want = ((h1 > 0).view(B * 400, 32).long() << torch.arange(32, device="cuda")).sum(1)
    assert torch.equal(bits[:-1].long() & 0xFFFFFFFF, want) and int(bits[-1]) == 12345
    g = torch.randn(B, 9, 9, 64, device="cuda")
    o_act, o_bits = torch.empty_like(h1), torch.empty_like(h1)
    native.nature_conv_dgrad_split(2, g, B, q[12], h1, o_act)
    native.nature_conv_dgrad_split(2, g, B, q[12], None, o_bits, relu_bits=bits)
    assert torch.equal(o_act, o_bits)


@pytest.mark.parametrize("B", [1, 7, 300])
def test_conv23_relu_bits_drive_dgrad3_and_fc_dgrad(B):
    """The conv2 / conv3 split forwards' ReLU bitmasks (2 words per pixel, 64 channels) equal
    h > 0, and the conv3 dgrad / fc dgrad reading them equal the ones reading h2 / h3, bitwise."""
    import native
    torch.manual_seed(B + 11)
    w1 = torch.randn(32, 4, 8, 8, device="cuda") * 0.02
    w2 = torch.randn(64, 32, 4, 4, device="cuda") * 0.05
    w3 = torch.randn(64, 64, 3, 3, device="cuda") * 0.05
    q = {k: torch.empty(native.nature_split_pack_elems(k), dtype=torch.int16, device="cuda") for k in (1, 2, 3, 12, 13)}
    native.nature_pack_split(w1, w2, w3, q[1], q[2], q[3], q[12], q[13])
    h1 = torch.relu(torch.randn(B, 20, 20, 32, device="cuda"))
    b2, b3 = torch.randn(64, device="cuda") * 0.1, torch.randn(64, device="cuda") * 0.1
    h2, h3 = torch.empty(B, 9, 9, 64, device="cuda"), torch.empty(B, 7, 7, 64, device="cuda")
    bits2 = torch.full((B * 81 * 2 + 2,), 777, dtype=torch.int32, device="cuda")
    bits3 = torch.full((B * 49 * 2 + 2,), 777, dtype=torch.int32, device="cuda")
    native.nature_conv_fwd_split(2, h1, B, None, 0, 0, 0, q[2], b2, h2, relu_bits=bits2)
    native.nature_conv_fwd_split(3, h2, B, None, 0, 0, 0, q[3], b3, h3, relu_bits=bits3)
    for h, bits, P in ((h2, bits2, 81), (h3, bits3, 49)):
        want = ((h > 0).view(B * P * 2, 32).long() << torch.arange(32, device="cuda")).sum(1)
        assert torch.equal(bits[:-2].long() & 0xFFFFFFFF, want) and bits[-2:].tolist() == [777, 777]
    g3 = torch.randn(B, 7, 7, 64, device="cuda")
    o_act, o_bits = torch.empty_like(h2), torch.empty_like(h2)
    native.nature_conv_dgrad_split(3, g3, B, q[13], h2, o_act)
    native.nature_conv_dgrad_split(3, g3, B, q[13], None, o_bits, relu_bits=bits2)
    assert torch.equal(o_act, o_bits)
    W = torch.randn(512, 3136, device="cuda") * 0.02
    n = native.nature_fc_pack_elems()
    qf, qd = torch.empty(n, dtype=torch.int16, device="cuda"), torch.empty(n, dtype=torch.int16, device="cuda")
    native.nature_fc_pack(W, qf, qd)
    df = torch.randn(B, 512, device="cuda")
    f_act, f_bits = torch.empty_like(h3), torch.empty_like(h3)
    native.nature_fc_dgrad(df, B, qd, h3, f_act)
    native.nature_fc_dgrad(df, B, qd, None, f_bits, relu_bits=bits3)
    assert torch.equal(f_act, f_bits)


@pytest.mark.parametrize("intrinsic,B", [(False, 40), (True, 40), (False, 600)])
def test_cnn_explicit_backward_matches_autograd(intrinsic, B):
    """CnnActorCritic.forward_train/backward_train (no autograd graph, grads straight into
    the flat buffer) == autograd through forward() on the same libppox trunk."""
    import models
    import convs
    torch.manual_seed(3)
    net = models.CnnActorCritic(4, 6, intrinsic=intrinsic)
    flat = models.FlatParams(net, "cuda")
    convs.attach(net, flat, "f32")
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda")
    dout, dv = torch.randn(B, 6, device="cuda"), torch.randn(B, device="cuda")
    div = torch.randn(B, device="cuda") if intrinsic else None
    flat.zero_grad()
    out, v, iv = net(x)
    ts, gs = [out, v], [dout, dv]
    if intrinsic:
        ts.append(iv)
        gs.append(div)
    torch.autograd.backward(ts, gs)
    ref = flat.grad.clone()
    flat.zero_grad()
    out2, v2, iv2, ctx = net.forward_train(x)
    # the explicit heads run the skinny-row kernels (fixed reduction order), autograd's nn.Linear
    # rocBLAS: two f32 evaluations of 512-term dot products (un-normalised u8 frames: large terms)
    for a_, b_ in ((out2, out.detach()), (v2, v.detach())):
        torch.testing.assert_close(a_, b_, rtol=1e-4, atol=1e-5 * (b_.abs().max().item() + 1))
    with torch.no_grad():  # the collect forward runs the same head kernels as forward_train
        out3, v3, _ = net(x)
    assert torch.equal(out3, out2) and torch.equal(v3, v2)
    net.backward_train(ctx, dout, dv, div)
    got = flat.grad
    for p in flat.params:  # per-tensor relative check (views into the flat buffer)
        off = (p.grad.data_ptr() - flat.grad.data_ptr()) // 4
        r, g = ref[off:off + p.numel()], got[off:off + p.numel()]
        scale = r.abs().max().item() + 1e-12
        assert (r - g).abs().max().item() <= 1e-5 * scale + 1e-7, p.shape


@pytest.mark.parametrize("rows,A,intrinsic", [(1, 4, False), (5000, 18, True), (16384, 4, False)])
def test_head_grads_match_fp64(rows, A, intrinsic):
    """ppox_head_grads (fused column reductions of the head backward) vs float64 torch."""
    import native
    H = 512
    g = torch.Generator(device="cuda").manual_seed(rows)
    mk = lambda *s: torch.randn(*s, device="cuda", generator=g)
    f, e, de, df, dout, dv = mk(rows, H).relu(), mk(rows, H).relu(), mk(rows, H), mk(rows, H), mk(rows, A), mk(rows)
    ie, die, div = (mk(rows, H).relu(), mk(rows, H), mk(rows)) if intrinsic else (None, None, None)
    outs = [torch.full(s, float("nan"), device="cuda") for s in [(A, H), (A,), (1, H), (1,), (H,), (H,)]]
    iouts = [torch.full(s, float("nan"), device="cuda") for s in [(1, H), (1,), (H,)]] if intrinsic else [None] * 3
    ws = torch.empty(native.head_grads_workspace_bytes(rows, H, A, intrinsic), dtype=torch.uint8, device="cuda")
    native.head_grads(f, e, dout, dv, de, df, ws, *outs, ie=ie, div=div, die=die, w_critic_int=iouts[0],
                      b_critic_int=iouts[1], b_int_extra=iouts[2])
    d = lambda t: t.double()
    refs = [d(dout).t() @ d(f), d(dout).sum(0), (d(dv) @ d(e)).view(1, H), d(dv).sum().view(1), d(de).sum(0),
            d(df).sum(0)]
    if intrinsic:
        refs += [(d(div) @ d(ie)).view(1, H), d(div).sum().view(1), d(die).sum(0)]
        outs += iouts
    for o, r in zip(outs, refs):
        scale = r.abs().max().item() + 1.0
        assert (o.double() - r).abs().max().item() <= 2e-5 * scale * max(1.0, (rows / 1000) ** 0.5), o.shape


def test_normalize_obs_with_fresh_scalar_rms():
    """ppo.py:111-118 with the shape-() RunningMeanStd never updated (train before any
    collect): numpy broadcasts the scalar moments; the device path expands them first
    (the kernel reads per-feature moments) and the wrapper rejects mismatched sizes."""
    import native
    import ppo
    alg = ppo.PPO_RND(env_id="MontezumaRevengeNoFrameskip-v4", n_envs=4, nstep=8, batch_size=16, n_epochs=1, quiet=True)
    obs = torch.randint(0, 256, (6, 84 * 84), dtype=torch.uint8, device="cuda")
    out = alg.normalize_obs(obs)
    u = obs.cpu().numpy()
    ref = RM.normalize_obs(u, np.zeros(()), np.ones(())).astype(np.float32)  # numpy broadcasting
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    with pytest.raises(ValueError):
        native.normalize_obs(obs, 6, 7056, 7056, torch.zeros(1, dtype=torch.float64, device="cuda"),
                             torch.ones(1, dtype=torch.float64, device="cuda"), out)


@pytest.mark.parametrize("rows,n", [(1, 1), (2048, 4), (777, 8)])
def test_head_dgrad_outer_equals_separate_kernels(rows, n):
    """ppox_head_dgrad_outer (the actor dgrad and the critic's ReLU-layer grad in one launch) ==
    ppox_skinny_dgrad + ppox_outer_relu_backward, bitwise, amax slots included."""
    import native
    g = torch.Generator(device="cuda").manual_seed(rows + n)
    mk = lambda *s: torch.randn(*s, device="cuda", generator=g)
    dout, wa, dv, e = mk(rows, n), mk(n, 512), mk(rows), mk(rows, 512).relu()
    wc = mk(1, 512)
    am_a, am_b = native.amax_table(2, "cuda")
    df, de = native.head_dgrad_outer(dout, wa, dv, wc, e, amax_de=am_a)
    de2 = torch.empty_like(e)
    native.outer_relu_backward(dv.view(rows, 1), wc, e, de2, amax=am_b)
    assert torch.equal(df, native.head_dgrad(dout, wa)) and torch.equal(de, de2)
    assert torch.equal(am_a.max(), am_b.max())


@pytest.mark.parametrize("rows", [1, 2048, 5000])
def test_head_grads_fused_relu_df(rows):
    """ppox_head_grads with relu_df (the fc ReLU backward applied to df in place first) ==
    ppox_relu_backward_amax_ then ppox_head_grads: df, every output and df's amax bitwise."""
    import native
    H, A = 512, 4
    g = torch.Generator(device="cuda").manual_seed(rows)
    mk = lambda *s: torch.randn(*s, device="cuda", generator=g)
    f, e, de, df, dout, dv = mk(rows, H).relu(), mk(rows, H).relu(), mk(rows, H), mk(rows, H), mk(rows, A), mk(rows)
    ws = torch.empty(native.head_grads_workspace_bytes(rows, H, A, False), dtype=torch.uint8, device="cuda")
    res = []
    for fused in (True, False):
        d = df.clone()
        am = native.amax_table(1, "cuda")[0]
        outs = [torch.full(s, float("nan"), device="cuda") for s in [(A, H), (A,), (1, H), (1,), (H,), (H,)]]
        if not fused:
            native.relu_backward_(d, f, amax=am)
        native.head_grads(f, e, dout, dv, de, d, ws, *outs, relu_df=fused, amax_df=am if fused else None)
        res.append((d, am.max(), outs))
    (d1, m1, o1), (d2, m2, o2) = res
    assert torch.equal(d1, d2) and torch.equal(m1, m2)
    assert all(torch.equal(x, y) for x, y in zip(o1, o2))


@pytest.mark.parametrize("rows,n", [(1, 1), (2048, 4), (777, 8)])
def test_skinny_heads_match_fp64(rows, n):
    import native
    g = torch.Generator(device="cuda").manual_seed(rows)
    x = torch.randn(rows, 512, device="cuda", generator=g)
    w = torch.randn(n, 512, device="cuda", generator=g)
    b = torch.randn(n, device="cuda", generator=g)
    y = native.head_linear(x, w, b)
    ref = x.double() @ w.double().t() + b.double()
    assert (y.double() - ref).abs().max().item() <= 1e-5 * (ref.abs().max().item() + 1)
    gr = torch.randn(rows, n, device="cuda", generator=g)
    d = native.head_dgrad(gr, w)
    refd = gr.double() @ w.double()
    assert (d.double() - refd).abs().max().item() <= 1e-5 * (refd.abs().max().item() + 1)


def test_pack_all_matches_separate_packers():
    """ppox_nature_pack_all (one launch, output-major 16-B units) == the per-layout packers."""
    import native
    torch.manual_seed(0)
    w1, w2, w3 = torch.randn(32, 4, 8, 8, device="cuda"), torch.randn(64, 32, 4, 4, device="cuda"), \
        torch.randn(64, 64, 3, 3, device="cuda")
    wfc = torch.randn(512, 3136, device="cuda")
    q = lambda k: torch.zeros(native.nature_split_pack_elems(k), dtype=torch.int16, device="cuda")
    nfc = native.nature_fc_pack_elems()
    fc = lambda: torch.zeros(nfc, dtype=torch.int16, device="cuda")
    a = [q(1), q(2), q(3), q(12), q(13), fc(), fc(), torch.zeros(16 * 64 * 32, device="cuda")]
    b = [q(1), q(2), q(3), q(12), q(13), fc(), fc(), torch.zeros(16 * 64 * 32, device="cuda")]
    b1 = torch.randn(32, device="cuda")
    native.nature_pack_all(w1, w2, w3, wfc, a[7], a[0], a[1], a[2], a[3], a[4], a[5], a[6], b1=b1)
    native.nature_pack_split(w1, w2, w3, b[0], b[1], b[2], b[3], b[4])
    # pack_all also derives the H1P exponent of conv1's output into q1's tail (pack_split does not)
    tail = a[0][native.nature_split_pack_elems(1) - 2 * native.PACK_TAIL32:].view(torch.int32)
    assert int(tail[native.AMAX_SLOTS + 1]) == _h1p_exponent(w1, b1)
    tail[native.AMAX_SLOTS + 1] = 0
    native.nature_fc_pack(wfc, b[5], b[6])
    wp = [torch.empty(n, device="cuda") for n in (256 * 32, 512 * 64, 576 * 64)]
    native.nature_pack_weights(w1, w2, w3, wp[0], wp[1], wp[2], b[7], None)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_u8_to_f32_exact():
    import native
    x = torch.randint(0, 256, (37, 4, 84, 84), dtype=torch.uint8, device="cuda")
    assert torch.equal(native.u8_to_f32(x), x.float())


def test_vecnormalize_matches_numpy_restatement():
    """env.VecNormalize (device) vs oracle/vecnorm.py (SB3 0.x VecNormalize restated in
    numpy; parity unpinned): normalised obs and rewards, returns and both running stats
    bit-exact over 12 steps with episode ends, on a synthetic vector env."""
    import env as E
    from oracle.vecnorm import VecNormalizeNumpy
    N, D = 300, 11
    rew = torch.empty(N, device="cuda")
    done = torch.empty(N, dtype=torch.uint8, device="cuda")
    # full-sequence check on recorded raw inputs (kernels vs numpy, same inputs)
    venv2 = E.DeviceVecEnv("Hopper-v2", N, seed=3, p_done=0.05)
    raw_obs = torch.empty(N, D, device="cuda")
    venv2.reset_into(raw_obs)
    vn2 = E.VecNormalize(E.DeviceVecEnv("Hopper-v2", N, seed=3, p_done=0.05), norm_reward=True)
    out = torch.empty(N, D, device="cuda")
    vn2.reset_into(out)
    ref2 = VecNormalizeNumpy(N, D)
    ref2.reset(raw_obs.cpu().numpy())
    r_raw = torch.empty(N, device="cuda")
    d_raw = torch.empty(N, dtype=torch.uint8, device="cuda")
    for t in range(12):
        venv2.step_into(raw_obs, raw_obs, None, r_raw, d_raw)
        vn2.step_into(out, out, None, rew, done)
        assert torch.equal(d_raw, done)
        o_r, r_r = ref2.step(raw_obs.cpu().numpy(), r_raw.cpu().numpy(), d_raw.cpu().numpy().astype(bool))
        np.testing.assert_array_equal(out.cpu().numpy(), o_r.astype(np.float32))
        np.testing.assert_array_equal(rew.cpu().numpy(), r_r.astype(np.float32))
        np.testing.assert_array_equal(vn2.ret.cpu().numpy(), ref2.ret)
        np.testing.assert_array_equal(vn2.obs_rms.mean.cpu().numpy(), ref2.obs_rms.mean)
        np.testing.assert_array_equal(vn2.obs_rms.var.cpu().numpy(), ref2.obs_rms.var)
        assert float(vn2.ret_rms.var.cpu()) == float(ref2.ret_rms.var)
        assert float(vn2.ret_rms.mean.cpu()) == float(ref2.ret_rms.mean)
    # unnormalize_obs inverts the normalisation (up to f32 rounding of the stored obs)
    back = vn2.unnormalize_obs(out).cpu().numpy()
    np.testing.assert_allclose(back, vn2.raw.cpu().numpy(), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("B", [1, 130, 1000])
def test_fc_split_gemm_vs_fp64(B):
    """Split-f16 fc GEMM (3136 -> 512) forward and fused dgrad vs float64, error no
    larger than torch's f32 GEMM's (x2 headroom)."""
    import native
    torch.manual_seed(B)
    W = torch.randn(512, 3136, device="cuda") * 0.02
    b = torch.randn(512, device="cuda") * 0.1
    h3n = torch.relu(torch.randn(B, 7, 7, 64, device="cuda"))      # NHWC, as the split conv3 writes it
    h3 = h3n.permute(0, 3, 1, 2).reshape(B, 3136)                    # the reference's Flatten order
    df = torch.randn(B, 512, device="cuda")
    n = native.nature_fc_pack_elems()
    qf, qd = torch.empty(n, dtype=torch.int16, device="cuda"), torch.empty(n, dtype=torch.int16, device="cuda")
    native.nature_fc_pack(W, qf, qd)
    f = torch.empty(B, 512, device="cuda")
    native.nature_fc_fwd(h3n, B, qf, b, f)
    ref = torch.relu(h3.double() @ W.double().t() + b.double())
    e_s = (f.double() - ref).abs().max() / ref.abs().max()
    e_f = (torch.relu(torch.addmm(b, h3, W.t())).double() - ref).abs().max() / ref.abs().max()
    assert e_s <= 2 * e_f + 1e-7, (float(e_s), float(e_f))
    g3 = torch.empty(B, 7, 7, 64, device="cuda")
    native.nature_fc_dgrad(df, B, qd, h3n, g3)
    mask = h3n > 0
    refd = (df.double() @ W.double()).view(B, 64, 7, 7).permute(0, 2, 3, 1) * mask
    e_s = (g3.double() - refd).abs().max() / refd.abs().max()
    e_f = ((df @ W).view(B, 64, 7, 7).permute(0, 2, 3, 1) * mask).double().sub(refd).abs().max() / refd.abs().max()
    assert e_s <= 2 * e_f + 1e-7, (float(e_s), float(e_f))


@pytest.mark.parametrize("B", [1, 130, 512, 2048, 4000])
def test_fc_fwd_splitk_vs_fp64(B):
    """fc forward split over K (ppox_nature_fc_fwd_splitk: 1-8 K-ranges by batch, partials
    reduced in order with bias + ReLU) vs float64: error no larger than torch's f32 GEMM's (x2
    headroom), and run-to-run bitwise."""
    import native
    torch.manual_seed(B + 7)
    W = torch.randn(512, 3136, device="cuda") * 0.02
    b = torch.randn(512, device="cuda") * 0.1
    h3n = torch.relu(torch.randn(B, 7, 7, 64, device="cuda"))
    h3 = h3n.permute(0, 3, 1, 2).reshape(B, 3136)
    n = native.nature_fc_pack_elems()
    qf, qd = torch.empty(n, dtype=torch.int16, device="cuda"), torch.empty(n, dtype=torch.int16, device="cuda")
    native.nature_fc_pack(W, qf, qd)
    ws = torch.empty(native.nature_fc_fwd_splitk_workspace_bytes(B), dtype=torch.uint8, device="cuda")
    f = torch.full((B, 512), float("nan"), device="cuda")
    native.nature_fc_fwd_splitk(h3n, B, qf, b, ws, f)
    ref = torch.relu(h3.double() @ W.double().t() + b.double())
    e_s = (f.double() - ref).abs().max() / ref.abs().max()
    e_f = (torch.relu(torch.addmm(b, h3, W.t())).double() - ref).abs().max() / ref.abs().max()
    assert e_s <= 2 * e_f + 1e-7, (float(e_s), float(e_f))
    f2 = torch.empty_like(f)
    native.nature_fc_fwd_splitk(h3n, B, qf, b, ws, f2)
    assert torch.equal(f, f2)
    # the fused actor head (the small-batch training forward): the same f bitwise, logits bitwise
    # those of ppox_skinny_linear on it, and f's amax slots as the plain reduce records them
    for A in (1, 4, 8):
        wa, ba = torch.randn(A, 512, device="cuda") * 0.05, torch.randn(A, device="cuda")
        f3, lg = torch.empty_like(f), torch.full((B, A), float("nan"), device="cuda")
        am_a, am_b = native.amax_table(2, "cuda")
        native.nature_fc_fwd_splitk(h3n, B, qf, b, ws, f3, amax_f=am_a, actor=(wa, ba), logits=lg)
        native.nature_fc_fwd_splitk(h3n, B, qf, b, ws, f2, amax_f=am_b)
        assert torch.equal(f3, f) and torch.equal(lg, native.head_linear(f, wa, ba))
        assert am_a.max() == am_b.max() == f.abs().max().view(torch.int32)


@pytest.mark.parametrize("B", [1, 33, 1000, 2048, 5000])
def test_fc_wgrad_split_vs_fp64(B):
    """fc weight gradient on the split wgrad kernel (ppox_nature_fc_wgrad: h3 NHWC, dW in the
    weight's Flatten order) vs float64: error no larger than torch's f32 GEMM's (x2 headroom);
    ragged batches (partial 32-row steps, empty splits), and bitwise run-to-run determinism."""
    import native
    torch.manual_seed(B + 7)
    h3n = torch.relu(torch.randn(B, 7, 7, 64, device="cuda"))
    h3 = h3n.permute(0, 3, 1, 2).reshape(B, 3136)
    df = torch.randn(B, 512, device="cuda") * (torch.rand(B, 512, device="cuda") > 0.3)
    ws = torch.empty(native.nature_fc_wgrad_workspace_bytes(B), dtype=torch.uint8, device="cuda")
    dw = torch.full((512, 3136), float("nan"), device="cuda")
    native.nature_fc_wgrad(df, B, h3n, ws, dw)
    ref = df.double().t() @ h3.double()
    scale = ref.abs().max()
    e_s = (dw.double() - ref).abs().max() / scale
    e_f = ((df.t() @ h3).double() - ref).abs().max() / scale
    assert torch.isfinite(dw).all()
    assert e_s <= 2 * e_f + 1e-7, (float(e_s), float(e_f))
    dw2 = torch.empty_like(dw)
    native.nature_fc_wgrad(df, B, h3n, ws, dw2)
    assert torch.equal(dw, dw2)


def test_amax_slots_record_the_max():
    """ppox_amax: the slots' maximum is max |x| (f32 bits), any sign, zeros and subnormals."""
    import native
    for x in (torch.randn(1000, 12, device="cuda") * 1e-3, torch.zeros(64, device="cuda"),
              torch.full((8,), -3.5, device="cuda"), torch.tensor([1e-40, -2e-40, 0.0, 0.0], device="cuda")):
        am = native.amax_table(1, "cuda")[0]
        native.amax(x, am)
        got = am.view(torch.float32).max().item()
        assert got == x.abs().max().item()


@pytest.mark.parametrize("mag", [1e-15, 1e-7, 1e7, 1e15, "lognormal"])
def test_split_f16_any_operand_range(mag):
    """Split-f16 operands are scaled per tensor by a power of two from their amax: the fc
    forward, fused dgrad and weight gradient keep an error no larger than torch's f32 GEMM's
    (x2 headroom) for operands of any magnitude, and for entries spread over ~13 decades."""
    import native
    B = 300
    torch.manual_seed(5)
    W = torch.randn(512, 3136, device="cuda") * 0.02
    b = torch.zeros(512, device="cuda")
    h3n = torch.relu(torch.randn(B, 7, 7, 64, device="cuda"))
    df = torch.randn(B, 512, device="cuda")
    if mag == "lognormal":
        h3n = h3n * torch.exp(3 * torch.randn_like(h3n))
        df = df * torch.exp(3 * torch.randn_like(df))
    else:
        h3n, df = h3n * mag, df * mag
    h3 = h3n.permute(0, 3, 1, 2).reshape(B, 3136)
    n = native.nature_fc_pack_elems()
    qf, qd = torch.empty(n, dtype=torch.int16, device="cuda"), torch.empty(n, dtype=torch.int16, device="cuda")
    native.nature_fc_pack(W, qf, qd)
    rel = lambda got, ref: ((got.double() - ref).abs().max() / ref.abs().max()).item()
    f = torch.empty(B, 512, device="cuda")
    native.nature_fc_fwd(h3n, B, qf, b, f)
    ref = torch.relu(h3.double() @ W.double().t())
    assert rel(f, ref) <= 2 * rel(torch.relu(h3 @ W.t()), ref) + 1e-7
    g3 = torch.empty(B, 7, 7, 64, device="cuda")
    native.nature_fc_dgrad(df, B, qd, h3n, g3)
    refd = (df.double() @ W.double()).view(B, 64, 7, 7).permute(0, 2, 3, 1) * (h3n > 0)
    e_f = rel((df @ W).view(B, 64, 7, 7).permute(0, 2, 3, 1) * (h3n > 0), refd)
    assert rel(g3, refd) <= 2 * e_f + 1e-7
    ws = torch.empty(native.nature_fc_wgrad_workspace_bytes(B), dtype=torch.uint8, device="cuda")
    dw = torch.empty(512, 3136, device="cuda")
    native.nature_fc_wgrad(df, B, h3n, ws, dw)
    refw = df.double().t() @ h3.double()
    assert rel(dw, refw) <= 2 * rel(df.t() @ h3, refw) + 1e-7


@pytest.mark.parametrize("B", [1, 70, 2048, 9000])
def test_head_hidden_split_vs_fp64(B):
    """The heads' hidden layer Linear(512, 512) on the split-f16 kernels vs float64: forward
    relu(f W^T + b), the in-place accumulated + ReLU-masked input grad (f > 0) ? df + de W : 0
    and the weight gradient de^T f — errors no larger than torch's f32 GEMMs' (x2 headroom);
    the weight gradient bitwise run-to-run, and zero rows give a zero gradient."""
    import native
    g = torch.Generator(device="cuda").manual_seed(B)
    W = torch.randn(512, 512, device="cuda", generator=g) * 0.04
    bias = torch.randn(512, device="cuda", generator=g) * 0.1
    f = torch.relu(torch.randn(B, 512, device="cuda", generator=g))
    de = torch.randn(B, 512, device="cuda", generator=g) * (torch.rand(B, 512, device="cuda", generator=g) > 0.4)
    df0 = torch.randn(B, 512, device="cuda", generator=g) * 0.1
    n = native.head_hidden_pack_elems()
    qf, qd = torch.empty(n, dtype=torch.int16, device="cuda"), torch.empty(n, dtype=torch.int16, device="cuda")
    w1, w2, w3 = torch.randn(32, 4, 8, 8, device="cuda"), torch.randn(64, 32, 4, 4, device="cuda"), \
        torch.randn(64, 64, 3, 3, device="cuda")
    native.nature_pack_all(w1, w2, w3, None, None, None, None, None, None, None, None, None, W, qf, qd)
    rel = lambda got, ref: ((got.double() - ref).abs().max() / ref.abs().max()).item()
    e = torch.empty(B, 512, device="cuda")
    native.head_hidden_fwd(f, qf, bias, e)
    ref = torch.relu(f.double() @ W.double().t() + bias.double())
    assert rel(e, ref) <= 2 * rel(torch.relu(torch.addmm(bias, f, W.t())), ref) + 1e-7
    df = df0.clone()
    am = native.amax_table(1, "cuda")[0]
    native.head_hidden_dgrad(de, qd, f, df, amax_df=am)
    refd = (df0.double() + de.double() @ W.double()) * (f > 0)
    assert rel(df, refd) <= 2 * rel((df0 + de @ W) * (f > 0), refd) + 1e-7
    assert am.view(torch.float32).max().item() == df.abs().max().item()
    ws = torch.empty(max(native.head_hidden_wgrad_workspace_bytes(B), 16), dtype=torch.uint8, device="cuda")
    dw, dw2 = torch.empty(512, 512, device="cuda"), torch.empty(512, 512, device="cuda")
    native.head_hidden_wgrad(de, f, ws, dw)
    native.head_hidden_wgrad(de, f, ws, dw2)
    refw = de.double().t() @ f.double()
    assert rel(dw, refw) <= 2 * rel(de.t() @ f, refw) + 1e-7
    assert torch.equal(dw, dw2)
    z = torch.ones(512, 512, device="cuda")
    native.head_hidden_wgrad(torch.empty(0, 512, device="cuda"), torch.empty(0, 512, device="cuda"), ws, z)
    assert not z.any()


@pytest.mark.parametrize("B", [1, 3, 127, 512, 2048, 4099])
def test_head_hidden_fwd_splitk_vs_fp64(B):
    """The hidden layer's forward split over K (small batches, every split count 8 .. 1): e vs float64
    within 2x torch's own f32 GEMM error, bitwise the same e with and without the fused critic head,
    the fused value bitwise equal to the skinny kernel on that e, run-to-run bitwise."""
    import native
    g = torch.Generator(device="cuda").manual_seed(B + 7)
    W = torch.randn(512, 512, device="cuda", generator=g) * 0.04
    bias = torch.randn(512, device="cuda", generator=g) * 0.1
    f = torch.relu(torch.randn(B, 512, device="cuda", generator=g))
    wc = torch.randn(1, 512, device="cuda", generator=g) * 0.05
    bc = torch.randn(1, device="cuda", generator=g)
    n = native.head_hidden_pack_elems()
    qf = torch.empty(n, dtype=torch.int16, device="cuda")
    w1, w2, w3 = torch.randn(32, 4, 8, 8, device="cuda"), torch.randn(64, 32, 4, 4, device="cuda"), \
        torch.randn(64, 64, 3, 3, device="cuda")
    native.nature_pack_all(w1, w2, w3, None, None, None, None, None, None, None, None, None, W, qf, None)
    ws = torch.empty(max(native.head_hidden_fwd_splitk_workspace_bytes(B), 16), dtype=torch.uint8, device="cuda")
    e, e2, e3 = (torch.empty(B, 512, device="cuda") for _ in range(3))
    v, v2 = torch.empty(B, device="cuda"), torch.empty(B, device="cuda")
    native.head_hidden_fwd_splitk(f, qf, bias, ws, e)
    native.head_hidden_fwd_splitk(f, qf, bias, ws, e2, critic=(wc, bc), value=v)
    native.head_hidden_fwd_splitk(f, qf, bias, ws, e3, critic=(wc, bc), value=v2)
    ref = torch.relu(f.double() @ W.double().t() + bias.double())
    rel = lambda got, r: ((got.double() - r).abs().max() / r.abs().max()).item()
    assert rel(e, ref) <= 2 * rel(torch.relu(torch.addmm(bias, f, W.t())), ref) + 1e-7
    assert torch.equal(e, e2) and torch.equal(e2, e3) and torch.equal(v, v2)
    assert torch.equal(v, native.head_linear(e2, wc, bc).squeeze(-1))


def test_fc_wgrad_zero_rows_writes_zero():
    import native
    dw = torch.full((512, 3136), 1.0, device="cuda")
    native.nature_fc_wgrad(torch.empty(0, 512, device="cuda"), 0, torch.empty(0, 7, 7, 64, device="cuda"),
                           torch.empty(1, dtype=torch.uint8, device="cuda"), dw)
    assert not dw.any()


def test_stream_ptr_is_torch_current_stream():
    """native.stream_ptr() (raw-stream accessor) == torch.cuda.current_stream().cuda_stream,
    on the default stream and inside a side-stream context."""
    import native
    raw = lambda p: p.value or 0  # the legacy default stream is the null pointer
    assert raw(native.stream_ptr()) == torch.cuda.current_stream().cuda_stream
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        assert raw(native.stream_ptr()) == s.cuda_stream == torch.cuda.current_stream().cuda_stream != 0
    assert raw(native.stream_ptr(s)) == s.cuda_stream


@pytest.mark.parametrize("B", [8192, 9001])
def test_conv3_wgrad_split_big_batch_vs_fp64(B):
    """conv3 weight gradient at training-size batches (392-441 split-K slices of ~2048 pixels, 9
    k-blocks) vs float64 on the device: error no larger than an f32 GEMM's (x2 headroom), a ragged
    batch, the bias grad, and bitwise run-to-run determinism."""
    import native
    torch.manual_seed(B)
    h2 = torch.relu(torch.randn(B, 9, 9, 64, device="cuda"))
    g3 = torch.randn(B, 7, 7, 64, device="cuda") * (torch.rand(B, 7, 7, 64, device="cuda") > 0.4)
    ws = torch.empty(native.nature_wgrad_split_workspace_bytes(3, B), dtype=torch.uint8, device="cuda")
    dw = torch.full((64, 64, 3, 3), float("nan"), device="cuda")
    db = torch.full((64,), float("nan"), device="cuda")
    native.nature_conv_wgrad_split(3, h2, B, 0, g3, ws, dw, db)

    def ref(dt):  # dW[co][ci][ky][kx] = sum_(n, p) im2col(h2)[n, p, (ci, ky, kx)] g3[n, p, co]
        cols = torch.nn.functional.unfold(h2.permute(0, 3, 1, 2).to(dt), 3)  # (B, 576, 49)
        g = g3.reshape(B, 49, 64).to(dt)
        return torch.einsum("bkp,bpc->ck", cols, g).reshape(64, 64, 3, 3)
    r64, r32 = ref(torch.float64), ref(torch.float32)
    scale = r64.abs().max()
    e_s = (dw.double() - r64).abs().max() / scale
    e_f = (r32.double() - r64).abs().max() / scale
    assert torch.isfinite(dw).all()
    assert e_s <= 2 * e_f + 1e-7, (float(e_s), float(e_f))
    rb = g3.double().sum(dim=(0, 1, 2))
    assert ((db.double() - rb).abs().max() / rb.abs().max()).item() < 1e-5
    dw2, db2 = torch.empty_like(dw), torch.empty_like(db)
    native.nature_conv_wgrad_split(3, h2, B, 0, g3, ws, dw2, db2)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)


@pytest.mark.parametrize("B", [8192, 9001])
def test_sg2_conv_big_batch_vs_fp64(B):
    """The sg2 split kernels at training-size batches: conv2 / conv3 forward (bias + ReLU, NHWC)
    and the conv3 dgrad (x ReLU mask of h2) vs float64 on the device, error no larger than the
    same math in f32 (x2 headroom), a ragged batch, bitwise run-to-run determinism, and each
    forward's ReLU bitmask."""
    import native
    F = torch.nn.functional
    torch.manual_seed(B)
    w1 = torch.randn(32, 4, 8, 8, device="cuda") * 0.05
    w2 = torch.randn(64, 32, 4, 4, device="cuda") * 0.05
    w3 = torch.randn(64, 64, 3, 3, device="cuda") * 0.05
    b2, b3 = torch.randn(64, device="cuda") * 0.1, torch.randn(64, device="cuda") * 0.1
    q = [torch.empty(native.nature_split_pack_elems(L), dtype=torch.int16, device="cuda") for L in (1, 2, 3)]
    qd3 = torch.empty(native.nature_split_pack_elems(13), dtype=torch.int16, device="cuda")
    native.nature_pack_split(w1, w2, w3, q[0], q[1], q[2], None, qd3)
    h1 = torch.randn(B, 20, 20, 32, device="cuda").relu()
    h2 = torch.randn(B, 9, 9, 64, device="cuda").relu()
    g3 = torch.randn(B, 7, 7, 64, device="cuda")

    def fwd_ref(x, w, b, k, s, dt):  # NHWC in -> NHWC out, relu(conv + b)
        cols = F.unfold(x.permute(0, 3, 1, 2).to(dt), k, stride=s)  # (B, CIN k k, P)
        y = torch.einsum("ck,bkp->bpc", w.reshape(64, -1).to(dt), cols) + b.to(dt)
        return y.relu()

    def dgrad3_ref(dt):
        cg = torch.einsum("ck,bpc->bkp", w3.reshape(64, -1).to(dt), g3.reshape(B, 49, 64).to(dt))
        return F.fold(cg, (9, 9), 3).permute(0, 2, 3, 1) * (h2 > 0).to(dt)

    def check(got, r64, r32):
        scale = r64.abs().max()
        e_s = (got.double() - r64).abs().max() / scale
        e_f = (r32.double() - r64).abs().max() / scale
        assert torch.isfinite(got).all()
        assert e_s <= 2 * e_f + 1e-7, (float(e_s), float(e_f))

    for layer, x, w, b, k, s, P in ((2, h1, w2, b2, 4, 2, 81), (3, h2, w3, b3, 3, 1, 49)):
        ys = []
        for _ in range(2):
            y = torch.full((B, P, 64), float("nan"), device="cuda")
            bits = torch.zeros(B * P * 2, dtype=torch.int32, device="cuda")
            native.nature_conv_fwd_split(layer, x, B, None, 0, 0, 0, q[layer - 1], b, y, relu_bits=bits)
            ys.append((y, bits))
        check(ys[0][0], fwd_ref(x, w, b, k, s, torch.float64), fwd_ref(x, w, b, k, s, torch.float32))
        assert torch.equal(ys[0][0], ys[1][0])
        words = ys[0][1].view(torch.int64).view(B * P, 1)  # bit c of the pixel's 64-bit pair = channel c > 0
        want = ((ys[0][0].reshape(B * P, 64) > 0).long() << torch.arange(64, device="cuda")).sum(1, keepdim=True)
        assert torch.equal(words, want)
    ds = []
    for _ in range(2):
        d = torch.full((B, 9, 9, 64), float("nan"), device="cuda")
        native.nature_conv_dgrad_split(3, g3, B, qd3, h2, d)
        ds.append(d)
    check(ds[0], dgrad3_ref(torch.float64), dgrad3_ref(torch.float32))
    assert torch.equal(ds[0], ds[1])


def _h1p_setup(B, seed, scale_w1=0.05):
    """Random frames through the conv1 forward writing H1P, with the weights packed by
    ppox_nature_pack_all (q1 carries the H1P exponent): (q, h1p, h1 as f32, E, weights)."""
    import native
    g = torch.Generator(device="cuda").manual_seed(seed)
    w1 = torch.randn(32, 4, 8, 8, device="cuda", generator=g) * scale_w1
    w2 = torch.randn(64, 32, 4, 4, device="cuda", generator=g) * 0.05
    w3 = torch.randn(64, 64, 3, 3, device="cuda", generator=g) * 0.05
    b1 = torch.randn(32, device="cuda", generator=g)
    q = {k: torch.empty(native.nature_split_pack_elems(k), dtype=torch.int16, device="cuda") for k in (1, 2, 3)}
    native.nature_pack_all(w1, w2, w3, None, None, q[1], q[2], q[3], None, None, None, None, b1=b1)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda", generator=g)
    h1p = torch.empty(B, 20, 20, 64, dtype=torch.int16, device="cuda")
    bits = torch.empty(B * 400, dtype=torch.int32, device="cuda")
    native.nature_conv1_fwd_planes(x, B, None, 0, 0, 28224, q[1], b1, h1p, relu_bits=bits)
    E = _h1p_exponent(w1, b1)
    return q, x, h1p, _h1_from_planes(h1p, E), E, (w1, b1, w2, w3), bits


@pytest.mark.parametrize("B", [1, 3, 37, 300, 2048])
def test_h1p_conv1_forward_is_split_of_f32_forward(B):
    """The conv1 forward writing H1P (its output split into two f16 planes in the epilogue, at the
    exponent ppox_nature_pack_all derived from the weights' bound) == the H1P split of the same
    kernel's f32 output, bitwise, plain rows and rollout rows (idx); its ReLU bitmask too."""
    import native
    q, x, h1p, h1, E, (w1, b1, _, _), bits = _h1p_setup(B, B)
    y = torch.empty(B, 20, 20, 32, device="cuda")
    native.nature_conv_fwd_split(1, x, B, None, 0, 0, 28224, q[1], b1, y)
    assert torch.equal(h1p, _h1_planes(y, E))
    assert torch.equal(bits, _relu_bits(y))
    assert float(y.abs().max()) * 2.0 ** E < 2 ** 15  # the bound holds
    T, N = 3, (B + 2) // 3
    frames = torch.randint(0, 256, (T, N, 4, 84, 84), dtype=torch.uint8, device="cuda")
    idx = torch.randperm(T * N, device="cuda")[:B].to(torch.int64)
    rows = torch.empty(B, 4, 84, 84, dtype=torch.uint8, device="cuda")
    native.gather_rows(frames, T, N, 28224, 28224, idx, B, rows)
    a, b = torch.empty_like(h1p), torch.empty_like(h1p)
    native.nature_conv1_fwd_planes(frames, B, idx, T, N, 0, q[1], b1, a)
    native.nature_conv1_fwd_planes(rows, B, None, 0, 0, 28224, q[1], b1, b)
    assert torch.equal(a, b)


@pytest.mark.parametrize("B", [1, 5, 300, 9001, 16384])
def test_h1p_conv2_fwd_and_wgrad_vs_fp64(B):
    """conv2 forward and the direct conv2 weight gradient on H1P vs float64 on the device, error no
    larger than the same math in f32 (x2 headroom): ragged and training-size batches (16,384 rows:
    64 samples per CU), the bias grad, each output's bitwise run-to-run determinism, the forward's
    ReLU bitmask; the weight gradient also per element against a dot-product error bound, on an
    output grad whose magnitudes spread over ~10 decades (log-normal)."""
    import native
    F = torch.nn.functional
    q, x, h1p, h1, E, (w1, b1, w2, w3), _ = _h1p_setup(B, 1000 + B)
    b2 = torch.randn(64, device="cuda") * 0.1
    cols = lambda dt: F.unfold(h1.permute(0, 3, 1, 2).to(dt), 4, stride=2)  # (B, 512 = (ci, ky, kx), 81)

    def check(got, r64, r32):
        scale = r64.abs().max()
        e_s = (got.double() - r64).abs().max() / scale
        e_f = (r32.double() - r64).abs().max() / scale
        assert torch.isfinite(got).all()
        assert e_s <= 2 * e_f + 1e-7, (float(e_s), float(e_f))
    ys = []
    for _ in range(2):
        y = torch.full((B, 9, 9, 64), float("nan"), device="cuda")
        bits = torch.zeros(B * 81 * 2, dtype=torch.int32, device="cuda")
        native.nature_conv2_fwd_planes(h1p, q[1], B, q[2], b2, y, relu_bits=bits)
        ys.append((y, bits))
    ref = lambda dt: (torch.einsum("ck,bkp->bpc", w2.reshape(64, -1).to(dt), cols(dt)) + b2.to(dt)).relu()
    check(ys[0][0].reshape(B, 81, 64), ref(torch.float64), ref(torch.float32))
    assert torch.equal(ys[0][0], ys[1][0]) and torch.equal(ys[0][1], ys[1][1])
    words = ys[0][1].view(torch.int64).view(B * 81, 1)
    want = ((ys[0][0].reshape(B * 81, 64) > 0).long() << torch.arange(64, device="cuda")).sum(1, keepdim=True)
    assert torch.equal(words, want)
    del ys
    gen = torch.Generator(device="cuda").manual_seed(B)
    for wide in (False, True):
        g2 = torch.randn(B, 9, 9, 64, device="cuda", generator=gen) * (torch.rand(B, 9, 9, 64, device="cuda",
                                                                                   generator=gen) > 0.3)
        if wide:
            g2 = g2 * torch.exp(3.0 * torch.randn(B, 9, 9, 64, device="cuda", generator=gen))
        ws = torch.empty(native.nature_conv2_wgrad_planes_workspace_bytes(B), dtype=torch.uint8, device="cuda")
        outs = []
        for _ in range(2):
            dw = torch.full((64, 32, 4, 4), float("nan"), device="cuda")
            db = torch.full((64,), float("nan"), device="cuda")
            native.nature_conv2_wgrad_planes(h1p, q[1], B, g2, ws, dw, db)
            outs.append((dw, db))
        assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
        dw, db = outs[0]
        gm = lambda dt: g2.reshape(B, 81, 64).to(dt)
        wref = lambda dt: torch.einsum("bkp,bpc->ck", cols(dt), gm(dt)).reshape(64, 32, 4, 4)
        r64, r32 = wref(torch.float64), wref(torch.float32)
        check(dw, r64, r32)
        rb = g2.double().sum(dim=(0, 1, 2))
        assert ((db.double() - rb).abs().max() / rb.abs().max()).item() < 1e-5
        # per element: |error| within twice the f32 GEMM's worst multiple of 2^-24 sum |x||g| (+ 4),
        # plus the split representation's floor: an operand value below 2^-17 of its tensor's max
        # keeps an absolute error of at most 2^-39 of that max, i.e. per output element
        # 2^-39 (max|g| sum |x| + max|x| sum |g|)
        c64, g64 = cols(torch.float64), gm(torch.float64)
        S = torch.einsum("bkp,bpc->ck", c64.abs(), g64.abs()).reshape(64, 32, 4, 4) * 2.0 ** -24
        floor = 2.0 ** -39 * (g64.abs().max() * c64.abs().sum(dim=(0, 2))[None, :] +
                              c64.abs().max() * g64.abs().sum(dim=(0, 1))[:, None]).reshape(64, 32, 4, 4)
        q_f = ((r32.double() - r64).abs() / S.clamp_min(1e-300)).max().item()
        excess = (dw.double() - r64).abs() - (2 * q_f + 4) * S - 2 * floor
        assert excess.max().item() <= 0, (wide, excess.max().item(), q_f)


@pytest.mark.parametrize("B", [3, 301, 16384])
def test_conv2_dgrad_counted_waits_equal_vmcnt0(B, monkeypatch):
    """The persistent conv2 dgrad's counted vmcnt waits (derived from its per-step memory
    operation counts, csrc/conv.hip C2_WAIT_I0*) against the same kernel with every wait a full
    vmcnt(0) (PPOX_COLP_VMCNT0=1): bitwise equal — a wait that let a tap DMA land late would read
    a stale LDS tap and change the result."""
    import native
    torch.manual_seed(B)
    w1 = torch.randn(32, 4, 8, 8, device="cuda") * 0.02
    w2 = torch.randn(64, 32, 4, 4, device="cuda") * 0.05
    w3 = torch.randn(64, 64, 3, 3, device="cuda") * 0.05
    q = {k: torch.empty(native.nature_split_pack_elems(k), dtype=torch.int16, device="cuda") for k in (1, 2, 3, 12, 13)}
    native.nature_pack_split(w1, w2, w3, q[1], q[2], q[3], q[12], q[13])
    g = torch.randn(B, 9, 9, 64, device="cuda")
    bits = torch.randint(-2 ** 31, 2 ** 31 - 1, (B * 400,), dtype=torch.int32, device="cuda")
    outs = []
    for safe in ("0", "1"):
        monkeypatch.setenv("PPOX_COLP_VMCNT0", safe)
        o = torch.full((B, 20, 20, 32), float("nan"), device="cuda")
        native.nature_conv_dgrad_split(2, g, B, q[12], None, o, relu_bits=bits)
        outs.append(o)
    assert torch.isfinite(outs[0]).all() and torch.equal(outs[0], outs[1])


def _fp64_check(got, r64, r32, what):
    """normwise error vs float64 no larger than the same math in f32 (x2 headroom)"""
    scale = r64.abs().max()
    e_s = (got.double() - r64).abs().max() / scale
    e_f = (r32.double() - r64).abs().max() / scale
    assert torch.isfinite(got).all(), what
    assert e_s <= 2 * e_f + 1e-7, (what, float(e_s), float(e_f))


@pytest.mark.parametrize("B", [9001, 16384])
def test_conv1_split_training_size_vs_fp64(B):
    """The conv1 ops at training-size batches, reading their rows from step-major rollout frames
    through the minibatch index (the bench's form): the persistent forward writing H1P and the
    weight gradient (split-K over ~2,048-pixel slabs, fixed-order reduce) vs float64 on the device,
    no larger than f32 math's error (x2), bitwise run-to-run; the weight gradient also per element
    on a log-normal output grad (the f32 dot-product bound + the split floor, as
    test_h1p_conv2_fwd_and_wgrad_vs_fp64)."""
    import native
    F = torch.nn.functional
    torch.manual_seed(B)
    T, N = 64, (B + 63) // 64 + 3
    frames = torch.randint(0, 256, (T, N, 4, 84, 84), dtype=torch.uint8, device="cuda")
    idx = torch.randperm(T * N, device="cuda")[:B].to(torch.int64)
    w1 = torch.randn(32, 4, 8, 8, device="cuda") * 0.02
    b1 = torch.randn(32, device="cuda") * 0.1
    w2, w3 = torch.randn(64, 32, 4, 4, device="cuda") * 0.05, torch.randn(64, 64, 3, 3, device="cuda") * 0.05
    q = {k: torch.empty(native.nature_split_pack_elems(k), dtype=torch.int16, device="cuda") for k in (1, 2, 3)}
    native.nature_pack_all(w1, w2, w3, None, None, q[1], q[2], q[3], None, None, None, None, b1=b1)
    E = _h1p_exponent(w1, b1)
    outs = []
    for _ in range(2):
        h1p = torch.empty(B, 20, 20, 64, dtype=torch.int16, device="cuda")
        native.nature_conv1_fwd_planes(frames, B, idx, T, N, 0, q[1], b1, h1p)
        outs.append(h1p)
    assert torch.equal(outs[0], outs[1])
    rows = frames.permute(1, 0, 2, 3, 4).reshape(T * N, 4, 84, 84)[idx]  # env-major row i = n * T + t
    ref = lambda dt: F.conv2d(rows.to(dt), w1.to(dt), b1.to(dt), stride=4).relu().permute(0, 2, 3, 1)
    _fp64_check(_h1_from_planes(outs[0], E), ref(torch.float64), ref(torch.float32), "conv1 fwd")
    del outs
    gen = torch.Generator(device="cuda").manual_seed(B + 1)
    for wide in (False, True):
        g1 = torch.randn(B, 20, 20, 32, device="cuda", generator=gen) * (torch.rand(B, 20, 20, 32, device="cuda",
                                                                                    generator=gen) > 0.5)
        if wide:
            g1 = g1 * torch.exp(3.0 * torch.randn(B, 20, 20, 32, device="cuda", generator=gen))
        ws = torch.empty(native.nature_wgrad_split_workspace_bytes(1, B), dtype=torch.uint8, device="cuda")
        res = []
        for _ in range(2):
            dw, db = torch.full_like(w1, float("nan")), torch.full_like(b1, float("nan"))
            native.nature_conv_wgrad_split_idx(1, frames, B, idx, T, N, g1, ws, dw, db)
            res.append((dw, db))
        assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
        dw, db = res[0]
        gn = g1.permute(0, 3, 1, 2)
        wref = lambda dt: torch.nn.grad.conv2d_weight(rows.to(dt), w1.shape, gn.to(dt), stride=4)
        r64, r32 = wref(torch.float64), wref(torch.float32)
        _fp64_check(dw, r64, r32, f"conv1 wgrad wide={wide}")
        rb = g1.double().sum(dim=(0, 1, 2))
        assert ((db.double() - rb).abs().max() / rb.abs().max()).item() < 1e-5
        # per element: frames are exact (one f16 plane), so only G carries the split floor
        S = torch.nn.grad.conv2d_weight(rows.double(), w1.shape, gn.double().abs(), stride=4) * 2.0 ** -24
        floor = 2.0 ** -39 * g1.double().abs().max() * torch.nn.grad.conv2d_weight(
            rows.double(), w1.shape, torch.ones_like(gn, dtype=torch.float64), stride=4)
        q_f = ((r32.double() - r64).abs() / S.clamp_min(1e-300)).max().item()
        excess = (dw.double() - r64).abs() - (2 * q_f + 4) * S - 2 * floor
        assert excess.max().item() <= 0, (wide, excess.max().item(), q_f)


@pytest.mark.parametrize("B", [1, 2, 3, 255, 257, 2048])
def test_conv1_wgrad_direct_ragged_vs_fp64(B):
    """The direct conv1 weight gradient (wgrad1_frames_kernel: one workgroup per CU over runs of whole
    samples in half-sample units, frames phase-split in LDS, two parity slabs per workgroup) at batches
    below, at and above one sample per CU: vs float64 within 2x f32 math's error, per element within
    the f32 dot-product bound + the split floor, the bias exact to 1e-5, bitwise run to run and
    through the rollout index (env-major rows of step-major frames) == on gathered rows."""
    import native
    F = torch.nn.functional
    torch.manual_seed(B + 7)
    T, N = 16, (B + 15) // 16 + 1
    frames = torch.randint(0, 256, (T, N, 4, 84, 84), dtype=torch.uint8, device="cuda")
    idx = torch.randperm(T * N, device="cuda")[:B].to(torch.int64)
    rows = frames.permute(1, 0, 2, 3, 4).reshape(T * N, 4, 84, 84)[idx].contiguous()
    w1 = torch.empty(32, 4, 8, 8, device="cuda")
    b1 = torch.empty(32, device="cuda")
    g1 = torch.randn(B, 20, 20, 32, device="cuda") * (torch.rand(B, 20, 20, 32, device="cuda") > 0.3)
    g1 = g1 * torch.exp(2.0 * torch.randn(B, 20, 20, 32, device="cuda"))
    ws = torch.empty(native.nature_wgrad_split_workspace_bytes(1, B), dtype=torch.uint8, device="cuda")
    res = []
    for i in range(3):
        dw, db = torch.full_like(w1, float("nan")), torch.full_like(b1, float("nan"))
        if i < 2:
            native.nature_conv_wgrad_split_idx(1, frames, B, idx, T, N, g1, ws, dw, db)
        else:
            native.nature_conv_wgrad_split(1, rows, B, 28224, g1, ws, dw, db)
        res.append((dw, db))
    for d in res[1:]:
        assert torch.equal(res[0][0], d[0]) and torch.equal(res[0][1], d[1])
    dw, db = res[0]
    gn = g1.permute(0, 3, 1, 2)
    wref = lambda dt: torch.nn.grad.conv2d_weight(rows.to(dt), w1.shape, gn.to(dt), stride=4)
    r64, r32 = wref(torch.float64), wref(torch.float32)
    _fp64_check(dw, r64, r32, f"conv1 wgrad direct B={B}")
    rb = g1.double().sum(dim=(0, 1, 2))
    assert ((db.double() - rb).abs().max() / rb.abs().max()).item() < 1e-5
    S = torch.nn.grad.conv2d_weight(rows.double(), w1.shape, gn.double().abs(), stride=4) * 2.0 ** -24
    floor = 2.0 ** -39 * g1.double().abs().max() * torch.nn.grad.conv2d_weight(
        rows.double(), w1.shape, torch.ones_like(gn, dtype=torch.float64), stride=4)
    q_f = ((r32.double() - r64).abs() / S.clamp_min(1e-300)).max().item()
    excess = (dw.double() - r64).abs() - (2 * q_f + 4) * S - 2 * floor
    assert excess.max().item() <= 0, (excess.max().item(), q_f)


@pytest.mark.parametrize("B", [9001, 16384])
def test_conv2_dgrad_persistent_training_size_vs_fp64(B):
    """The persistent col2im conv2 dgrad at training-size batches (3,001 / 5,462 sample triples over
    one workgroup per CU; conv1's ReLU mask from the forward's bitmask) vs float64 on the device:
    no larger than f32 math's error (x2), bitwise run-to-run, nothing written past the batch."""
    import native
    torch.manual_seed(B)
    w1 = torch.randn(32, 4, 8, 8, device="cuda") * 0.05
    w2 = torch.randn(64, 32, 4, 4, device="cuda") * 0.05
    w3 = torch.randn(64, 64, 3, 3, device="cuda") * 0.05
    q = {k: torch.empty(native.nature_split_pack_elems(k), dtype=torch.int16, device="cuda") for k in (1, 2, 3, 12, 13)}
    native.nature_pack_split(w1, w2, w3, q[1], q[2], q[3], q[12], q[13])
    g = torch.randn(B, 9, 9, 64, device="cuda")
    h1 = torch.relu(torch.randn(B, 20, 20, 32, device="cuda"))
    bits = _relu_bits(h1)
    outs = []
    for _ in range(2):
        o = torch.full((B + 1, 20, 20, 32), 7.0, device="cuda")
        native.nature_conv_dgrad_split(2, g, B, q[12], None, o, relu_bits=bits)
        outs.append(o)
    assert torch.equal(outs[0], outs[1]) and bool((outs[0][B] == 7.0).all())
    gn, mask = g.permute(0, 3, 1, 2), (h1.permute(0, 3, 1, 2) > 0)
    ref = lambda dt: (torch.nn.grad.conv2d_input((B, 32, 20, 20), w2.to(dt), gn.to(dt), stride=2) * mask).permute(
        0, 2, 3, 1)
    _fp64_check(outs[0][:B], ref(torch.float64), ref(torch.float32), "conv2 dgrad")


def test_current_stream_orders_like_torch():
    """convs.current_stream (the backward's cheap current-stream lookup) is torch's current stream:
    a side-stream read forked after a long main-stream write sees the write, and the main stream
    after the join sees the side stream's result (convs.fork / join)."""
    import convs
    dev = torch.device("cuda", 0)
    cur = convs.current_stream(dev)
    assert cur.cuda_stream == torch.cuda.current_stream().cuda_stream
    side = convs.side_stream(dev)
    a = torch.randn(4096, 4096, device=dev)
    x = torch.zeros(1, device=dev)
    torch.cuda.synchronize()
    for _ in range(20):
        a = a @ a * 1e-3
    x.fill_(1.0)
    convs.fork(side, cur)
    with torch.cuda.stream(side):
        y = x * 2
    convs.join(side, cur)
    z = y + 1
    torch.cuda.synchronize()
    assert float(y) == 2.0 and float(z) == 3.0
    s2 = torch.cuda.Stream()
    with torch.cuda.stream(s2):
        assert convs.current_stream(dev).cuda_stream == s2.cuda_stream


def test_big_minibatch_offsets_are_64bit():
    """the direct conv2 weight gradient (H1P samples 51,200 B apart) and the persistent
    conv2 dgrad (G rows 256 B apart) address their operands in 64 bits, so a full-rollout minibatch
    (batch_size=None, buffer.py:249) past the old 32-bit limits (83,886 / 207,126 rows) trains: the
    samples beyond the limit contribute what they contribute alone (same operand scales)."""
    import native
    g = torch.Generator(device="cuda").manual_seed(5)
    w1 = torch.randn(32, 4, 8, 8, device="cuda", generator=g) * 0.02
    w2 = torch.randn(64, 32, 4, 4, device="cuda", generator=g) * 0.05
    w3 = torch.randn(64, 64, 3, 3, device="cuda", generator=g) * 0.05
    b1 = torch.randn(32, device="cuda", generator=g)
    q = {k: torch.empty(native.nature_split_pack_elems(k), dtype=torch.int16, device="cuda") for k in (1, 2, 3, 12)}
    native.nature_pack_all(w1, w2, w3, None, None, q[1], q[2], q[3], q[12], None, None, None, b1=b1)
    B, cut = 90000, 80000
    h1p = torch.zeros(B, 20, 20, 64, dtype=torch.int16, device="cuda")  # hi planes random, lo planes zero
    h1p.view(B, 400, 64)[:, :, :32] = (torch.rand(B, 400, 32, device="cuda", generator=g) * 100).half().view(torch.int16)
    g2 = torch.randn(B, 9, 9, 64, device="cuda", generator=g)
    am = native.amax_table(1, "cuda")[0]
    native.amax(g2, am)
    ws = torch.empty(native.nature_conv2_wgrad_planes_workspace_bytes(B), dtype=torch.uint8, device="cuda")
    res = []
    for lo, hi in ((0, B), (0, cut), (cut, B)):
        dw, db = torch.empty(64, 32, 4, 4, device="cuda"), torch.empty(64, device="cuda")
        native.nature_conv2_wgrad_planes(h1p[lo:hi], q[1], hi - lo, g2[lo:hi], ws, dw, db, amax_g=am)
        res.append((dw.double(), db.double()))
    for k in range(2):
        whole, parts = res[0][k], res[1][k] + res[2][k]
        assert (whole - parts).abs().max().item() <= 1e-5 * whole.abs().max().item()
    del h1p, ws
    B = 210000
    g2 = torch.randn(B, 9, 9, 64, device="cuda", generator=g)
    bits = torch.randint(-2 ** 31, 2 ** 31 - 1, (B * 400,), dtype=torch.int32, device="cuda", generator=g)
    native.amax(g2, am)
    out = torch.empty(B, 20, 20, 32, device="cuda")
    native.nature_conv_dgrad_split(2, g2, B, q[12], None, out, amax_g=am, relu_bits=bits)
    tail = torch.empty(30, 20, 20, 32, device="cuda")
    native.nature_conv_dgrad_split(2, g2[-30:], 30, q[12], None, tail, amax_g=am, relu_bits=bits[-30 * 400:])
    assert torch.equal(out[-30:], tail)
