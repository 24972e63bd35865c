"""K11 ICM kernels (csrc/icm.hip, ppo-exploration_amd/icm.py) vs a float64 torch autograd of
the reference module (models.py:270-320) and loss (ppo.py:684-688); and PPO_ICM on the
kernels vs PPO_ICM on the torch module (PPOX_ICM_NATIVE=0).  GPU box only.

Tolerances: the encoder's Linear(K, 32) runs split-f16 (every product exact, f32
accumulation), so its error vs fp64 is held to that of torch's own f32 GEMM (x2) on the same
rows; gradients / losses are compared against fp64 with a per-tensor bound (2e-5 of the
tensor's largest entry — fp32-class: the f32 product-sum errors, not f16's 5e-4)."""
import copy

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

K_ATARI = 4 * 84 * 84


def _module(K, A, seed):
    from env import Discrete
    from models import FlatParams, IntrinsicCuriosityModule
    from util import ActionConverter
    torch.manual_seed(seed)
    icm = IntrinsicCuriosityModule(K, ActionConverter(Discrete(A)), 32)
    ref = copy.deepcopy(icm).double()
    flat = FlatParams(icm, "cuda")
    return icm, ref, flat


def _native(icm, flat, K):
    import icm as icm_native
    assert icm_native.supported(icm, flat, (K,), torch.uint8)
    return icm_native.NativeIcm(icm, flat, K)


def _frames(M, K, seed):
    g = np.random.default_rng(seed)
    return g.integers(0, 256, size=(M, K), dtype=np.uint8)


def _ref_grads(ref):
    return [p.grad.detach().numpy().reshape(-1) for p in ref.parameters()]


@pytest.mark.parametrize("M", [1, 33, 512, 1000, 2048, 4100])
def test_encode_vs_fp64(M):
    K, A = K_ATARI, 4
    icm, ref, flat = _module(K, A, 3)
    nat = _native(icm, flat, K)
    x = _frames(M, K, M)
    xd = torch.from_numpy(x).cuda()
    pre1, phi = nat.encode(xd)
    x64 = torch.from_numpy(x).double()
    with torch.no_grad():
        pre_ref = ref.state_encoder[0](x64)
        phi_ref = ref.state_encoder(x64)
        pre_f32 = F.linear(xd.float(), icm.state_encoder[0].weight, icm.state_encoder[0].bias).cpu().double()
    e_ours = (pre1.cpu().double() - pre_ref).abs().max().item()
    e_f32 = (pre_f32 - pre_ref).abs().max().item()
    assert e_ours <= max(2 * e_f32, 1e-6 * pre_ref.abs().max().item()), (e_ours, e_f32)
    scale = phi_ref.abs().max().item()
    np.testing.assert_allclose(phi.cpu().double().numpy(), phi_ref.numpy(), rtol=0, atol=1e-5 * scale)


def test_encode_per_feature_scale_vs_fp64():
    """W1 rows spanning 1e-6 .. 1e3 (bias zero): each feature's split uses its own exponent, so
    every output column is held to 2x torch's f32 error on that column (and 1e-6 of its own
    scale), not to the largest column's."""
    K, A, M = K_ATARI, 4, 300
    icm, ref, flat = _module(K, A, 8)
    w = icm.state_encoder[0].weight
    with torch.no_grad():
        w.mul_(torch.logspace(-6, 3, 32, device=w.device)[:, None])
        icm.state_encoder[0].bias.zero_()
        ref.state_encoder[0].weight.copy_(w.detach().cpu().double())
        ref.state_encoder[0].bias.zero_()
    nat = _native(icm, flat, K)
    x = _frames(M, K, 21)
    xd = torch.from_numpy(x).cuda()
    pre1, _ = nat.encode(xd)
    with torch.no_grad():
        pre_ref = ref.state_encoder[0](torch.from_numpy(x).double()).numpy()
        pre_f32 = F.linear(xd.float(), w).cpu().double().numpy()
    e_ours = np.abs(pre1.cpu().double().numpy() - pre_ref).max(0)
    e_f32 = np.abs(pre_f32 - pre_ref).max(0)
    scale = np.abs(pre_ref).max(0)
    assert (e_ours <= np.maximum(2 * e_f32, 1e-6 * scale)).all(), (e_ours / scale, e_f32 / scale)


def test_encode_rollout_rows_equal_gathered():
    """RolloutRows (env-major idx into step-major frames) read in place == the gathered rows."""
    import convs
    K, A, T, N = K_ATARI, 6, 8, 24
    icm, _, flat = _module(K, A, 4)
    nat = _native(icm, flat, K)
    g = torch.Generator().manual_seed(1)
    frames = torch.randint(0, 256, (T, N, 4, 84, 84), dtype=torch.uint8, generator=g).cuda()
    idx = torch.randperm(T * N, generator=g)[:100].cuda()
    rows = (idx % T) * N + idx // T
    _, phi_r, rn = nat.encode(convs.RolloutRows(frames, idx), "a", rowno=True)
    _, phi_g = nat.encode(frames.reshape(T * N, K)[rows].contiguous(), "b")
    assert torch.equal(phi_r, phi_g)
    assert torch.equal(rn.long(), rows)


def _minibatch(K, A, B, seed, beta=0.2):
    icm, ref, flat = _module(K, A, seed)
    nat = _native(icm, flat, K)
    x = _frames(B, K, seed + 100)
    acts = np.random.default_rng(seed).integers(0, A, size=B).astype(np.int32)
    acc = torch.zeros(1, dtype=torch.float64, device="cuda")

    class One:
        enabled = False
    flat.grad.fill_(float("nan"))  # every gradient must be written
    nat.train_minibatch(torch.from_numpy(x).cuda(), torch.from_numpy(acts).cuda(), None, B, beta, One(), acc)
    ours = flat.grad[:flat.n].cpu().double().numpy()
    # fp64 reference: ppo.py:684-688 on the same rows
    x64 = torch.from_numpy(x).double()
    a = torch.from_numpy(acts).long()
    phi = ref.state_encoder(x64)
    s, n, a0 = phi[:-1], phi[1:], a[:-1]
    ahat = ref.inverse_model(torch.cat((s, n), 1))
    nhat = ref.forward_model(torch.cat((s, ref.action_encoder(a0)), 1))
    loss = (1 - beta) * F.cross_entropy(ahat, a0) + beta * F.mse_loss(nhat, n)
    loss.backward()
    return ours, _ref_grads(ref), [p.numel() for p in ref.parameters()], acc.item(), loss.item(), flat


@pytest.mark.parametrize("K,A,B", [(K_ATARI, 4, 2048), (K_ATARI, 4, 33), (K_ATARI, 18, 300), (2048, 9, 2)])
def test_minibatch_grads_vs_fp64(K, A, B):
    ours, ref, sizes, loss, loss_ref, _ = _minibatch(K, A, B, 7)
    assert np.isfinite(ours).all()
    off = 0
    names = ["W1", "b1", "W2", "b2", "Wf1", "bf1", "Wf2", "bf2", "Wi1", "bi1", "Wi2", "bi2", "Wae"]
    for name, g_ref, k in zip(names, ref, sizes):
        g = ours[off:off + k]
        off += k
        scale = max(np.abs(g_ref).max(), 1e-30)
        err = np.abs(g - g_ref).max()
        assert err <= 2e-5 * scale, (name, err, scale)
    np.testing.assert_allclose(loss, loss_ref, rtol=1e-5)


def test_minibatch_one_row_has_no_pairs():
    """B = 1 (the last minibatch of an uneven split): no pairs -> zero gradients everywhere;
    the loss is the reference's mean over zero pairs (nan)."""
    ours, _, _, loss, _, _ = _minibatch(2048, 4, 1, 9)
    assert (ours == 0).all()
    assert np.isnan(loss)


def test_minibatch_deterministic():
    a = _minibatch(K_ATARI, 4, 2048, 11)[0]
    b = _minibatch(K_ATARI, 4, 2048, 11)[0]
    assert np.array_equal(a, b)


@pytest.mark.parametrize("B", [2048, 33])
def test_minibatch_sharded_path_one_rank_matches_one_process(B):
    """The world > 1 branch of train_minibatch (features + actions summed into minibatch positions,
    the owned positions as the pair list — B - 1 among them, skipped by the kernel — dL/dphi summed
    back) on one rank whose rows arrive in a shuffled order: the same gradients and loss as the
    one-process branch on the rows in minibatch order."""
    K, A, seed = K_ATARI, 4, 13
    icm, _, flat = _module(K, A, seed)
    nat = _native(icm, flat, K)
    x = torch.from_numpy(_frames(B, K, seed + 100)).cuda()
    acts = torch.from_numpy(np.random.default_rng(seed).integers(0, A, size=B).astype(np.int32)).cuda()

    class One:
        enabled = False

    class Ranks:  # one rank with the data-parallel branch on (its sums are the identity)
        enabled = True

        @staticmethod
        def all_reduce_(t):
            return t
    acc = torch.zeros(1, dtype=torch.float64, device="cuda")
    nat.train_minibatch(x, acts, None, B, 0.2, One(), acc)
    want, want_loss = flat.grad[:flat.n].clone(), acc.item()
    order = torch.randperm(B, generator=torch.Generator().manual_seed(5)).cuda()  # row i sits at pos[i]
    inv = torch.empty_like(order)
    inv[order] = torch.arange(B, device="cuda")
    acc.zero_()
    flat.grad.fill_(float("nan"))
    nat.train_minibatch(x[order].contiguous(), acts[order].contiguous(), order, B, 0.2, Ranks(), acc)
    got = flat.grad[:flat.n]
    assert torch.isfinite(got).all()
    scale = want.abs().max().item()
    assert (got - want).abs().max().item() <= 1e-6 * scale
    np.testing.assert_allclose(acc.item(), want_loss, rtol=1e-6)


def test_pair_list_with_last_position():
    """ppox_icm_pair_backward with a pair list: dS / dN are output-only (pre-filled with
    NaN here, every element written), a listed B - 1 is skipped, and n_pairs may then be B: the list
    [all positions] gives the same dS / dN as the list without B - 1 (n_pairs = B - 1), and a partial
    list leaves the unlisted rows zero."""
    import native
    from icm import H
    K, A, B = K_ATARI, 4, 37
    icm, _, flat = _module(K, A, 21)
    nat = _native(icm, flat, K)
    g = torch.Generator(device="cuda").manual_seed(3)
    fa = torch.randn(B * (H + 1), device="cuda", generator=g)
    fa[B * H:] = torch.randint(0, A, (B,), device="cuda", generator=g).float()
    partials = torch.empty(native.icm_partials_bytes(B, A) // 4, device="cuda")

    def run(pairs):
        dS = torch.full((B, H), float("nan"), device="cuda")
        dN = torch.full((B, H), float("nan"), device="cuda")
        native.icm_pair_backward(fa, B, None, None, pairs, pairs.numel(), B - 1, A, 0.2, nat.seg, dS, dN, partials)
        torch.cuda.synchronize()
        return dS, dN
    every = torch.randperm(B, generator=torch.Generator().manual_seed(4)).cuda()
    dS_all, dN_all = run(every)
    dS_ref, dN_ref = run(every[every != B - 1].contiguous())
    assert torch.isfinite(dS_all).all() and torch.isfinite(dN_all).all()
    assert torch.equal(dS_all, dS_ref) and torch.equal(dN_all, dN_ref)
    part = torch.tensor([B - 1, 0, 5], device="cuda")
    dS_p, dN_p = run(part)
    listed = torch.zeros(B, dtype=torch.bool, device="cuda")
    listed[part] = True
    assert (dS_p[~listed] == 0).all()
    assert torch.equal(dS_p[0], dS_all[0]) and torch.equal(dS_p[5], dS_all[5])
    assert (dS_p[B - 1] == 0).all()
    # dN holds the pair's second row: rows 1 and 6 get pairs 0 and 5
    sec = torch.zeros(B, dtype=torch.bool, device="cuda")
    sec[torch.tensor([1, 6], device="cuda")] = True
    assert (dN_p[~sec] == 0).all()
    assert torch.equal(dN_p[1], dN_all[1]) and torch.equal(dN_p[6], dN_all[6])


@pytest.mark.parametrize("N,A", [(512, 4), (77, 18)])
def test_int_reward_vs_fp64(N, A):
    """ppo.py:629-631: int_reward(s, s', a) = clamp(mean((fwd(phi(s), a) - phi(s'))^2), -5, 5),
    rewards <- (1 - eta) rewards + eta int_reward."""
    K, eta = K_ATARI, 0.05
    icm, ref, flat = _module(K, A, 5)
    nat = _native(icm, flat, K)
    s, s2 = _frames(N, K, 1), _frames(N, K, 2)
    acts = np.random.default_rng(3).integers(0, A, size=N).astype(np.int32)
    rew = np.random.default_rng(4).random(N).astype(np.float32)
    phs = nat.encode(torch.from_numpy(s).cuda(), "s")[1]
    phn = nat.encode(torch.from_numpy(s2).cuda(), "n")[1]
    r = torch.from_numpy(rew).cuda()
    ir = torch.empty(N, device="cuda")
    nat.int_reward(phs, phn, torch.from_numpy(acts).cuda(), r, eta, ir)
    with torch.no_grad():
        ir_ref = ref.int_reward(torch.from_numpy(s).double(), torch.from_numpy(s2).double(),
                                torch.from_numpy(acts).long()).numpy()
    np.testing.assert_allclose(ir.cpu().numpy(), ir_ref, rtol=1e-4, atol=1e-6 * max(1.0, np.abs(ir_ref).max()))
    np.testing.assert_allclose(r.cpu().numpy(), (1 - eta) * rew + eta * ir_ref, rtol=1e-5, atol=1e-6)


def test_ppo_icm_native_matches_torch_module(monkeypatch):
    """PPO_ICM (Breakout frames) collect + train with the ICM on K11 vs on the torch module:
    same rollout rewards (int rewards mixed in) and ICM weights within fp32-class tolerance."""
    import logger
    import ppo
    cfg = dict(env_id="BreakoutNoFrameskip-v4", n_envs=8, nstep=16, batch_size=40, n_epochs=2, seed=3, quiet=True)
    logger.configure("ICM", "BreakoutNoFrameskip-v4", quiet=True)
    runs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("PPOX_ICM_NATIVE", flag)
        np.random.seed(5)
        torch.manual_seed(5)
        alg = ppo.PPO_ICM(**cfg)
        assert (alg._icm_native is not None) == (flag == "1")
        alg.collect_samples()
        rew = alg.rollout.rewards.cpu().numpy().copy()
        alg.train()
        runs.append((rew, alg.icm_flat.data[:alg.icm_flat.n].cpu().numpy(), alg.icm_accum.item(),
                     alg.flat.data[:alg.flat.n].cpu().numpy()))
    (r1, w1, l1, p1), (r0, w0, l0, p0) = runs
    np.testing.assert_allclose(r1, r0, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(l1, l0, rtol=1e-4)
    # Adam normalises each weight's step: near-zero gradients can land an lr-sized step
    # apart, so the bulk is held to rtol 1e-4 and at most 1e-4 of the weights may differ more
    bad = np.abs(w1 - w0) > 1e-4 * np.abs(w0) + 1e-5
    assert bad.mean() <= 1e-4, (int(bad.sum()), w1.size)
    # and no weight further apart than every Adam step (lr 3e-4, 2 epochs x 4 minibatches) in opposite directions
    np.testing.assert_allclose(w1, w0, rtol=1e-4, atol=2 * 3e-4 * 8)
    bad = np.abs(p1 - p0) > 1e-4 * np.abs(p0) + 1e-5
    assert bad.mean() <= 1e-4, (int(bad.sum()), p1.size)
