"""End-to-end parity of the product API (ppo.PPO / buffer.RolloutStorage) on the GPU
against the reference's own recorded runs (tests/golden/train_ppo.npz) and the oracle."""
import numpy as np
import pytest
import torch

import f64_pass
from oracle import models as OM
from oracle.algos import OraclePPO
from replay_env import ReplayVecEnv, space_from_code

pytestmark = pytest.mark.gpu


def _space(E, code):
    """fixture space code -> the product's space type (n > 0: Discrete(n); -k: Box((k,)))."""
    return E.Discrete(int(code)) if code > 0 else E.Box((int(-code),))


def _load_weights(module, f, prefix):
    sd = module.state_dict()
    with torch.no_grad():
        for k, v in sd.items():
            v.copy_(torch.from_numpy(f[prefix + k]).to(v.device))


def _train_kwargs(name):
    """'cartpole' (BASELINE config 1: 8 envs x 128 steps, hidden 128, batch 128, 10 epochs)
    ran with the reference's defaults; the other train_ppo cases with max_grad_norm 0.5."""
    return {} if name == "cartpole" else dict(max_grad_norm=0.5, ent_coef=0.01, vf_coef=1.0)


@pytest.mark.parametrize("name", ["disc2", "disc4sat", "disc18", "box2", "cartpole"])
def test_ppo_train_matches_reference_run(golden, name):
    """Same rollout + same weights + same numpy seed => product train() reproduces the
    reference's post-update weights (ppo.py:200-259).  box2: the Normal head with the
    reference's f64 log_prob / ratio / surrogate (models.py:66-71).  cartpole: BASELINE
    config 1 at its full size (80 optimizer steps)."""
    import ppo
    import env as E
    f = golden("train_ppo")
    p = name + "_"
    D, N, T, B, E_, H, seed, code = (int(x) for x in f[p + "cfg"])
    # oracle regenerates the reference rollout bit-for-bit (pinned by test_oracle_golden)
    renv = ReplayVecEnv(f[p + "env_obs"], f[p + "env_rew"], f[p + "env_done"], space_from_code(code))
    np.random.seed(seed)
    torch.manual_seed(seed)
    orc = OraclePPO(renv, nstep=T, batch_size=B, n_epochs=E_, hidden_size=H, **_train_kwargs(name))
    if name == "disc4sat":
        with torch.no_grad():
            orc.net.actor[-1].weight.mul_(60.0)
    orc.collect()
    ro_ref = orc.rollout
    # product on the GPU
    np.random.seed(seed)  # RolloutStorage draws randn(16, D) at construction (buffer.py:137)
    denv = E.DeviceVecEnv("custom", N, obs_dim=D, action_space=_space(E, code))
    alg = ppo.PPO(env_id="custom", env=denv, n_envs=N, nstep=T, batch_size=B, n_epochs=E_, hidden_size=H,
                  quiet=True, **_train_kwargs(name))
    _load_weights(alg.policy.net, f, p + "w0_")
    ro = alg.rollout
    for t in range(T):
        ro.add(ro_ref.obs[t], ro_ref.actions[t], ro_ref.rewards[t], ro_ref.values[t], ro_ref.masks[t],
               ro_ref.log_probs[t])
    ro.compute_returns_and_advantages(ro_ref.values[T - 1], ro_ref.masks[T - 1])
    np.testing.assert_array_equal(ro.advantages.cpu().numpy(), ro_ref.adv)
    alg.train()
    sd = alg.policy.net.state_dict()
    for k, v in sd.items():
        np.testing.assert_allclose(v.cpu().numpy(), f[p + "w1_" + k], rtol=2e-5, atol=2e-6, err_msg=k)
    np.testing.assert_array_equal(np.random.get_state()[1], f[p + "np_state_after"])
    acc = alg.loss_accum.cpu().numpy()
    n = acc[5]
    np.testing.assert_allclose(acc[0] / n, f[p + "policy_gradient_loss"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(acc[1] / n, f[p + "value_loss"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(acc[2] / n, f[p + "entropy_loss"], rtol=1e-4, atol=1e-6)


def test_get_yields_reference_minibatches(golden):
    """buffer.get(): same permutation + env-major order as buffer.py:233-267."""
    import buffer
    import env as E
    f = golden("get_perm")
    p = "c0_"
    T, N, D, B, Ep, seed = (int(x) for x in f[p + "cfg"])
    np.random.seed(seed)
    st = buffer.RolloutStorage(T, N, E.Box((D,)), E.Discrete(4))
    obs = np.arange(T * N * D, dtype=np.float32).reshape(T, N, D)
    for t in range(T):
        st.add(obs[t], np.full((N, 1), t), np.zeros(N, np.float32), np.arange(N, dtype=np.float32) + 100 * t,
               np.zeros(N, bool), np.full((N, 1), float(t)))
    st.compute_returns_and_advantages(np.zeros(N, np.float32), np.zeros(N, bool))
    mb = 0
    for _ in range(Ep):
        for b in st.get(B):
            np.testing.assert_array_equal(b.observations.cpu().numpy(), f[p + f"obs{mb}"])
            np.testing.assert_array_equal(b.actions.cpu().numpy(), f[p + f"act{mb}"])
            np.testing.assert_array_equal(b.old_values.cpu().numpy(), f[p + f"oldv{mb}"])
            np.testing.assert_array_equal(b.old_log_probs.cpu().numpy(), f[p + f"oldlp{mb}"])
            np.testing.assert_array_equal(b.advantages.cpu().numpy(), f[p + f"adv{mb}"])
            np.testing.assert_array_equal(b.returns.cpu().numpy(), f[p + f"ret{mb}"])
            mb += 1
    assert mb == int(f[p + "nmb"])


def test_nature_cnn_forward_matches_oracle(golden):
    import models
    f = golden("cnn")
    torch.manual_seed(51)
    net = models.CnnActorCritic(4, 4)
    models.FlatParams(net, "cuda")
    x = torch.from_numpy(f["x"]).cuda()
    with torch.no_grad():
        logits, v, _ = net(x)
    np.testing.assert_allclose(logits.cpu().numpy(), f["logits"], rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(v.cpu().numpy(), f["value"][:, 0], rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("algo", ["PPO", "PPO_RND", "PPO_ICM"])
def test_atari_iteration_runs(algo):
    """One tiny Breakout/Montezuma iteration through every kernel: finite losses, params move."""
    import ppo
    import logger
    cls = getattr(ppo, algo)
    env_id = "MontezumaRevengeNoFrameskip-v4" if algo == "PPO_RND" else "BreakoutNoFrameskip-v4"
    kw = dict(rnd_start=4) if algo == "PPO_RND" else {}
    alg = cls(env_id=env_id, n_envs=8, nstep=16, batch_size=32, n_epochs=2, quiet=True, seed=3, **kw)
    w0 = alg.flat.data.clone()
    logger.configure("t", env_id, quiet=True)
    alg.collect_samples()
    assert torch.isfinite(alg.rollout.advantages).all()
    alg.train()
    acc = alg.loss_accum.cpu().numpy()
    assert acc[5] == 2 * 4 and np.isfinite(acc[:5]).all()
    assert not torch.equal(w0, alg.flat.data)
    alg.collect_samples()  # second rollout continues from slot T


def test_ppo_train_rollout_rows_equals_gathered():
    """The CNN minibatch read in place from the rollout (convs.RolloutRows) and the gathered
    minibatch (buffer._gather) give bitwise-identical post-train weights."""
    import ppo
    import logger
    res = []
    for force_gather in (False, True):
        np.random.seed(5)
        torch.manual_seed(5)
        alg = ppo.PPO(env_id="BreakoutNoFrameskip-v4", n_envs=8, nstep=16, batch_size=40, n_epochs=2, quiet=True,
                      seed=3)
        if force_gather:
            alg._train_obs = lambda ro, idx: ro._gather(ro.observations, idx)
        else:
            import convs
            assert isinstance(alg._train_obs(alg.rollout, torch.arange(4, device="cuda")), convs.RolloutRows)
        logger.configure("t", "BreakoutNoFrameskip-v4", quiet=True)
        alg.collect_samples()
        alg.train()
        res.append(alg.flat.data.clone())
    assert torch.equal(res[0], res[1])


def test_rnd_train_matches_reference_run(golden):
    """PPO_RND.train() (ppo.py:409-502: two normalised advantage streams, clipped int value
    loss, randn()<0.25-gated RND updates) on the reference's rollout."""
    import ppo
    import env as E
    from oracle.algos import OracleRND
    f = golden("train_rnd")
    p = "rnd_"
    D, N, T, B, E_, H, IH, seed, rnd_start = (int(x) for x in f[p + "cfg"])
    renv = ReplayVecEnv(f[p + "env_obs"], f[p + "env_rew"], f[p + "env_done"], space_from_code(3))
    np.random.seed(seed)
    torch.manual_seed(seed)
    orc = OracleRND(renv, nstep=T, batch_size=B, n_epochs=E_, hidden_size=H, int_hidden_size=IH,
                    rnd_start=rnd_start, max_grad_norm=0.5)
    orc.collect()
    r = orc.rollout
    np.random.seed(seed)
    alg = ppo.PPO_RND(env_id="custom", env=E.DeviceVecEnv("custom", N, obs_dim=D, action_space=E.Discrete(3)),
                      n_envs=N, nstep=T, batch_size=B, n_epochs=E_, hidden_size=H, int_hidden_size=IH,
                      rnd_start=rnd_start, max_grad_norm=0.5, quiet=True)
    _load_weights(alg.policy.net, f, p + "w0_")
    _load_weights(alg.rnd, f, p + "r0_")
    ro = alg.rollout
    for t in range(T):
        ro.add(r.obs[t], r.actions[t], r.rewards[t], r.int_rewards[t], r.values[t], r.int_values[t], r.masks[t],
               r.log_probs[t])
    ro.compute_returns_and_advantages(r.values[T - 1], r.int_values[T - 1], r.masks[T - 1])
    np.testing.assert_array_equal(ro.int_advantages.cpu().numpy(), r.iadv)
    alg.obs_rms._mean = torch.from_numpy(np.asarray(orc.obs_rms.mean, np.float64)).cuda()
    alg.obs_rms._var = torch.from_numpy(np.asarray(orc.obs_rms.var, np.float64)).cuda()
    alg.obs_rms.count = orc.obs_rms.count
    alg.train()
    for k, v in alg.policy.net.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), f[p + "w1_" + k], rtol=2e-5, atol=2e-6, err_msg=k)
    for k, v in alg.rnd.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), f[p + "r1_" + k], rtol=1e-4, atol=1e-5, err_msg=k)
    np.testing.assert_array_equal(np.random.get_state()[1], f[p + "np_state_after"])
    acc = alg.loss_accum.cpu().numpy()
    np.testing.assert_allclose(acc[4] / acc[5], f[p + "intrinsic_loss"], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("name,code", [("icm_disc", 3), ("icm_box", -2)])
def test_icm_train_matches_reference_run(golden, name, code):
    """PPO_ICM.train() (ppo.py:651-713) on the reference's rollout (Discrete: CrossEntropy
    inverse loss; Box: MSE inverse loss, util.py:61-69)."""
    import ppo
    import env as E
    from oracle.algos import OracleICM
    f = golden("train_icm")
    p = name + "_"
    D, N, T, B, E_, H, IH, seed = (int(x) for x in f[p + "cfg"])
    renv = ReplayVecEnv(f[p + "env_obs"], f[p + "env_rew"], f[p + "env_done"], space_from_code(code))
    np.random.seed(seed)
    torch.manual_seed(seed)
    orc = OracleICM(renv, nstep=T, batch_size=B, n_epochs=E_, hidden_size=H, int_hidden_size=IH,
                    max_grad_norm=0.5, int_rew_integration=0.1)
    orc.collect()
    r = orc.rollout
    np.random.seed(seed)
    alg = ppo.PPO_ICM(env_id="custom", env=E.DeviceVecEnv("custom", N, obs_dim=D, action_space=_space(E, code)),
                      n_envs=N, nstep=T, batch_size=B, n_epochs=E_, hidden_size=H, int_hidden_size=IH,
                      max_grad_norm=0.5, int_rew_integration=0.1, quiet=True)
    _load_weights(alg.policy.net, f, p + "w0_")
    _load_weights(alg.intrinsic_module, f, p + "i0_")
    ro = alg.rollout
    for t in range(T):
        ro.add(r.obs[t], r.actions[t], r.rewards[t], r.values[t], r.masks[t], r.log_probs[t])
    ro.compute_returns_and_advantages(r.values[T - 1], r.masks[T - 1])
    alg.train()
    for k, v in alg.policy.net.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), f[p + "w1_" + k], rtol=2e-5, atol=2e-6, err_msg=k)
    for k, v in alg.intrinsic_module.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), f[p + "i1_" + k], rtol=2e-5, atol=2e-6, err_msg=k)


def test_simhash_matches_reference(golden):
    """RolloutStorage(sim_hash=True).add (buffer.py:165-200): same A draw, rewards after the
    count bonus bit-exact vs the reference's own runs, table persisting across reset()."""
    import buffer
    import env as E
    f = golden("simhash")
    for k in range(3):
        p = f"s{k}_"
        T, N, D, rollouts, seed = (int(x) for x in f[p + "cfg"])
        np.random.seed(seed)
        st = buffer.RolloutStorage(T, N, E.Box((D,)), E.Discrete(2), sim_hash=True)
        np.testing.assert_array_equal(st.A, f[p + "A"])
        step = 0
        for _ in range(rollouts):
            st.reset()
            for t in range(T):
                st.add(f[p + "obs"][step], np.zeros(N), f[p + "rew_in"][step], np.zeros(N, np.float32),
                       np.zeros(N, bool), np.zeros(N, np.float32))
                np.testing.assert_array_equal(st.rewards[t].cpu().numpy(), f[p + "rew_out"][step])
                step += 1
        assert int((st.count_table > 0).sum().item()) == int(f[p + "n_keys"])


def test_simhash_sharded_apply_equals_single():
    """Two env shards with replicated count tables (the multi-GPU path: keys all-gathered,
    each rank applies the bonus to its own envs) == one process over all envs."""
    import native
    rs = np.random.RandomState(5)
    N, D, steps = 1000, 3, 4
    A = torch.tensor(rs.randn(16, D), device="cuda")
    one = torch.zeros(native.SIMHASH_KEYS, dtype=torch.int32, device="cuda")
    tabs = [torch.zeros_like(one), torch.zeros_like(one)]
    for _ in range(steps):
        obs = rs.randn(N, D).astype(np.float32)
        obs[rs.rand(N) < 0.6] = obs[0]
        x = torch.tensor(obs, device="cuda")
        rew = torch.tensor(rs.randn(N).astype(np.float32), device="cuda")
        keys = torch.empty(N, dtype=torch.int32, device="cuda")
        native.simhash_keys(x, N, D, D, A, keys)
        r_one = rew.clone()
        native.simhash_apply(keys, N, 0, N, one, 0.1, r_one)
        halves = []
        for rank in range(2):
            r = rew[rank * N // 2:(rank + 1) * N // 2].clone()
            native.simhash_apply(keys, N, rank * N // 2, N // 2, tabs[rank], 0.1, r)
            halves.append(r)
        assert torch.equal(torch.cat(halves), r_one)
        assert torch.equal(tabs[0], one) and torch.equal(tabs[1], one)


def test_vector_env_ppo_runs_through_vecnormalize():
    """make_env wraps vector envs in VecNormalize (env.py:10-11): a PPO iteration on a
    MuJoCo-shaped synthetic env trains on normalised obs/rewards (|x| <= 10)."""
    import ppo
    import env as E
    np.random.seed(0)
    torch.manual_seed(0)
    alg = ppo.PPO(env_id="Swimmer-v3", n_envs=16, nstep=32, batch_size=64, n_epochs=2, quiet=True)
    assert isinstance(alg.env, E.VecNormalize)
    alg.collect_samples()
    ro = alg.rollout
    assert float(ro.obs_slots.abs().max()) <= 10.0 and float(ro.rewards.abs().max()) <= 10.0
    assert alg.env.ret_rms.count > 16 * 32
    alg.train()
    assert np.isfinite(alg.loss_accum.cpu().numpy()).all()


def _weight_sample_index(numel, k):
    """tests/golden/make_golden.py weight_sample_index (the fixture stores it too)."""
    if numel <= 8192:
        return np.arange(numel, dtype=np.int64)
    return np.sort(np.random.RandomState(1000 + k).choice(numel, 8192, replace=False)).astype(np.int64)


@pytest.mark.parametrize("math,rtol,head_min", [("split", 1e-4, None), ("split", 1e-4, 0), ("f32", 5e-5, None)])
@pytest.mark.parametrize("name", ["cnn4", "cnn18"])
def test_cnn_train_matches_reference_run(golden, name, math, rtol, head_min, monkeypatch):
    """The benchmarked Atari path end to end against the reference: the product PPO.train()
    (NatureCNN on the libppox conv kernels in `math`, rollout rows read in place by conv1,
    fused loss, explicit backward, head-gradient kernel, flat Adam) on the rollout of the
    reference's own run (live ppo.PPO with the checkpoint CnnActorCritic as policy.net,
    ppo.py:200-259, models-checkpoint.py:48-90) reproduces its post-update weights and
    losses.  Tolerances: weights rtol 1e-4 (split-f16 convs) / 5e-5 (exact-f32 MFMA) with
    atol 2e-6 (1 % of one Adam step, lr 3e-4); losses 1e-5 relative (head_min 0: the heads' hidden
    layer on the split-f16 kernels too, as at the bench's 16,384-row minibatches).  The reference's own f32
    weights are only accurate to ~2e-5 of exact arithmetic on these trajectories
    (test_oracle_golden.test_cnn_fixture_is_well_conditioned), so a tighter bound would
    measure the reference's rounding, not the product's."""
    import env as E
    import models
    import ppo
    monkeypatch.setenv("PPOX_CONV_MATH", math)
    if head_min is not None:
        import convs
        monkeypatch.setattr(convs, "HEAD_SPLIT_MIN_BATCH", head_min)
    f = golden("train_cnn")
    p = name + "_"
    N, T, B, E_, A, seed, net_seed = (int(x) for x in f[p + "cfg"])
    np.random.seed(seed)  # RolloutStorage draws randn(16, 4) at construction (buffer.py:137)
    env_id = "BreakoutNoFrameskip-v4" if A == 4 else "MontezumaRevengeNoFrameskip-v4"
    alg = ppo.PPO(env_id=env_id, env=E.DeviceAtariEnv(env_id, N), n_envs=N, nstep=T, batch_size=B, n_epochs=E_,
                  quiet=True)
    assert alg.policy.net.conv_impl.math == math
    torch.manual_seed(net_seed)
    init = models.CnnActorCritic(4, A).state_dict()  # the reference's init from the same torch seed
    sd = alg.policy.net.state_dict()
    with torch.no_grad():
        for k, v in sd.items():
            # orthogonal_ runs LAPACK's QR on the host CPU: bitwise equal in the build container
            # (tests/test_oracle_golden.py), last-bit different on other CPUs (GPU box)
            np.testing.assert_allclose(init[k].flatten()[:16].numpy(), f[p + "whead0_" + k], rtol=1e-5, atol=1e-7)
            np.testing.assert_allclose(float(init[k].double().sum()), float(f[p + "wsum0_" + k]), rtol=1e-5,
                                       atol=1e-5)
            v.copy_(init[k].to(v.device))
    alg.policy.net.conv_impl.invalidate()
    ro = alg.rollout
    obs = f[p + "obs"]
    for t in range(T):
        ro.add(obs[t], f[p + "roll_actions"][t], f[p + "roll_rewards"][t], f[p + "roll_values"][t],
               f[p + "roll_masks"][t], f[p + "roll_action_log_probs"][t])
    ro.compute_returns_and_advantages(f[p + "roll_values"][T - 1], f[p + "roll_masks"][T - 1])
    np.testing.assert_array_equal(ro.advantages.cpu().numpy(), f[p + "roll_advantages"])
    np.testing.assert_array_equal(ro.returns.cpu().numpy(), f[p + "roll_returns"])
    alg.train()
    sd = alg.policy.net.state_dict()
    lr = alg.lr
    wstats, fails = {}, []
    for k, (key, v) in enumerate(sd.items()):
        idx = f[p + "w1idx_" + key]
        assert np.array_equal(idx, _weight_sample_index(v.numel(), k))
        w, ref = v.flatten().cpu().numpy()[idx], f[p + "w1_" + key]
        err = np.abs(w.astype(np.float64) - ref)
        # every sampled weight within 5 % of one Adam step (lr) beyond the relative bound, and at
        # most 0.2 % of them beyond the strict one (atol 2e-6): an f32 reordering decides the sign
        # of a pre-activation within rounding of zero differently (a ReLU-boundary flip), which
        # moves that unit's weights by a fraction of an Adam step
        frac = float((err > rtol * np.abs(ref) + 2e-6).mean())
        d = (v.double().cpu() - init[key].double())
        dabs_rel = abs(float(d.abs().sum()) - float(f[p + "dabs_" + key])) / float(f[p + "dabs_" + key])
        wstats[key] = {"max_err": float(err.max()), "max_err_over_lr": float(err.max()) / lr, "frac_beyond_strict": frac,
                       "dabs_rel": dabs_rel}
        if not ((err <= rtol * np.abs(ref) + 0.05 * lr).all() and frac <= 2e-3 and dabs_rel <= 2e-3):
            fails.append((key, wstats[key]))
    np.testing.assert_array_equal(np.random.get_state()[1], f[p + "np_state_after"])
    acc = alg.loss_accum.cpu().numpy()
    n = acc[5]
    # policy-gradient, value and total loss within 1e-5 of the reference; the entropy of the
    # near-saturated softmax over raw-pixel logits (|logit| ~ 1e2) is set by the logits' last
    # bits, so the reference's own f32 entropy loss is 2.8e-5 (cnn18) / 2.7e-4 (cnn4) from
    # exact arithmetic (the float64 oracle run recorded in the fixture): the product's is held
    # to within twice that distance of float64 in split math, 2.5x with the exact-f32 MFMA
    # kernels (floor 1e-5; _loss_ok)
    stats = {}
    for i, key in ((0, "policy_gradient_loss"), (1, "value_loss"), (2, "entropy_loss"), (3, "total_loss")):
        got, ref, x64 = float(acc[i] / n), float(f[p + key]), float(f[p + "f64_" + key])
        stats[key] = {"rel_prod_ref": abs(got - ref) / abs(ref), "rel_prod_f64": abs(got - x64) / abs(x64),
                      "rel_ref_f64": abs(ref - x64) / abs(x64)}
    _parity_report(f"cnn_train_{name}_{math}_{head_min}", {"losses": stats, "weights": wstats})
    for i, key in ((0, "policy_gradient_loss"), (1, "value_loss"), (2, "entropy_loss"), (3, "total_loss")):
        if not _loss_ok(key, float(acc[i] / n), float(f[p + key]), float(f[p + "f64_" + key]), math):
            fails.append((key, stats[key]))
    assert not fails, fails


def _loss_ok(key, got, ref, x64, math):
    """A loss scalar matches the reference if it is within 1e-5 relative of the reference's
    value, or at most twice as far from exact arithmetic (the float64 oracle) as the reference's
    own float32 value is (a loss with cancellation — the policy-gradient mean of +-adv*ratio —
    can be further than 1e-5 from exact in the reference itself).  The entropy of the
    near-saturated softmax over raw-pixel logits is set by the logits' last bits and by the
    Adam trajectory of the earlier minibatches (a weight whose gradient is zero to rounding
    steps +-lr either way): it is held to within 2x the reference's own distance from exact in
    split math (the product default; measured 1.16-1.49x over the fixtures), 2.5x with the
    exact-f32 MFMA kernels (measured 0.59-2.26x), floor 1e-5 relative (profiles/r04_parity/)."""
    if key == "entropy_loss":
        k = 2.0 if math == "split" else 2.5
        return abs(got - x64) <= max(k * abs(ref - x64), 1e-5 * abs(x64))
    return abs(got - ref) <= 1e-5 * abs(ref) or abs(got - x64) <= 2 * abs(ref - x64)


def _parity_report(name, stats):
    """Observed errors of a parity test (PPOX_PARITY_OUT=dir writes them as JSON), so a
    regression that stays inside the tolerance is still visible."""
    import json
    import os
    d = os.environ.get("PPOX_PARITY_OUT")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, name + ".json"), "w") as fh:
            json.dump(stats, fh, indent=1)


def _first_minibatch_flips(f, p, alg, idx, masks, grad, A):
    """The first minibatch (initial weights) re-evaluated in float64 (tests/f64_pass.py) with float64's own ReLU
    decisions — pinned to the fixture's float64 gradient — and with the device pass's: the ReLU decisions the pass
    took differently from float64, per layer, and each sampled tensor's gradient error split into the part those
    decisions make (|g64(pass masks) - g64|) and the arithmetic error given them (|prod - g64(pass masks)|), both
    relative to the tensor's largest float64 entry."""
    ro, T = alg.rollout, alg.nstep
    i = idx.long()
    t_, n_ = i % T, i // T
    x = ro.obs_slots[t_, n_]
    mb = {"advantages": ro.advantages[t_, n_].view(-1, 1), "returns": ro.returns[t_, n_],
          "old_values": ro.values[t_, n_], "old_log_probs": ro.log_probs[t_, n_].view(-1, 1),
          "actions": ro.actions[t_, n_].long().view(-1, 1)}
    init = {k: torch.from_numpy(f[p + "init_" + k]) for k in alg.policy.net.state_dict()}
    g64, pre64 = f64_pass.minibatch_grads(init, x, mb, A)
    own, _ = f64_pass.minibatch_grads(init, x, mb, A, masks=masks)
    out = {"flips": f64_pass.flips(masks, pre64), "tensors": {}}
    off = 0
    for key, v in alg.policy.net.state_dict().items():
        g = grad[off:off + v.numel()].double()
        off += v.numel()
        a, b = g64[key].flatten(), own[key].flatten()
        sc = float(a.abs().max())
        w = torch.from_numpy(f[p + "w1idx_" + key]).to(a.device)
        pin = float((a[w].cpu() - torch.from_numpy(f[p + "g64_" + key])).abs().max()) / sc \
            if (p + "g64_" + key) in f.files else None
        out["tensors"][key] = {"arith": float((g - b).abs().max()) / sc, "relu": float((b - a).abs().max()) / sc,
                               "total": float((g - a).abs().max()) / sc, "pin_f64_vs_fixture": pin}
    return out


@pytest.mark.parametrize("math", ["split", "f32"])
def test_cnn_train_16384_rows_matches_reference_run(golden, math, monkeypatch):
    """The benchmark's dispatch end to end: one NatureCNN PPO iteration of 128 envs x 128
    steps trained as ONE 16,384-row minibatch per epoch (2 epochs) — the sg2 fc forward, the
    solo persistent conv2 dgrad, the split heads' hidden layer, multi-slab split-K weight
    gradients — against the reference's own run (ppo.py:200-259 with the checkpoint
    CnnActorCritic, models-checkpoint.py:48-90; tests/golden/make_golden.py gen_cnn_train_big)
    and against the same train() in float64 (oracle, recorded in the fixture).

    The frames are regenerated on the device by the synthetic Atari env from the recorded
    actions (bitwise: a crc32 per step).  Tolerances, in terms of the reference's own float32
    error e_ref = |ref - f64| measured on this trajectory:
      * weights, per tensor: max |prod - f64| <= k max e_ref + 1e-3 max_net(max e_ref) and mean
        |prod - f64| <= k mean e_ref + 1e-3 max_net(mean e_ref) — the product is as close to exact
        arithmetic as the reference is, within a factor k = 3 (measured round 4: split 0.4-2.0x max,
        exact-f32 MFMA 0.8-3.1x), k = 8 / 6 for the heads downstream of the hidden layer's ReLU, where
        one mask flip in the first minibatch dominates (measured 2.1-7.2x max, 3.4-4.1x mean: see the
        comment at the check; the floors are relative to the net's own rounding scale); plus every weight within
        rtol |ref| + 0.1 lr of the reference but for at most 0.2 % outliers (measured <= 0.061 %),
        which stay within three quarters of one Adam step (rtol |ref| + 0.75 lr, measured <= 0.52 lr:
        Adam's first steps move a weight by +-lr whatever its gradient's size, so a weight whose
        gradient is zero to rounding moves either way — the reference's own run is up to a third of
        a step off exact arithmetic here), and at most 0.5 % beyond rtol |ref| + 2e-6;
      * losses: policy-gradient, value, total within 1e-5 relative of the reference; the entropy
        of the near-saturated softmax within max(k e_ref, 1e-5 |f64|) of float64, k = 2 in split
        math, 2.5 with the exact-f32 kernels (_loss_ok)."""
    import env as E
    import models
    import ppo
    import zlib
    monkeypatch.setenv("PPOX_CONV_MATH", math)
    f = golden("train_cnn_big")
    p = "big_"
    N, T, B, E_, A, seed, net_seed, env_seed = (int(x) for x in f[p + "cfg"])
    np.random.seed(seed)  # RolloutStorage draws randn(16, 4) at construction (buffer.py:137)
    env_id = "BreakoutNoFrameskip-v4"
    env = E.DeviceAtariEnv(env_id, N, seed=env_seed, p_done=float(f[p + "p_done"]))
    alg = ppo.PPO(env_id=env_id, env=env, n_envs=N, nstep=T, batch_size=B, n_epochs=E_, quiet=True)
    assert alg.policy.net.conv_impl.math == math
    torch.manual_seed(net_seed)
    init = models.CnnActorCritic(4, A).state_dict()
    init_diff = {}
    with torch.no_grad():
        for k, v in alg.policy.net.state_dict().items():
            np.testing.assert_allclose(init[k].flatten()[:16].numpy(), f[p + "whead0_" + k], rtol=1e-5, atol=1e-7)
            # start from the reference's exact initial weights (this CPU's LAPACK QR may differ in
            # the last bits from the one the reference ran on)
            ref0 = torch.from_numpy(f[p + "init_" + k])
            init_diff[k] = float((init[k] - ref0).abs().max())
            init[k] = ref0
            v.copy_(ref0.to(v.device))
    alg.policy.net.conv_impl.invalidate()
    ro = alg.rollout
    acts = f[p + "roll_actions"]
    crc = f[p + "obs_crc"]
    obs = env.reset()
    assert zlib.crc32(obs.cpu().numpy().tobytes()) == crc[0]
    for t in range(T):
        ro.add(obs, acts[t], f[p + "roll_rewards"][t], f[p + "roll_values"][t], f[p + "roll_masks"][t],
               f[p + "roll_action_log_probs"][t])
        obs, _, done, _ = env.step(acts[t].reshape(N))
        assert zlib.crc32(obs.cpu().numpy().tobytes()) == crc[t + 1], t
        assert np.array_equal(done.cpu().numpy(), f[p + "roll_masks"][t].astype(bool)), t
    ro.compute_returns_and_advantages(f[p + "roll_values"][T - 1], f[p + "roll_masks"][T - 1])
    np.testing.assert_array_equal(ro.advantages.cpu().numpy(), f[p + "roll_advantages"])
    np.testing.assert_array_equal(ro.returns.cpu().numpy(), f[p + "roll_returns"])
    # the first minibatch's raw gradient (the flat bucket before clip + Adam)
    first = []
    step = alg.flat.adam_step

    def adam_step(*a, **k):
        if not first:
            first.append(alg.flat.grad.detach().clone())
        return step(*a, **k)
    monkeypatch.setattr(alg.flat, "adam_step", adam_step)
    fwd0, idx0, masks0 = [], [], []
    fwd, tobs = alg._fwd_train, alg._train_obs

    def train_obs(ro_, idx):
        if not idx0:
            idx0.append(idx.detach().clone())
        return tobs(ro_, idx)

    def fwd_train(obs):
        r = fwd(obs)
        if not fwd0:
            fwd0.append((r[0].detach().double().cpu().numpy(), r[1].detach().double().cpu().numpy()))
            masks0.extend(m.clone() for m in f64_pass.pass_masks(r[3]))  # the pass's own ReLU decisions
        return r
    monkeypatch.setattr(alg, "_train_obs", train_obs)
    monkeypatch.setattr(alg, "_fwd_train", fwd_train)
    alg.train()
    np.testing.assert_array_equal(np.random.get_state()[1], f[p + "np_state_after"])
    lr = alg.lr
    grads = {}
    off = 0
    for key, v in alg.policy.net.state_dict().items():
        grads[key] = first[0][off:off + v.numel()].cpu().numpy()
        off += v.numel()
    assert off == alg.flat.n
    rtol = 1e-4 if math == "split" else 5e-5
    stats, fails = {"math": math, "weights": {}, "losses": {}, "init_max_diff_local_vs_ref": init_diff}, []
    # floors relative to the net's own scale of rounding (no absolute floors): 1e-3 of the largest
    # per-tensor reference error |ref - f64| over the net, max and mean
    e_ref_max, e_ref_mean = [], []
    for key in alg.policy.net.state_dict():
        d = np.abs(f[p + "w1_" + key].astype(np.float64) - f[p + "w64_" + key])
        e_ref_max.append(d.max())
        e_ref_mean.append(d.mean())
    fl_max, fl_mean = 1e-3 * max(e_ref_max), 1e-3 * max(e_ref_mean)
    # the first minibatch's forward outputs (minibatch order) against float64, beside the reference's
    for name_, got, r32, r64 in (("logits", fwd0[0][0], f[p + "mb0_logits32"], f[p + "mb0_logits64"]),
                                 ("value", fwd0[0][1], f[p + "mb0_v32"], f[p + "mb0_v64"])):
        sc = np.abs(r64).max()
        stats["fwd_first_minibatch_" + name_] = {
            "max_prod_f64_rel": float(np.abs(got - r64).max() / sc), "max_ref_f64_rel": float(np.abs(r32 - r64).max() / sc),
            "mean_prod_f64_rel": float(np.abs(got - r64).mean() / sc), "mean_ref_f64_rel": float(np.abs(r32 - r64).mean() / sc),
            "mean_signed_prod_f64_rel": float((got - r64).mean() / sc), "mean_signed_ref_f64_rel": float((r32 - r64).mean() / sc)}
    # the first minibatch against float64, split into ReLU decisions and arithmetic (tests/f64_pass.py), beside
    # the reference's own split of its f32 run (tests/golden/train_cnn_big_flips.npz, tools/flip_analysis.py):
    # the product's arithmetic given its ReLU decisions within 3x the reference's given its own (+ 2e-7 of the
    # tensor's largest entry) for every tensor, and no more than 3x as many differing ReLU decisions.  (The exact-f32
    # mode's fc weight gradient is the library f32 GEMM over K = 16,384 rows, in the library's accumulation order:
    # 5.2e-6 measured, the reference's CPU GEMM 1.9e-7 — that mode's floor is 1e-5.)
    fm = stats["first_minibatch_relu"] = _first_minibatch_flips(f, p, alg, idx0[0], masks0, first[0], A)
    rf = golden("train_cnn_big_flips")
    for key, t in fm["tensors"].items():
        t["arith_ref"], t["relu_ref"] = float(rf["arith_" + key]), float(rf["relu_" + key])
        assert t["pin_f64_vs_fixture"] is None or t["pin_f64_vs_fixture"] <= 1e-12, (key, t)
        if not t["arith"] <= 3 * t["arith_ref"] + (2e-7 if math == "split" else 1e-5):
            fails.append(("first-minibatch arithmetic " + key, t))
    fm["flips_ref"] = dict(zip(f64_pass.LAYERS, rf["flips"].tolist()))
    if sum(fm["flips"].values()) > 3 * int(rf["flips"].sum()) or fm["flips"]["hidden"] > 3 * int(rf["flips"][4]) + 2:
        fails.append(("ReLU decisions vs float64", fm["flips"], fm["flips_ref"]))
    for k, (key, v) in enumerate(alg.policy.net.state_dict().items()):
        idx = f[p + "w1idx_" + key]
        assert np.array_equal(idx, _weight_sample_index(v.numel(), k))
        w = v.flatten().cpu().numpy()[idx].astype(np.float64)
        ref, w64 = f[p + "w1_" + key].astype(np.float64), f[p + "w64_" + key]
        e_p, e_r, e_pr = np.abs(w - w64), np.abs(ref - w64), np.abs(w - ref)
        frac = float((e_pr > rtol * np.abs(ref) + 2e-6).mean())
        frac_lr = float((e_pr > rtol * np.abs(ref) + 0.1 * lr).mean())
        d_abs = float((v.double().cpu() - init[key].double()).abs().sum())
        g, g32, g64 = grads[key][idx].astype(np.float64), f[p + "g32_" + key], f[p + "g64_" + key]
        gs = np.abs(g64).max()
        stats["grad_first_minibatch"] = stats.get("grad_first_minibatch", {})
        stats["grad_first_minibatch"][key] = {"max_prod_f64_rel": float(np.abs(g - g64).max() / gs),
                                              "max_ref_f64_rel": float(np.abs(g32 - g64).max() / gs),
                                              "mean_prod_f64_rel": float(np.abs(g - g64).mean() / gs),
                                              "mean_ref_f64_rel": float(np.abs(g32 - g64).mean() / gs)}
        stats["weights"][key] = {"max_prod_f64": float(e_p.max()), "max_ref_f64": float(e_r.max()),
                                 "mean_prod_f64": float(e_p.mean()), "mean_ref_f64": float(e_r.mean()),
                                 "max_prod_ref": float(e_pr.max()), "max_prod_ref_over_lr": float(e_pr.max()) / lr,
                                 "frac_beyond_strict": frac, "frac_beyond_tenth_lr": frac_lr,
                                 "dabs_rel": abs(d_abs - float(f[p + "d64abs_" + key])) / float(f[p + "d64abs_" + key])}
        # the heads downstream of the hidden layer's ReLU (extra_layer.*, critic_ext.*) are held to k = 8 / 6
        # (max / mean) instead of 3 only when the first minibatch shows that the extra layer's gradient error is
        # ReLU decisions, not arithmetic (asserted below from the float64 decomposition: its ReLU part >= 10x its
        # arithmetic part).  Two f32 passes take a few pre-activations within a rounding of 0 to the other side
        # (round 6: the reference's own run 1 of the 16,384 x 512 hidden ones, ours 1-2 and different ones); each
        # moves that row of the extra layer's gradient by a whole term (9.6e-5 of its largest entry here in both
        # math modes, the reference's own flip 2.0e-5), and Adam carries that into the heads' trajectories
        # (measured: critic_ext.weight 7.2x / 6.1x e_ref max, extra_layer 3.6-4.1x mean, split / f32)
        relu_driven = fm["tensors"]["extra_layer.0.weight"]["relu"] >= 10 * fm["tensors"]["extra_layer.0.weight"]["arith"]
        head = key.startswith(("extra_layer", "critic_ext")) and relu_driven
        k_max, k_mean = (8.0, 6.0) if head else (3.0, 3.0)
        stats["weights"][key]["k_max"], stats["weights"][key]["k_mean"] = k_max, k_mean
        if not (e_p.max() <= k_max * e_r.max() + fl_max and e_p.mean() <= k_mean * e_r.mean() + fl_mean
                and (e_pr <= rtol * np.abs(ref) + 0.75 * lr).all() and frac_lr <= 2e-3 and frac <= 5e-3):
            fails.append((key, stats["weights"][key]))
    acc = alg.loss_accum.cpu().numpy()
    n = acc[5]
    for i, key in ((0, "policy_gradient_loss"), (1, "value_loss"), (2, "entropy_loss"), (3, "total_loss")):
        got, ref, x64 = float(acc[i] / n), float(f[p + key]), float(f[p + "f64_" + key])
        stats["losses"][key] = {"prod": got, "ref": ref, "f64": x64, "rel_prod_ref": abs(got - ref) / abs(ref),
                                "rel_prod_f64": abs(got - x64) / abs(x64), "rel_ref_f64": abs(ref - x64) / abs(x64)}
        ok = _loss_ok(key, got, ref, x64, math)
        if not ok:
            fails.append((key, stats["losses"][key]))
    _parity_report(f"cnn_train_16384_{math}", stats)
    assert not fails, fails


def _read_csv(folder):
    import csv
    import os
    (name,) = os.listdir(folder)
    with open(os.path.join(folder, name)) as fh:
        rows = list(csv.reader(fh))
    return rows[0], [dict(zip(rows[0], r)) for r in rows[1:]]


REF_LEARN_KEYS = {"total timesteps", "total_time", "ep_rew_mean", "num_episodes", "entropy_loss",
                  "policy_gradient_loss", "value_loss", "total_loss"}


def test_learn_logs_reference_schema(tmp_path, monkeypatch):
    """PPO.learn() (ppo.py:261-308) with log_interval=1 and log_to_file=True: the CSV under
    ./logs/PPO/<env>/ carries the reference's columns (prefixes dropped, logger.py:26-29), the
    train/* columns join from the second dump (header rewrite), and the logged counters are
    the run's own.  Also the north_star aliases collect_rollouts / RolloutBuffer."""
    import buffer
    import env as E
    import ppo
    monkeypatch.chdir(tmp_path)
    N, T = 8, 16
    env_id = "BreakoutNoFrameskip-v4"
    alg = ppo.PPO(env_id=env_id, env=E.DeviceAtariEnv(env_id, N, seed=1, p_done=0.2), n_envs=N, nstep=T,
                  batch_size=64, n_epochs=1, quiet=True)
    assert buffer.RolloutBuffer is buffer.RolloutStorage and isinstance(alg.rollout, buffer.RolloutBuffer)
    assert alg.collect_rollouts() is True and alg.num_timesteps == N * T
    assert alg.learn(total_timesteps=4 * N * T, log_interval=1, log_to_file=True) is alg
    header, rows = _read_csv(tmp_path / "logs" / "PPO" / env_id)
    assert REF_LEARN_KEYS <= set(header) and len(header) == len(set(header))
    assert [int(r["total timesteps"]) for r in rows] == [2 * N * T, 3 * N * T, 4 * N * T]
    assert rows[0]["total_loss"] == "" and all(r["total_loss"] != "" for r in rows[1:])
    assert int(rows[-1]["num_episodes"]) == alg.num_episodes > 0
    assert abs(float(rows[-1]["ep_rew_mean"]) - np.mean([e["r"] for e in alg.ep_info_buffer])) < 1e-9
    assert len(alg.ep_info_buffer) == min(50, alg.num_episodes)


def test_learn_reward_target_stops_early(tmp_path, monkeypatch):
    """reward_target (ppo.py:296-306): the first iteration whose ep_rew_mean exceeds it logs a
    final row and ends learn()."""
    import env as E
    import ppo
    monkeypatch.chdir(tmp_path)
    N, T = 8, 16
    env_id = "BreakoutNoFrameskip-v4"
    alg = ppo.PPO(env_id=env_id, env=E.DeviceAtariEnv(env_id, N, seed=2, p_done=0.3), n_envs=N, nstep=T,
                  batch_size=64, n_epochs=1, quiet=True)
    alg.learn(total_timesteps=100 * N * T, log_interval=1, reward_target=-1.0, log_to_file=True)
    assert alg.num_timesteps == N * T
    header, rows = _read_csv(tmp_path / "logs" / "PPO" / env_id)
    assert len(rows) == 2 and rows[1]["total timesteps"] == str(N * T)


@pytest.mark.parametrize("algo", ["PPO", "PPO_ICM"])
def test_collect_graph_matches_eager(algo):
    """collect_samples as one captured graph (after the first, eager, collect) == the eager
    step loop, bitwise, across collect/train iterations (counters on the device, packed
    weights refreshed before each replay; PPO_ICM: with the K11 curiosity rewards mixed in)."""
    import logger
    import ppo
    logger.configure(algo, "BreakoutNoFrameskip-v4", quiet=True)

    def run(graph):
        np.random.seed(0)
        torch.manual_seed(0)
        alg = getattr(ppo, algo)(env_id="BreakoutNoFrameskip-v4", n_envs=16, nstep=8, batch_size=64, n_epochs=1,
                                 quiet=True, seed=5)
        alg._collect_graph_enabled = graph
        outs = []
        for _ in range(3):
            alg.collect_samples()
            ro = alg.rollout
            outs.append([x.clone() for x in (ro.actions, ro.rewards, ro.values, ro.log_probs, ro.masks,
                                              ro.obs_slots, ro.advantages)])
            if algo == "PPO_ICM":
                outs[-1].append(alg._ir_sum.clone())
            alg.train()
        w = alg.flat.data.clone() if algo == "PPO" else torch.cat([alg.flat.data, alg.icm_flat.data])
        return outs, w, alg._cgraph is not None, alg.num_timesteps

    (a, wa, ga, na), (b, wb, gb, nb) = run(False), run(True)
    assert not ga and gb and na == nb
    for xa, xb in zip(a, b):
        for u, v in zip(xa, xb):
            assert torch.equal(u, v)
    assert torch.equal(wa, wb)
