"""End-to-end parity of the product API (ppo.PPO / buffer.RolloutStorage) on the GPU
against the reference's own recorded runs (tests/golden/train_ppo.npz) and the oracle."""
import numpy as np
import pytest
import torch

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


@pytest.mark.parametrize("name", ["disc2", "disc4sat", "disc18", "box2"])
def test_ppo_train_matches_reference_run(golden, name):
    """Same rollout + same weights + same numpy seed => product train() reproduces the
    reference's post-update weights (ppo.py:200-259).  box2: the Normal head with the
    reference's f64 log_prob / ratio / surrogate (models.py:66-71)."""
    import ppo
    import env as E
    f = golden("train_ppo")
    p = name + "_"
    D, N, T, B, E_, H, seed, code = (int(x) for x in f[p + "cfg"])
    # oracle regenerates the reference rollout bit-for-bit (pinned by test_oracle_golden)
    renv = ReplayVecEnv(f[p + "env_obs"], f[p + "env_rew"], f[p + "env_done"], space_from_code(code))
    np.random.seed(seed)
    torch.manual_seed(seed)
    orc = OraclePPO(renv, nstep=T, batch_size=B, n_epochs=E_, hidden_size=H, max_grad_norm=0.5,
                    ent_coef=0.01, vf_coef=1.0)
    if name == "disc4sat":
        with torch.no_grad():
            orc.net.actor[-1].weight.mul_(60.0)
    orc.collect()
    ro_ref = orc.rollout
    # product on the GPU
    np.random.seed(seed)  # RolloutStorage draws randn(16, D) at construction (buffer.py:137)
    denv = E.DeviceVecEnv("custom", N, obs_dim=D, action_space=_space(E, code))
    alg = ppo.PPO(env_id="custom", env=denv, n_envs=N, nstep=T, batch_size=B, n_epochs=E_, hidden_size=H,
                  max_grad_norm=0.5, ent_coef=0.01, vf_coef=1.0, quiet=True)
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
