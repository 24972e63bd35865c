"""BASELINE.json configs 3-5 at their full sizes on the device (config 1 is the `cartpole`
case of test_product_gpu.test_ppo_train_matches_reference_run; config 2 is the bench shape).

At these sizes the oracle cannot replay a whole iteration in seconds, so each test checks
the size-independent properties the path offers against the oracle on the rollout's OWN
buffers: GAE bit-exact (buffer.py:203-230 / :321-362), the running moments against the
numpy restatement on the recorded frames (util.py:20-44), the first RND rewards against a
torch-CPU restatement (ppo.py:394-398), the ES update against oracle.es.update_weights on
the device's own perturbations (evolution_strategies.py:224-246), and finite losses with a
real update."""
import numpy as np
import pytest
import torch

from oracle import es as OE
from oracle import gae as G
from oracle import models as OM
from oracle import rms as RM

pytestmark = pytest.mark.gpu


def _np(t):
    return t.cpu().numpy()


def test_c3_montezuma_rnd_1024x128():
    """PPO_RND, MontezumaRevengeNoFrameskip-v4 shape (18 actions), 1024 envs x 128 steps:
    63 warm-up steps (obs_rms on the last frame, zero int reward) then RND rewards."""
    import logger
    import ppo
    N, T, rnd_start = 1024, 128, 64
    np.random.seed(0)
    torch.manual_seed(0)
    alg = ppo.PPO_RND(env_id="MontezumaRevengeNoFrameskip-v4", n_envs=N, nstep=T, batch_size=16384, n_epochs=1,
                      rnd_start=rnd_start, quiet=True, seed=7)
    logger.configure("RND", "MontezumaRevengeNoFrameskip-v4", quiet=True)
    assert alg.n_actions == 18
    alg.collect_samples()
    ro = alg.rollout
    rew, irew, val, ival, masks = (_np(x) for x in (ro.rewards, ro.int_rewards, ro.values, ro.int_values, ro.masks))
    a, r, ia, ir = G.gae_dual(rew, irew, val, ival, masks, val[T - 1], ival[T - 1], masks[T - 1], alg.gamma,
                              ro.int_gamma, alg.gae_lam)
    np.testing.assert_array_equal(_np(ro.advantages), a)
    np.testing.assert_array_equal(_np(ro.returns), r)
    np.testing.assert_array_equal(_np(ro.int_advantages), ia)
    np.testing.assert_array_equal(_np(ro.int_returns), ir)
    # warm-up: obs_rms over the last frame of slots 0..rnd_start-2 (ppo.py:390-392)
    n_warm = rnd_start - 1
    rm = RM.RunningMoments()
    for t in range(n_warm):
        rm.update(_np(ro.obs_slots[t, :, 3].reshape(N, -1)))
    np.testing.assert_array_equal(_np(alg.obs_rms.mean), rm.mean)
    np.testing.assert_allclose(_np(alg.obs_rms.var), rm.var, rtol=1e-12)
    assert alg.obs_rms.count == rm.count
    assert not irew[:n_warm].any() and np.isfinite(irew).all() and (irew[n_warm:] > 0).all()
    # first RND step: normalise the NEXT obs' last frame, (pred - target)^2, int_rew_rms scaling
    rnd = OM.RndMLP(84 * 84, alg.rnd.predictor[0].out_features)
    rnd.load_state_dict({k: v.cpu() for k, v in alg.rnd.state_dict().items()})
    x = RM.normalize_obs(_np(ro.obs_slots[n_warm + 1, :, 3].reshape(N, -1)).astype(np.float64), rm.mean, rm.var)
    with torch.no_grad():
        raw = rnd.int_reward(torch.from_numpy(x).float()).numpy()
    irm = RM.RunningMoments()
    irm.update(raw)
    # rtol on O(1) rewards; near-zero rewards (pred ~ target) are cancellations: absolute bound
    np.testing.assert_allclose(irew[n_warm], raw / (np.sqrt(irm.var) + 1e-8), rtol=1e-4, atol=1e-6)
    w0 = alg.flat.data.clone()
    alg.train()
    acc = _np(alg.loss_accum)
    assert acc[5] == N * T // 16384 and np.isfinite(acc[:5]).all()
    assert not torch.equal(w0, alg.flat.data)


def test_c4_breakout_icm_per_rank_512x128():
    """PPO_ICM, Breakout shape, one rank's share of BASELINE config 4 (4096 envs / 8 GPUs =
    512 envs x 128 steps, minibatch 16384 / 8 = 2048), one epoch."""
    import logger
    import ppo
    N, T = 512, 128
    np.random.seed(1)
    torch.manual_seed(1)
    alg = ppo.PPO_ICM(env_id="BreakoutNoFrameskip-v4", n_envs=N, nstep=T, batch_size=2048, n_epochs=1, quiet=True,
                      seed=9)
    logger.configure("ICM", "BreakoutNoFrameskip-v4", quiet=True)
    alg.collect_samples()
    ro = alg.rollout
    rew, val, masks = _np(ro.rewards), _np(ro.values), _np(ro.masks)
    assert np.isfinite(rew).all()
    a, r = G.gae_single(rew, val, masks, val[T - 1], masks[T - 1], alg.gamma, alg.gae_lam)
    np.testing.assert_array_equal(_np(ro.advantages), a)
    np.testing.assert_array_equal(_np(ro.returns), r)
    w0, i0 = alg.flat.data.clone(), alg.icm_flat.data.clone()
    alg.train()
    acc = _np(alg.loss_accum)
    assert acc[5] == N * T // 2048 and np.isfinite(acc[:4]).all()
    assert np.isfinite(logger.get_values()["train/icm_loss"])
    assert not torch.equal(w0, alg.flat.data) and not torch.equal(i0, alg.icm_flat.data)


def test_c5_es_generation_p10000():
    """ES-NSRA, Swimmer shape (8 -> 64 -> 64 -> 2, 1000-step episodes), 10,000 perturbations:
    the device noise against the oracle's Philox restatement (sampled members), the device
    fitness against the oracle episode (sampled members), and the device update
    (Σ_p c_p ε_p, fixed-order reduction) against oracle.es.update_weights on the same noise."""
    import evolution_strategies as ES
    P = 10000
    np.random.seed(3)
    es = ES.EvolutionStrategy("Swimmer-v3", hidden_sizes=[64, 64], population_size=P, sigma=0.1,
                              learning_rate=0.01, seed=3)
    assert es.T == 1000 and es.n_params == 8 * 64 + 64 * 64 + 64 * 2
    eps = es._get_population()
    assert eps.shape == (P, es.n_params)
    members = np.array([0, 1, 4999, P - 1])
    np.testing.assert_allclose(_np(eps[members]), OE.perturbations(es.seed, 0, members, es.n_params), rtol=1e-13,
                               atol=1e-13)
    fit = es._get_rewards(None, eps)
    assert fit.shape == (P,) and np.isfinite(fit).all() and fit.std() > 0
    e = _np(eps)
    ws = []
    for p in members:
        off, w = 0, []
        for wi in es.weights:
            w.append(wi + es.SIGMA * e[p, off:off + wi.size].reshape(wi.shape))
            off += wi.size
        ws.append(w)
    # The closed-loop episode is chaotic at these weights: a 1e-15 relative weight change moves
    # the oracle's own 1000-step return by ~1 % (3e-7 at 300 steps, 1e-12 at 100; measured), so
    # per-member returns are compared over the first 100 steps of the same episodes.
    es.T = 100
    f100, _ = es._evaluate_dev(es._dev_weights(es.weights), eps[members].contiguous(), len(members))
    es.T = 1000
    f_ref, _ = OE.evaluate(ws, es.env_seed, 100)
    np.testing.assert_allclose(_np(f100), f_ref, rtol=1e-9, atol=1e-9)
    before = [w.copy() for w in es.weights]
    es.novelty_param = 0.4
    es._update_weights(fit, eps, 0.37)
    pops, off = [], 0
    for w in before:
        pops.append(e[:, off:off + w.size].reshape(P, *w.shape))
        off += w.size
    ref = OE.update_weights(before, pops, fit, 0.37, 0.4, 0.01, P, 0.1)
    for a_, b_ in zip(es.weights, ref):
        np.testing.assert_allclose(a_, b_, rtol=1e-11, atol=1e-13)
