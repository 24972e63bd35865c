"""ES-NSRA (evolution_strategies.py) restated in numpy, plus the numpy twin of the
synthetic continuous-control env and perturbation stream the device path uses.

Test infrastructure only (see oracle/__init__.py).

Reference pieces restated (pinned by tests/golden/es.npz, recorded by running the
reference, tests/golden/make_golden.py gen_es):
  predict            FeedForwardNetwork.predict, evolution_strategies.py:50-63 (+ :86-97):
                     out = obs; out = arctan(out @ W) per hidden layer; tanh(out @ W_last)
  update_weights     EvolutionStrategy._update_weights, :224-246
  knn_distance       get_kNN, :273-289 (sklearn NearestNeighbors, Euclidean, sum of S nearest)
  novelty_probs      calc_noveltiy_distribution, :291-297
  nsr_update         the novelty-weight schedule of run(), :352-360

Not from the reference (it steps MuJoCo Swimmer through gym, unavailable offline):
the synthetic env below and the Philox perturbation stream.  The reference draws its
population with numpy's global RandomState (:176-186); the device draws a counter-based
stream instead (shard-invariant), so ES parity is pinned at the update rule / novelty /
policy level on given populations, not on the population draw.
"""
import numpy as np

from .philox import philox4x32_10, u01

ENV_B_TAG, ENV_NOISE_TAG, EPS_TAG = 0xB0B0B0B0, 0xE0E0E0E0, 0xE5E5E5E5


# ------------------------------------------------------------------ reference pieces
def predict(weights, obs):
    """evolution_strategies.py:50-63 for a Box action space: float64 arctan MLP, tanh head.
    obs (n, D) -> actions (n, A)."""
    out = np.asarray(obs, np.float64).reshape(len(obs), -1)
    for w in weights[:-1]:
        out = np.arctan(out @ w)
    return np.tanh(out @ weights[-1])


def update_weights(weights, pops, rewards, novelty, novelty_param, learning_rate, population_size, sigma):
    """:224-246 -> new weights (list).  pops[i] is the (P, in, out) population of layer i."""
    std = rewards.std()
    if std == 0:
        return [w.copy() for w in weights]
    r = (rewards - rewards.mean()) / std
    f = learning_rate / (population_size * sigma)
    nov = np.full(r.shape, novelty)
    out = []
    for w, lp in zip(weights, pops):
        score = ((1 - novelty_param) * np.dot(lp.T, r).T + novelty_param * np.dot(lp.T, nov).T) / 2
        out.append(w + f * score)
    return out


def knn_distance(archive, bc, S):
    """:273-289: sum of the S smallest Euclidean distances from bc (1, k) to archive (n, k)."""
    d = np.sqrt(((np.asarray(archive) - np.asarray(bc).reshape(1, -1)) ** 2).sum(axis=1))
    return float(np.sort(d)[:S].sum())


def novelty_probs(novelties):
    """:291-297."""
    return [round(n / sum(novelties), 4) for n in novelties]


def nsr_update(novelty_param, r_koeff, plateau, lo, hi, step):
    """:352-356 (applied every 5th iteration)."""
    if r_koeff < plateau:
        return min(hi, novelty_param + step)
    return max(lo, novelty_param - step)


# ------------------------------------------------------------------ device twins
def _key(seed):
    return seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF


def env_matrix(seed, D, A):
    """B[i][j] = +-1 (action j pushes state i)."""
    k0, k1 = _key(seed)
    i = np.arange(D, dtype=np.uint32)[:, None]
    j = np.arange(A, dtype=np.uint32)[None, :]
    w = philox4x32_10(i, j, np.uint32(ENV_B_TAG), np.uint32(0), k0, k1)[0]
    return np.where(w & np.uint32(1), 1.0, -1.0)


def env_noise(seed, D, t):
    k0, k1 = _key(seed)
    i = np.arange(D, dtype=np.uint32)
    w = philox4x32_10(i, np.uint32(t), np.uint32(ENV_NOISE_TAG), np.uint32(0), k0, k1)[0]
    return u01(w).astype(np.float64) - 0.5


def evaluate(weights_list, env_seed, T):
    """Synthetic 'SwimmerLike' episode for each member (list of weight lists), float64:
      s_0 = 0;  a_t = predict(s_t);  s_{t+1} = 0.9 s_t + 0.1 B a_t + 0.02 xi_t (xi shared
      by all members);  r_t = s_{t+1}[0] - 0.05 |a_t|^2;  episode of T steps (Swimmer has
      no early termination).  -> (fitness (n,), behaviour (n, 2) = final s[0:2])."""
    D = weights_list[0][0].shape[0]
    A = weights_list[0][-1].shape[1]
    B = env_matrix(env_seed, D, A)
    n = len(weights_list)
    s = np.zeros((n, D))
    fit = np.zeros(n)
    for t in range(T):
        a = np.stack([predict(w, s[m:m + 1])[0] for m, w in enumerate(weights_list)])
        s = 0.9 * s + 0.1 * (a @ B.T) + 0.02 * env_noise(env_seed, D, t)[None, :]
        fit += s[:, 0] - 0.05 * (a * a).sum(axis=1)
    return fit, s[:, :2].copy()


def perturbations(seed, generation, members, n_params):
    """eps[p][j] ~ N(0, 1), float64 Box-Muller on two 53-bit uniforms from Philox counter
    (j // 2, global member p, generation, EPS_TAG); j even -> cos branch, odd -> sin."""
    k0, k1 = _key(seed)
    p = np.asarray(members, np.uint32)[:, None]
    q = np.arange((n_params + 1) // 2, dtype=np.uint32)[None, :]
    x0, x1, x2, x3 = philox4x32_10(q, p, np.uint32(generation), np.uint32(EPS_TAG), k0, k1)
    u1 = ((x0 >> np.uint32(5)).astype(np.float64) * 67108864.0 + (x1 >> np.uint32(6)).astype(np.float64) + 1.0) \
        * 2.0 ** -53
    u2 = ((x2 >> np.uint32(5)).astype(np.float64) * 67108864.0 + (x3 >> np.uint32(6)).astype(np.float64)) * 2.0 ** -53
    r = np.sqrt(-2.0 * np.log(u1))
    z = np.stack([r * np.cos(2 * np.pi * u2), r * np.sin(2 * np.pi * u2)], axis=-1).reshape(len(p), -1)
    return z[:, :n_params]
