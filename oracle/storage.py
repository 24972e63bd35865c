"""Rollout storage + minibatch iterator restated in numpy.

Test infrastructure only (see oracle/__init__.py).

Reference: buffer.py:111-267 (RolloutStorage) and :271-394 (IntrinsicStorage).
What matters for parity:
  * construction draws np.random.randn(16, obs_shape[0]) from numpy's global
    RNG (buffer.py:137) — it shifts every later permutation;
  * arrays are step-major (T, N, ...); obs float32, actions float64,
    masks int64 holding the done flag of transition t (buffer.py:153-161);
  * get(): one np.random.permutation(T*N) per call, drawn lazily at the first
    next() (buffer.py:239); the first call flattens every array env-major,
    flat index i = n*T + t (swap_and_flatten, buffer.py:41-52);
  * minibatches are consecutive slices of the permutation; the last one is a
    remainder when B does not divide T*N.
"""
import numpy as np

from . import gae as _gae


def flat_env_major(arr):
    """buffer.py:41-52: (T, N, ...) -> (N*T, ...); (T, N) -> (N*T, 1)."""
    a = np.asarray(arr)
    if a.ndim < 3:
        a = a.reshape(a.shape + (1,))
    return np.ascontiguousarray(a.swapaxes(0, 1)).reshape((a.shape[0] * a.shape[1],) + a.shape[2:])


def minibatch_slices(total, batch_size):
    """buffer.py:248-254: start offsets of the minibatches over one permutation."""
    bs = total if batch_size is None else batch_size
    return [(s, min(s + bs, total)) for s in range(0, total, bs)]


class Rollout:
    """Step-major rollout with one or two reward streams."""

    def __init__(self, T, N, obs_shape, action_dim, gamma=0.99, lam=0.95,
                 int_gamma=None, draw_hash_matrix=True):
        self.T, self.N = T, N
        self.obs_shape = tuple(obs_shape)
        self.action_dim = action_dim
        self.gamma, self.lam, self.int_gamma = gamma, lam, int_gamma
        self.dual = int_gamma is not None
        if draw_hash_matrix:  # buffer.py:137 — consumes the global numpy RNG
            self.hash_matrix = np.random.randn(16, self.obs_shape[0])
        self.clear()

    def clear(self):
        T, N = self.T, self.N
        self.obs = np.zeros((T, N) + self.obs_shape, np.float32)
        self.actions = np.zeros((T, N, self.action_dim))
        self.rewards = np.zeros((T, N), np.float32)
        self.values = np.zeros((T, N), np.float32)
        self.log_probs = np.zeros((T, N, self.action_dim), np.float32)
        self.masks = np.ones((T, N), np.int64)
        self.int_rewards = np.zeros((T, N), np.float32)
        self.int_values = np.zeros((T, N), np.float32)
        self.pos = 0
        self.flat = None

    def add(self, obs, action, reward, value, done, log_prob, int_reward=None, int_value=None):
        t = self.pos
        self.obs[t] = obs
        self.actions[t] = action
        self.rewards[t] = reward
        self.masks[t] = done
        self.values[t] = value
        self.log_probs[t] = log_prob
        if self.dual:
            self.int_rewards[t] = int_reward
            self.int_values[t] = np.asarray(int_value).reshape(self.N)
        self.pos += 1

    def finish(self, last_value, last_done, last_int_value=None):
        assert self.pos == self.T
        self.adv, self.ret = _gae.gae_single(self.rewards, self.values, self.masks, last_value,
                                             last_done, self.gamma, self.lam)
        if self.dual:
            self.iadv, self.iret = _gae.gae_intrinsic(self.int_rewards, self.int_values,
                                                      last_int_value, self.int_gamma, self.lam)

    def minibatches(self, batch_size):
        """Generator like buffer.py:233-267 / :365-394 (fields in namedtuple order)."""
        total = self.T * self.N
        perm = np.random.permutation(total)
        if self.flat is None:
            f = {"obs": flat_env_major(self.obs), "actions": flat_env_major(self.actions),
                 "values": flat_env_major(self.values), "log_probs": flat_env_major(self.log_probs),
                 "adv": flat_env_major(self.adv), "ret": flat_env_major(self.ret)}
            if self.dual:
                f.update(int_values=flat_env_major(self.int_values),
                         iadv=flat_env_major(self.iadv), iret=flat_env_major(self.iret))
            self.flat = f
        f = self.flat
        for s, e in minibatch_slices(total, batch_size):
            idx = perm[s:e]
            mb = {"observations": f["obs"][idx], "actions": f["actions"][idx],
                  "old_values": f["values"][idx].flatten()}
            if self.dual:
                mb["int_values"] = f["int_values"][idx].flatten()
            mb["old_log_probs"] = f["log_probs"][idx]
            mb["advantages"] = f["adv"][idx]
            if self.dual:
                mb["int_advantages"] = f["iadv"][idx]
            mb["returns"] = f["ret"][idx].flatten()
            if self.dual:
                mb["int_returns"] = f["iret"][idx].flatten()
            yield idx, mb


class SimHashCounter:
    """SimHash count bonus, buffer.py:188-200 (RolloutStorage(sim_hash=True).add):
    key = sign bits of A @ obs (A = randn(16, D) f64, obs promoted to f64); the
    count table outlives reset(); envs are processed in index order, each
    incrementing its key's count and adding beta / sqrt(count) to its reward
    (f32 reward + f64 bonus, stored back as f32).  Vector observations only."""

    def __init__(self, A, beta=0.1):
        self.A = np.asarray(A, np.float64)
        self.beta = beta
        self.count_table = {}

    def keys(self, obs):
        bits = (np.dot(self.A, np.asarray(obs).T).T > 0).astype(np.int64)
        return bits @ (1 << np.arange(bits.shape[1], dtype=np.int64))

    def apply(self, obs, rewards):
        r = np.array(rewards, dtype=np.float32, copy=True)
        for i, k in enumerate(self.keys(obs)):
            c = self.count_table.get(int(k), 0) + 1
            self.count_table[int(k)] = c
            r[i] = np.float32(np.float64(r[i]) + self.beta / np.sqrt(c))
        return r
