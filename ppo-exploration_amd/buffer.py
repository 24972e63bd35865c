"""Device-resident rollout storage with the reference's interface
(reference: buffer.py:13-394 — RolloutStorage, IntrinsicStorage).

Layout in HBM, per rank (T = buffer_size, N = n_envs on this rank), STEP-MAJOR
like the reference's (buffer_size, n_envs, ...) arrays:
  obs_slots     (T+1, N, *obs)  uint8 frames (Atari) / f32 — slot t+1 is written
                                by the env step that consumes slot t; slot T is
                                the next rollout's first observation
  actions       (T, N) int32 (Discrete) or (T, N, A) f32 (Box)
  rewards, values, log_probs (T, N) f32 ((T, N, A) log_probs for Box)
  masks         (T, N) uint8  — done flag of transition t (buffer.py:180 / ppo.py:192)
  advantages, returns (T, N) f32  (+ int_* for IntrinsicStorage)
Minibatches use the reference's ENV-MAJOR flat index i = n*T + t and its
numpy-RNG permutation (buffer.py:239), mapped to (t, n) inside the kernels —
the rollout is never flattened or copied.  get() still yields the reference's
RolloutSample namedtuple (field names and per-field shapes of buffer.py:261-267)
for API compatibility.
"""
from collections import namedtuple

import numpy as np
import torch

import logger
import native
from dist import DistContext
from phases import traced


def _space_dim(space):
    return 1 if space.__class__.__name__ == "Discrete" else space.shape[0]


def _to_dev(x, device, dtype=None):
    if isinstance(x, torch.Tensor):
        t = x.detach().to(device)
    else:
        t = torch.as_tensor(np.asarray(x), device=device)
    return t.to(dtype) if dtype is not None else t


class BaseBuffer:
    """buffer.py:13-109 (size / reset / swap_and_flatten semantics)."""

    def __init__(self, buffer_size, observation_space, action_space, n_envs=1):
        self.buffer_size = buffer_size
        self.observation_space = observation_space
        self.obs_shape = tuple(observation_space.shape)
        self.action_space = action_space
        self.pos = 0
        self.full = False
        self.n_envs = n_envs
        self.action_dim = _space_dim(action_space)

    def size(self):
        return self.buffer_size if self.full else self.pos

    def reset(self):
        self.pos = 0
        self.full = False


class RolloutStorage(BaseBuffer):
    """buffer.py:111-267.  `RolloutBuffer` is an alias (north_star name)."""

    _fields = ("observations", "actions", "old_values", "old_log_probs", "advantages", "returns")

    def __init__(self, buffer_size, n_envs, obs_space, action_space, gae_lam=0.95, gamma=0.99, sim_hash=False,
                 device="cuda", obs_dtype=None, draw_hash_matrix=True):
        super().__init__(buffer_size, obs_space, action_space, n_envs=n_envs)
        self.gae_lam = gae_lam
        self.gamma = gamma
        self.device = torch.device(device)
        self.discrete = action_space.__class__.__name__ == "Discrete"
        if obs_dtype is None:
            obs_dtype = torch.uint8 if getattr(obs_space, "dtype", None) is np.uint8 else torch.float32
        self.obs_dtype = obs_dtype
        # buffer.py:137 draws the SimHash matrix from numpy's global RNG at
        # construction; keep the draw so every later permutation matches.
        self.A = np.random.randn(16, self.obs_shape[0]) if draw_hash_matrix else None
        T, N, d = buffer_size, n_envs, self.device
        self.do_hash, self.beta = bool(sim_hash), 0.1                  # buffer.py:141-146
        if self.do_hash:
            if len(self.obs_shape) != 1 or self.A is None:
                raise NotImplementedError("sim_hash needs vector observations (A = randn(16, obs_dim), "
                                          "buffer.py:137); image observations are out of scope")
            self.hash_A = torch.from_numpy(self.A).to(d)
            # the count table (buffer.py:136) as one u32 counter per 16-bit key; outlives reset()
            self.count_table = torch.zeros(native.SIMHASH_KEYS, dtype=torch.int32, device=d)
        self.obs_slots = torch.zeros((T + 1, N) + self.obs_shape, dtype=obs_dtype, device=d)
        if self.discrete:
            self.actions = torch.zeros((T, N), dtype=torch.int32, device=d)
            self.log_probs = torch.zeros((T, N), device=d)
        else:
            self.actions = torch.zeros((T, N, self.action_dim), device=d)
            self.log_probs = torch.zeros((T, N, self.action_dim), device=d)
        self.rewards = torch.zeros((T, N), device=d)
        self.values = torch.zeros((T, N), device=d)
        self.masks = torch.zeros((T, N), dtype=torch.uint8, device=d)
        self.advantages = torch.zeros((T, N), device=d)
        self.returns = torch.zeros((T, N), device=d)
        self.done_ret = torch.full((T, N), float("nan"), device=d)
        self.done_len = torch.zeros((T, N), dtype=torch.int32, device=d)
        self.generator_ready = False
        self.RolloutSample = namedtuple("RolloutSample", list(self._fields))
        self.reset()

    @property
    def observations(self):
        return self.obs_slots[: self.buffer_size]

    def reset(self):
        """buffer.py:149-163 re-allocates; here the arrays are reused."""
        self.generator_ready = False
        super().reset()

    def tensors(self):
        """Step-major device arrays by role (what the fused loss kernels read)."""
        return {"actions": self.actions, "log_probs": self.log_probs, "values": self.values,
                "advantages": self.advantages, "returns": self.returns}

    def add(self, obs, action, reward, value, mask, log_prob):
        """buffer.py:165-186 (inputs may be numpy arrays or tensors on any device)."""
        t = self.pos
        self.obs_slots[t].copy_(_to_dev(obs, self.device).reshape(self.obs_slots[t].shape))
        if self.discrete:
            self.actions[t].copy_(_to_dev(action, self.device).reshape(self.n_envs))
            self.log_probs[t].copy_(_to_dev(log_prob, self.device).reshape(self.n_envs))
        else:
            self.actions[t].copy_(_to_dev(action, self.device).reshape(self.n_envs, self.action_dim))
            self.log_probs[t].copy_(_to_dev(log_prob, self.device).reshape(self.n_envs, self.action_dim))
        self.rewards[t].copy_(_to_dev(reward, self.device).reshape(self.n_envs))
        if self.do_hash:
            self.sim_hash(self.obs_slots[t], self.rewards[t])
        self.masks[t].copy_(_to_dev(mask, self.device).reshape(self.n_envs))
        self.values[t].copy_(_to_dev(value, self.device).reshape(self.n_envs))
        self.pos += 1
        if self.pos == self.buffer_size:
            self.full = True

    def sim_hash(self, obs, rewards):
        """buffer.py:188-200 on the device: count bonus added to `rewards` (this rank's
        (n_envs,) f32 row, mutated in place and returned).  Keys of all ranks are
        gathered so the replicated count table advances exactly as in one process."""
        x = obs.reshape(self.n_envs, -1)
        if x.dtype != torch.float32 or x.stride(-1) != 1:
            x = x.float().contiguous()
        keys = torch.empty(self.n_envs, dtype=torch.int32, device=self.device)
        native.simhash_keys(x, self.n_envs, x.shape[1], x.stride(0), self.hash_A, keys)
        ctx = DistContext.current()
        if ctx.enabled:
            keys_all, offset, total = ctx.all_gather_cat(keys, dim=0), ctx.rank * self.n_envs, \
                self.n_envs * ctx.world
        else:
            keys_all, offset, total = keys, 0, self.n_envs
        native.simhash_apply(keys_all, total, offset, self.n_envs, self.count_table, self.beta, rewards)
        return rewards

    @traced("gae")
    def compute_returns_and_advantages(self, last_value, dones):
        """buffer.py:203-230 on the device (bit-identical), libppox ppox_gae."""
        lv = _to_dev(last_value, self.device, torch.float32).reshape(self.n_envs).contiguous()
        ld = _to_dev(dones, self.device, torch.uint8).reshape(self.n_envs).contiguous()
        native.gae(self.rewards, self.values, self.masks, lv, ld, self.gamma, self.gae_lam, self.advantages,
                   self.returns)

    # ------------------------------------------------------------------ get()
    def epoch_permutation(self):
        """buffer.py:239 — one numpy global-RNG permutation per get() call."""
        return np.random.permutation(self.buffer_size * self.n_envs)

    def _gather(self, x, idx):
        """(T, N, ...) step-major -> rows for env-major indices idx (device int64)."""
        T, N = self.buffer_size, self.n_envs
        x = x.contiguous()
        row = x[0, 0].numel() * x.element_size()
        out = torch.empty((idx.numel(),) + tuple(x.shape[2:]), dtype=x.dtype, device=self.device)
        native.gather_rows(x, T, N, row, row, idx, idx.numel(), out)
        return out

    def _sample(self, idx):
        B = idx.numel()
        acts = self._gather(self.actions, idx).reshape(B, self.action_dim).double()
        lps = self._gather(self.log_probs, idx).reshape(B, self.action_dim)
        return self.RolloutSample(self._gather(self.observations, idx), acts, self._gather(self.values, idx), lps,
                                  self._gather(self.advantages, idx).reshape(B, 1), self._gather(self.returns, idx))

    def get(self, batch_size=None):
        """buffer.py:233-254: minibatch generator over a fresh permutation."""
        assert self.full, ""
        perm = self.epoch_permutation()
        self.generator_ready = True
        total = self.buffer_size * self.n_envs
        bs = total if batch_size is None else batch_size
        perm_dev = torch.as_tensor(perm, device=self.device)
        for s in range(0, total, bs):
            yield self._sample(perm_dev[s:s + bs])


class IntrinsicStorage(RolloutStorage):
    """buffer.py:271-394: second (non-episodic) intrinsic reward stream."""

    _fields = ("observations", "actions", "old_values", "int_values", "old_log_probs", "advantages",
               "int_advantages", "returns", "int_returns")

    def __init__(self, buffer_size, n_envs, obs_space, action_space, gae_lam=0.95, gamma=0.99, int_gamma=0.99,
                 device="cuda", obs_dtype=None, draw_hash_matrix=True):
        super().__init__(buffer_size, n_envs, obs_space, action_space, gae_lam, gamma, device=device,
                         obs_dtype=obs_dtype, draw_hash_matrix=draw_hash_matrix)
        self.int_gamma = int_gamma
        T, N = buffer_size, n_envs
        self.int_rewards = torch.zeros((T, N), device=self.device)
        self.int_values = torch.zeros((T, N), device=self.device)
        self.int_advantages = torch.zeros((T, N), device=self.device)
        self.int_returns = torch.zeros((T, N), device=self.device)

    def tensors(self):
        d = super().tensors()
        d.update(int_values=self.int_values, int_advantages=self.int_advantages, int_returns=self.int_returns)
        return d

    def add(self, obs, action, reward, int_reward, value, int_value, mask, log_prob):
        t = self.pos
        self.int_rewards[t].copy_(_to_dev(int_reward, self.device).reshape(self.n_envs))
        self.int_values[t].copy_(_to_dev(int_value, self.device).reshape(self.n_envs))
        super().add(obs, action, reward, value, mask, log_prob)

    @traced("gae")
    def compute_returns_and_advantages(self, last_value, last_int_value, dones):
        """buffer.py:321-362, libppox ppox_gae_dual (both streams bit-identical)."""
        logger.record("rollout/mean_int_reward", float(self.int_rewards.mean().item()))
        lv = _to_dev(last_value, self.device, torch.float32).reshape(self.n_envs).contiguous()
        liv = _to_dev(last_int_value, self.device, torch.float32).reshape(self.n_envs).contiguous()
        ld = _to_dev(dones, self.device, torch.uint8).reshape(self.n_envs).contiguous()
        native.gae_dual(self.rewards, self.values, self.masks, lv, ld, self.int_rewards, self.int_values, liv,
                        self.gamma, self.int_gamma, self.gae_lam, self.advantages, self.returns,
                        self.int_advantages, self.int_returns)

    def _sample(self, idx):
        B = idx.numel()
        acts = self._gather(self.actions, idx).reshape(B, self.action_dim).double()
        lps = self._gather(self.log_probs, idx).reshape(B, self.action_dim)
        g = self._gather
        return self.RolloutSample(g(self.observations, idx), acts, g(self.values, idx), g(self.int_values, idx), lps,
                                  g(self.advantages, idx).reshape(B, 1), g(self.int_advantages, idx).reshape(B, 1),
                                  g(self.returns, idx), g(self.int_returns, idx))


# north_star names (SURVEY.md API-name mismatch note)
RolloutBuffer = RolloutStorage
IntrinsicRolloutBuffer = IntrinsicStorage
