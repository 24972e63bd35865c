"""CPU restatement of the PPO / PPO+RND / PPO+ICM iteration (collect + GAE + train).

Test infrastructure only (see oracle/__init__.py).  Also the `port` CPU
baseline timed by bench.py.

Reference call stack:
  construction   ppo.py:154-160 / :349-365 / :586-600
  collect        ppo.py:166-198 / :367-407 / :603-649
  train          ppo.py:200-259 / :409-502 / :651-713
The env is any object with reset()/step(actions)->(obs, rew, done, infos)
(and unnormalize_obs for RND).  RNG use mirrors the reference: torch for init
and sampling, numpy's global RNG for randn(16,D) at storage construction, one
permutation per epoch, and (RND) one randn() per minibatch.
"""
import numpy as np
import torch
import torch.nn.functional as F

from . import models as M
from . import rms as R
from .storage import Rollout


def _space_info(space):
    name = space.__class__.__name__
    if name == "Discrete":
        return False, space.n, 1
    return True, space.shape[0], space.shape[0]


def clipped_value_loss(ret, v, old_v, clip):
    """ppo.py:229-232 — max of the two MEANS (not mean of max)."""
    vc = old_v + (v - old_v).clamp(-clip, clip)
    return torch.max(F.mse_loss(ret, v).mean(), F.mse_loss(ret, vc).mean()).mean()


def normalized(adv):
    """ppo.py:219 — per-minibatch, unbiased std."""
    return (adv - adv.mean()) / (adv.std() + 1e-8)


def surrogate(adv, ratio, clip):
    """ppo.py:222-226."""
    return -torch.min(adv * ratio, adv * torch.clamp(ratio, 1 - clip, 1 + clip)).mean()


def ppo_loss(v, lp, ent, mb, clip, ent_coef, vf_coef):
    """ppo.py:216-238 -> (loss, policy_loss, value_loss, entropy_loss)."""
    adv = normalized(mb["advantages"])
    pl = surrogate(adv, torch.exp(lp - mb["old_log_probs"]), clip)
    vl = clipped_value_loss(mb["returns"], v, mb["old_values"], clip)
    el = -torch.mean(ent)
    return pl + ent_coef * el + vf_coef * vl, pl, vl, el


def _tensors(mb, dtype=torch.float32):
    """Minibatch arrays as tensors; float32 fields promoted to `dtype` (float64 runs)."""
    out = {}
    for k, v in mb.items():
        t = torch.tensor(v)
        out[k] = t.to(dtype) if t.dtype == torch.float32 else t
    return out


class OraclePPO:
    """PPO (ppo.py:121-308) with an injected env and network factory."""

    def __init__(self, env, lr=3e-4, nstep=128, batch_size=128, n_epochs=10, gamma=0.99,
                 gae_lam=0.95, clip_range=0.2, ent_coef=0.01, vf_coef=1.0, max_grad_norm=0.2,
                 hidden_size=128, net=None, train_dtype=torch.float32):
        self.train_dtype = train_dtype  # float64: train() in double (collect stays f32, as the reference)
        self.lr = lr
        self.env = env
        self.N = env.num_envs
        self.obs_shape = tuple(env.observation_space.shape)
        self.box, self.n_act, self.act_out = _space_info(env.action_space)
        self.nstep, self.batch_size, self.n_epochs = nstep, batch_size, n_epochs
        self.clip, self.ent_coef, self.vf_coef, self.max_grad_norm = clip_range, ent_coef, vf_coef, max_grad_norm
        self.net = net if net is not None else M.MlpAC(self.obs_shape[0], self.n_act, hidden_size)
        self.rollout = Rollout(nstep, self.N, self.obs_shape, self.act_out, gamma, gae_lam)
        self.opt = torch.optim.Adam(self.net.parameters(), lr=lr)
        self.last_obs = env.reset()
        self.num_timesteps = 0
        self.stats = {}

    def collect(self):
        self.rollout.clear()
        for _ in range(self.nstep):
            with torch.no_grad():
                a, v, _, lp = M.act(self.net, self.last_obs, self.box)
            a = a.numpy()
            obs, rew, done, _ = self.env.step(a)
            self.num_timesteps += self.N
            self.rollout.add(self.last_obs, a.reshape(self.N, self.act_out), rew, v.numpy(), done,
                             lp.reshape(self.N, self.act_out).numpy())
            self.last_obs = obs
        self.rollout.finish(v.numpy(), done)

    def train(self):
        hist = {"loss": [], "pl": [], "vl": [], "el": []}
        dt = getattr(self, "train_dtype", torch.float32)
        if dt != torch.float32 and next(self.net.parameters()).dtype != dt:
            self.net.to(dt)
            self.opt = torch.optim.Adam(self.net.parameters(), lr=self.lr)
        for _ in range(self.n_epochs):
            for _idx, mb in self.rollout.minibatches(self.batch_size):
                mb = _tensors(mb, dt)
                v, _, lp, ent = M.evaluate(self.net, mb["observations"], mb["actions"], self.box, dt)
                loss, pl, vl, el = ppo_loss(v, lp, ent, mb, self.clip, self.ent_coef, self.vf_coef)
                self.opt.zero_grad()
                loss.backward()
                torch.nn.utils.clip_grad_norm_(self.net.parameters(), self.max_grad_norm)
                self.opt.step()
                for k, x in zip(("loss", "pl", "vl", "el"), (loss, pl, vl, el)):
                    hist[k].append(x.item())
        self.stats = {k: float(np.mean(v)) for k, v in hist.items()}


class OracleRND(OraclePPO):
    """PPO_RND (ppo.py:310-543)."""

    def __init__(self, env, lr=3e-4, nstep=128, batch_size=128, n_epochs=10, gamma=0.99,
                 int_gamma=0.99, gae_lam=0.95, clip_range=0.2, ent_coef=0.01, vf_coef=0.5,
                 int_vf_coef=0.5, max_grad_norm=0.2, hidden_size=128, int_hidden_size=128,
                 int_lr=3e-4, rnd_start=1e3, net=None, rnd=None, rnd_input=None):
        self.env = env
        self.N = env.num_envs
        self.obs_shape = tuple(env.observation_space.shape)
        self.box, self.n_act, self.act_out = _space_info(env.action_space)
        self.nstep, self.batch_size, self.n_epochs = nstep, batch_size, n_epochs
        self.clip, self.ent_coef, self.vf_coef, self.max_grad_norm = clip_range, ent_coef, vf_coef, max_grad_norm
        self.int_vf_coef, self.rnd_start = int_vf_coef, rnd_start
        self.net = net if net is not None else M.MlpAC(self.obs_shape[0], self.n_act, hidden_size, intrinsic=True)
        self.rnd = rnd if rnd is not None else M.RndMLP(self.obs_shape[0], int_hidden_size)
        # rnd_input maps an obs batch to the RND's input features (identity for MLP envs)
        self.rnd_input = rnd_input if rnd_input is not None else (lambda o: o)
        self.rollout = Rollout(nstep, self.N, self.obs_shape, self.act_out, gamma, gae_lam, int_gamma=int_gamma)
        self.opt = torch.optim.Adam(self.net.parameters(), lr=lr)
        self.rnd_opt = torch.optim.Adam(self.rnd.parameters(), lr=int_lr)
        self.last_obs = env.reset()
        self.obs_rms = R.RunningMoments()
        self.int_rew_rms = R.RunningMoments()
        self.num_timesteps = 0
        self.stats = {}

    def _norm(self, x):
        return R.normalize_obs(self.rnd_input(x), self.obs_rms.mean, self.obs_rms.var)

    def collect(self):
        self.rollout.clear()
        for _ in range(self.nstep):
            with torch.no_grad():
                a, v, iv, lp = M.act(self.net, self.last_obs, self.box)
            a = a.numpy()
            obs, rew, done, _ = self.env.step(a)
            self.num_timesteps += self.N
            if self.num_timesteps / self.N < self.rnd_start:        # ppo.py:390-392
                ir = np.zeros_like(rew)
                self.obs_rms.update(self.rnd_input(self.env.unnormalize_obs(self.last_obs)))
            else:                                                    # ppo.py:394-398
                ir = self.rnd.int_reward(torch.FloatTensor(self._norm(obs))).detach().numpy()
                self.int_rew_rms.update(ir)
                ir /= (np.sqrt(self.int_rew_rms.var) + 1e-08)
            self.rollout.add(self.last_obs, a.reshape(self.N, self.act_out), rew, v.numpy(), done,
                             lp.reshape(self.N, self.act_out).numpy(), int_reward=ir, int_value=iv.numpy())
            self.last_obs = obs
        self.mean_int_reward = float(np.mean(self.rollout.int_rewards))
        self.rollout.finish(v.numpy(), done, iv.numpy())

    def train_rnd(self, obs):
        """ppo.py:487-502."""
        p, t = self.rnd(torch.from_numpy(self._norm(obs.numpy())).float())
        loss = F.mse_loss(p, t)
        self.rnd_opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(self.rnd.parameters(), self.max_grad_norm)
        self.rnd_opt.step()

    def train(self):
        hist = {"loss": [], "pl": [], "vl": [], "el": [], "ivl": []}
        for _ in range(self.n_epochs):
            for _idx, mb in self.rollout.minibatches(self.batch_size):
                mb = _tensors(mb)
                v, iv, lp, ent = M.evaluate(self.net, mb["observations"], mb["actions"], self.box)
                adv = normalized(mb["advantages"]) + normalized(mb["int_advantages"])   # ppo.py:431-434
                pl = surrogate(adv, torch.exp(lp - mb["old_log_probs"]), self.clip)
                vl = clipped_value_loss(mb["returns"], v, mb["old_values"], self.clip)
                ivl = clipped_value_loss(mb["int_returns"], iv, mb["int_values"], self.clip)
                el = -torch.mean(ent)
                loss = pl + self.ent_coef * el + self.vf_coef * vl + self.int_vf_coef * ivl
                self.opt.zero_grad()
                loss.backward()
                torch.nn.utils.clip_grad_norm_(self.net.parameters(), self.max_grad_norm)
                self.opt.step()
                if np.random.randn() < 0.25:                                         # ppo.py:468
                    self.train_rnd(mb["observations"])
                for k, x in zip(("loss", "pl", "vl", "el", "ivl"), (loss, pl, vl, el, ivl)):
                    hist[k].append(x.item())
        self.stats = {k: float(np.mean(v)) for k, v in hist.items()}


class OracleICM(OraclePPO):
    """PPO_ICM (ppo.py:546-756).  Quirks kept: beta fixed at 0.2 (ppo.py:600),
    storage built without gamma (ppo.py:591), ICM pairs are consecutive rows of
    the PERMUTED minibatch (ppo.py:684)."""

    def __init__(self, env, lr=3e-4, int_lr=3e-4, nstep=128, batch_size=128, n_epochs=10,
                 gamma=0.99, gae_lam=0.95, clip_range=0.2, ent_coef=0.01, vf_coef=0.5,
                 max_grad_norm=0.2, hidden_size=128, int_hidden_size=32, int_rew_integration=0.05,
                 beta=0.2, policy_weight=1, net=None, icm_input=None):
        del gamma, beta  # ppo.py:591, 600
        self.env = env
        self.N = env.num_envs
        self.obs_shape = tuple(env.observation_space.shape)
        self.box, self.n_act, self.act_out = _space_info(env.action_space)
        self.nstep, self.batch_size, self.n_epochs = nstep, batch_size, n_epochs
        self.clip, self.ent_coef, self.vf_coef, self.max_grad_norm = clip_range, ent_coef, vf_coef, max_grad_norm
        self.eta, self.beta, self.policy_weight = int_rew_integration, 0.2, policy_weight
        self.net = net if net is not None else M.MlpAC(self.obs_shape[0], self.n_act, hidden_size)
        self.rollout = Rollout(nstep, self.N, self.obs_shape, self.act_out, 0.99, gae_lam)
        self.icm_input = icm_input if icm_input is not None else (lambda o: o)
        d_icm = int(np.prod(self.obs_shape)) if icm_input is not None else self.obs_shape[0]
        self.icm = M.IcmMLP(d_icm, self.n_act, not self.box, int_hidden_size)
        self.opt = torch.optim.Adam(self.net.parameters(), lr=lr)       # ppo.py:594 (policy.parameters)
        self.icm_opt = torch.optim.Adam(self.icm.parameters(), lr=int_lr)
        self.last_obs = env.reset()
        self.num_timesteps = 0
        self.stats = {}

    def collect(self):
        self.rollout.clear()
        means = []
        for _ in range(self.nstep):
            with torch.no_grad():
                a, v, _, lp = M.act(self.net, self.last_obs, self.box)
            obs, rew, done, _ = self.env.step(a.numpy())
            self.num_timesteps += self.N
            ir = self.icm.int_reward(torch.Tensor(self.icm_input(self.last_obs)),
                                     torch.Tensor(self.icm_input(obs)), a)       # ppo.py:629
            rew = (1 - self.eta) * rew + self.eta * ir.detach().numpy()          # ppo.py:630
            means.append(ir.mean().item())
            a = a.reshape(self.N, self.act_out)
            self.rollout.add(self.last_obs, a.numpy(), rew, v.numpy(), done,
                             lp.reshape(self.N, self.act_out).numpy())
            self.last_obs = obs
        self.mean_int_reward = float(np.round(np.mean(np.array(means)), 10))
        self.rollout.finish(v.numpy(), done)

    def train(self):
        hist = {"loss": [], "pl": [], "vl": [], "el": [], "icm": []}
        inv_loss_fn = torch.nn.MSELoss() if self.box else torch.nn.CrossEntropyLoss()
        for _ in range(self.n_epochs):
            for _idx, mb in self.rollout.minibatches(self.batch_size):
                mb = _tensors(mb)
                obs, acts = mb["observations"], mb["actions"]
                v, _, lp, ent = M.evaluate(self.net, obs, acts, self.box)
                adv = normalized(mb["advantages"])
                pl = surrogate(adv, torch.exp(lp - mb["old_log_probs"]), self.clip)
                vl = clipped_value_loss(mb["returns"], v, mb["old_values"], self.clip)
                x = self.icm_input(obs)
                a_hat, f_next, f_next_hat = self.icm(x[:-1], x[1:], acts[:-1])      # ppo.py:684
                fwd = F.mse_loss(f_next, f_next_hat)
                a_true = acts[:-1].float() if self.box else acts[:-1].squeeze().long()
                icm_loss = (1 - self.beta) * inv_loss_fn(a_hat, a_true) + self.beta * fwd
                el = -torch.mean(ent)
                loss = self.policy_weight * (pl + self.vf_coef * vl + self.ent_coef * el) + icm_loss
                self.opt.zero_grad()
                self.icm_opt.zero_grad()
                loss.backward()
                torch.nn.utils.clip_grad_norm_(self.net.parameters(), self.max_grad_norm)
                self.opt.step()
                self.icm_opt.step()
                for k, y in zip(("loss", "pl", "vl", "el", "icm"), (loss, pl, vl, el, icm_loss)):
                    hist[k].append(y.item())
        self.stats = {k: float(np.mean(v)) for k, v in hist.items()}
