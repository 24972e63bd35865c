"""Synthetic, device-resident vectorised environments.

Reference: env.py:7-12 builds SB3 `VecNormalize(make_vec_env(SubprocVecEnv))`
over gym/MuJoCo (and, in .ipynb_checkpoints/env-checkpoint.py:5-23, Atari with
VecFrameStack(4) + VecTransposeImage).  None of those simulators is available
offline, and the reference's env processes are the one process boundary of
its hot loop, so this build steps synthetic envs of the same observation/action
shapes on the GPU (libppox ppox_atari_env_* / ppox_vec_env_*), sharded by
global env index.  `make_env` keeps the reference's name and env_id argument.
"""
import math

import numpy as np
import torch

import native


class Discrete:
    def __init__(self, n):
        self.n = int(n)
        self.shape = ()

    def __repr__(self):
        return f"Discrete({self.n})"


class Box:
    def __init__(self, shape, low=-math.inf, high=math.inf, dtype=np.float32):
        self.shape = tuple(shape)
        self.low, self.high, self.dtype = low, high, dtype

    def __repr__(self):
        return f"Box{self.shape}"


# obs dim, action space, max episode length (classic control / MuJoCo shapes)
VECTOR_ENVS = {
    "CartPole-v1": (4, Discrete(2), 500),
    "CartPole-v0": (4, Discrete(2), 200),
    "Acrobot-v1": (6, Discrete(3), 500),
    "MountainCar-v0": (2, Discrete(3), 200),
    "LunarLander-v2": (8, Discrete(4), 1000),
    "Swimmer-v2": (8, Box((2,)), 1000),
    "Swimmer-v3": (8, Box((2,)), 1000),
    "Hopper-v2": (11, Box((3,)), 1000),
    "InvertedPendulum-v2": (4, Box((1,)), 1000),
    "InvertedDoublePendulum-v2": (11, Box((1,)), 1000),
    "Reacher-v2": (11, Box((2,)), 50),
    "BipedalWalker-v3": (24, Box((4,)), 1600),
}
ATARI_ACTIONS = {"Breakout": 4, "MontezumaRevenge": 18, "Pong": 6, "SpaceInvaders": 6, "Seaquest": 18,
                 "Qbert": 6, "BeamRider": 9, "Enduro": 9}


def is_atari(env_id):
    return "NoFrameskip" in env_id or env_id.split("-")[0] in ATARI_ACTIONS


class DeviceAtariEnv:
    """(N, 4, 84, 84) uint8 frame stacks on the device.  reward ~ Bernoulli(p_reward),
    done ~ Bernoulli(p_done) (SURVEY.md §8d synthetic inputs)."""

    def __init__(self, env_id, n_envs, seed=0, env_offset=0, p_reward=0.02, p_done=1e-3, device="cuda"):
        name = env_id.split("NoFrameskip")[0].split("-")[0]
        self.env_id = env_id
        self.num_envs = n_envs
        self.env_offset = env_offset
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.p_reward, self.p_done = p_reward, p_done
        self.device = torch.device(device)
        self.observation_space = Box((4, 84, 84), 0, 255, np.uint8)
        self.action_space = Discrete(ATARI_ACTIONS.get(name, 4))
        self.obs_dtype = torch.uint8
        self.ep_ret = torch.zeros(n_envs, device=self.device)
        self.ep_len = torch.zeros(n_envs, dtype=torch.int32, device=self.device)
        self.k = 0
        self._obs = None

    def reset_into(self, obs):
        native.atari_env_reset(obs, self.num_envs, self.env_offset, self.seed, self.ep_ret, self.ep_len)
        self.k = 0

    def step_into(self, obs_in, obs_out, actions, rewards, dones, done_ret=None, done_len=None):
        self.k += 1
        native.atari_env_step(obs_in, obs_out, actions, self.num_envs, self.env_offset, self.seed, self.k,
                              self.p_reward, self.p_done, rewards, dones, self.ep_ret, self.ep_len, done_ret,
                              done_len)

    def step_into_dc(self, obs_in, obs_out, actions, rewards, dones, done_ret, done_len, step_base, step_off):
        """step_into with the step counter read on the device (*step_base + step_off): the form a
        captured collect graph replays; the caller advances self.k on the host."""
        native.atari_env_step_dc(obs_in, obs_out, actions, self.num_envs, self.env_offset, self.seed, step_base,
                                 step_off, self.p_reward, self.p_done, rewards, dones, self.ep_ret, self.ep_len,
                                 done_ret, done_len)

    # VecEnv-style API (allocating; the training loop uses the *_into forms)
    def reset(self):
        self._obs = torch.empty((self.num_envs, 4, 84, 84), dtype=torch.uint8, device=self.device)
        self.reset_into(self._obs)
        return self._obs

    def step(self, actions):
        a = torch.as_tensor(actions, device=self.device).to(torch.int32).reshape(-1).contiguous()
        nxt = torch.empty_like(self._obs)
        rew = torch.empty(self.num_envs, device=self.device)
        done = torch.empty(self.num_envs, dtype=torch.uint8, device=self.device)
        dret = torch.empty(self.num_envs, device=self.device)
        dlen = torch.empty(self.num_envs, dtype=torch.int32, device=self.device)
        self.step_into(self._obs, nxt, a, rew, done, dret, dlen)
        self._obs = nxt
        return nxt, rew, done.bool(), episode_infos(dret, dlen)


class DeviceVecEnv:
    """Low-dimensional observation env of a classic-control / MuJoCo shape."""

    def __init__(self, env_id, n_envs, seed=0, env_offset=0, p_done=0.0, device="cuda", obs_dim=None,
                 action_space=None, max_len=None):
        d, space, ml = VECTOR_ENVS.get(env_id, (obs_dim or 4, action_space or Discrete(2), 200))
        self.env_id = env_id
        self.num_envs = n_envs
        self.env_offset = env_offset
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.obs_dim = obs_dim or d
        self.action_space = action_space or space
        self.max_len = ml if max_len is None else max_len
        self.p_done = p_done
        self.device = torch.device(device)
        self.observation_space = Box((self.obs_dim,))
        self.obs_dtype = torch.float32
        self.ep_ret = torch.zeros(n_envs, device=self.device)
        self.ep_len = torch.zeros(n_envs, dtype=torch.int32, device=self.device)
        self.k = 0
        self._obs = None

    def reset_into(self, obs):
        native.vec_env_reset(obs, self.num_envs, self.obs_dim, self.env_offset, self.seed, self.ep_ret, self.ep_len)
        self.k = 0

    def step_into(self, obs_in, obs_out, actions, rewards, dones, done_ret=None, done_len=None):
        self.k += 1
        if obs_out.data_ptr() != obs_in.data_ptr():
            obs_out.copy_(obs_in)
        a = actions if (actions is not None and actions.dtype == torch.int32) else None
        native.vec_env_step(obs_out, a, self.num_envs, self.obs_dim, self.env_offset, self.seed, self.k, self.p_done,
                            self.max_len, rewards, dones, self.ep_ret, self.ep_len, done_ret, done_len)

    def reset(self):
        self._obs = torch.empty((self.num_envs, self.obs_dim), device=self.device)
        self.reset_into(self._obs)
        return self._obs

    def step(self, actions):
        a = torch.as_tensor(actions, device=self.device)
        a = a.to(torch.int32).reshape(-1).contiguous() if self.action_space.__class__.__name__ == "Discrete" else None
        nxt = torch.empty_like(self._obs)
        rew = torch.empty(self.num_envs, device=self.device)
        done = torch.empty(self.num_envs, dtype=torch.uint8, device=self.device)
        dret = torch.empty(self.num_envs, device=self.device)
        dlen = torch.empty(self.num_envs, dtype=torch.int32, device=self.device)
        self.step_into(self._obs, nxt, a, rew, done, dret, dlen)
        self._obs = nxt
        return nxt, rew, done.bool(), episode_infos(dret, dlen)

    def unnormalize_obs(self, obs):
        return obs


DeviceAtariEnv.unnormalize_obs = DeviceVecEnv.unnormalize_obs


class VecNormalize:
    """env.py:10-11 wraps every env in stable_baselines3's VecNormalize(env,
    norm_reward=True).  SB3 is not vendored in the reference (README.md:19, unpinned;
    the cmd_util import dates it to the 2020 0.x series) and is not installed here, so
    its published algorithm is restated on the device — parity unpinned (oracle:
    oracle/vecnorm.py restates the same numpy program; tests check the kernels against it):
      step: obs_rms.update(obs); obs = clip((obs - mean) / sqrt(var + eps), +-clip_obs)
            ret = ret * gamma + r; ret_rms.update(ret); r = clip(r / sqrt(ret_rms.var + eps),
            +-clip_reward); ret[dones] = 0
      reset: ret = 0; (training) ret_rms.update(ret); obs normalised with the current stats
    The wrapped env's raw state stays in this wrapper (the device envs step in place);
    episode infos keep the raw returns (Monitor sits inside VecNormalize in SB3)."""

    def __init__(self, venv, training=True, norm_obs=True, norm_reward=True, clip_obs=10.0, clip_reward=10.0,
                 gamma=0.99, epsilon=1e-8):
        from util import RunningMeanStd
        self.venv = venv
        self.num_envs = venv.num_envs
        self.observation_space, self.action_space = venv.observation_space, venv.action_space
        self.obs_dtype = torch.float32
        self.device = venv.device
        self.training, self.norm_obs, self.norm_reward = training, norm_obs, norm_reward
        self.clip_obs, self.clip_reward, self.gamma, self.epsilon = clip_obs, clip_reward, gamma, epsilon
        D = int(np.prod(venv.observation_space.shape))
        self.obs_rms = RunningMeanStd(shape=(D,), device=self.device)
        self.ret_rms = RunningMeanStd(shape=(), device=self.device)
        self.ret = torch.zeros(self.num_envs, dtype=torch.float64, device=self.device)
        self.raw = torch.zeros((self.num_envs, D), device=self.device)
        self._obs = None

    def __getattr__(self, name):  # env_id, seed, ... of the wrapped env
        return getattr(self.__dict__["venv"], name)

    def _normalize_into(self, out):
        if self.norm_obs:
            native.normalize_obs_f32_ex(self.raw, self.num_envs, self.raw.shape[1], self.raw.shape[1],
                                        self.obs_rms.mean, self.obs_rms.var, self.epsilon, self.clip_obs, out)
        elif out.data_ptr() != self.raw.data_ptr():
            out.copy_(self.raw.view_as(out))

    def _reward(self, rewards, dones, update):
        """Return accumulator + ret_rms update; rewards normalised in place (norm_reward)."""
        target = rewards if self.norm_reward else rewards.clone()
        native.vecnorm_reward(target, dones, self.ret, self.gamma, self.ret_rms._mean, self.ret_rms._var,
                              self.ret_rms.count, self.epsilon, self.clip_reward, update)
        if update:
            self.ret_rms.count += self.num_envs

    def reset_into(self, obs):
        self.venv.reset_into(self.raw)
        self.ret.zero_()
        if self.training and self.norm_reward:
            zero = torch.zeros(self.num_envs, device=self.device)
            self._reward(zero, None, True)
        self._normalize_into(obs)

    def step_into(self, obs_in, obs_out, actions, rewards, dones, done_ret=None, done_len=None):
        self.venv.step_into(self.raw, self.raw, actions, rewards, dones, done_ret, done_len)
        if self.training and self.norm_obs:
            self.obs_rms.update(self.raw)
        self._normalize_into(obs_out)
        self._reward(rewards, dones, self.training)

    def reset(self):
        self._obs = torch.empty_like(self.raw)
        self.reset_into(self._obs)
        return self._obs

    def step(self, actions):
        a = torch.as_tensor(actions, device=self.device)
        a = a.to(torch.int32).reshape(-1).contiguous() if self.action_space.__class__.__name__ == "Discrete" else None
        nxt = torch.empty_like(self.raw)
        rew = torch.empty(self.num_envs, device=self.device)
        done = torch.empty(self.num_envs, dtype=torch.uint8, device=self.device)
        dret = torch.empty(self.num_envs, device=self.device)
        dlen = torch.empty(self.num_envs, dtype=torch.int32, device=self.device)
        self.step_into(None, nxt, a, rew, done, dret, dlen)
        self._obs = nxt
        return nxt, rew, done.bool(), episode_infos(dret, dlen)

    def get_original_obs(self):
        return self.raw.clone()

    def unnormalize_obs(self, obs):
        """obs * sqrt(var + eps) + mean (ppo.py:392 feeds this to the RND obs_rms)."""
        o = torch.as_tensor(obs, device=self.device).reshape(self.num_envs, -1).double()
        return (o * torch.sqrt(self.obs_rms.var + self.epsilon) + self.obs_rms.mean).float()


def episode_infos(done_ret, done_len):
    """SB3 Monitor-style infos for envs whose episode ended this step."""
    r = done_ret.cpu().numpy()
    ln = done_len.cpu().numpy()
    return [{"episode": {"r": float(r[i]), "l": int(ln[i])}} if not np.isnan(r[i]) else {} for i in range(len(r))]


def make_env(env_id, n_envs=4, seed=0, env_offset=0, device="cuda", normalize=True, **kw):
    """env.py:7-12 counterpart: the synthetic device env for env_id; vector envs are wrapped
    in VecNormalize(norm_reward=True) as in env.py:11 (Atari envs, which the reference
    builds in env-checkpoint.py without it, are not)."""
    if is_atari(env_id):
        return DeviceAtariEnv(env_id, n_envs, seed=seed, env_offset=env_offset, device=device, **kw)
    env = DeviceVecEnv(env_id, n_envs, seed=seed, env_offset=env_offset, device=device, **kw)
    return VecNormalize(env, norm_reward=True) if normalize else env
