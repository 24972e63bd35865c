"""SB3 VecNormalize restated in numpy (test infrastructure only, see oracle/__init__.py).

Reference site: env.py:10-11 wraps every env as VecNormalize(env, norm_reward=True).
stable_baselines3 is a third-party dependency NOT vendored in /root/reference and not
installed here (README.md:19 lists it unpinned; the `stable_baselines3.common.cmd_util`
import at env.py:2 dates it to the 2020 0.x series).  This file restates the published
0.x algorithm (vec_env/vec_normalize.py: defaults training=True, norm_obs=True,
norm_reward=True, clip_obs=10, clip_reward=10, gamma=0.99, epsilon=1e-8; its
RunningMeanStd is the same update as the reference's util.py:9-44) — PARITY UNPINNED:
no reference run or fixture holds its outputs; the device kernels are checked against
this restatement only.
"""
import numpy as np

from .rms import RunningMoments


class VecNormalizeNumpy:
    def __init__(self, n_envs, obs_dim, gamma=0.99, epsilon=1e-8, clip_obs=10.0, clip_reward=10.0, training=True):
        self.obs_rms = RunningMoments(shape=(obs_dim,))
        self.ret_rms = RunningMoments(shape=())
        self.ret = np.zeros(n_envs)
        self.gamma, self.epsilon, self.clip_obs, self.clip_reward = gamma, epsilon, clip_obs, clip_reward
        self.training = training

    def _update_reward(self, reward):
        """vec_normalize.py _update_reward: ret = ret * gamma + reward; ret_rms.update(ret)."""
        self.ret = self.ret * self.gamma + reward
        self.ret_rms.update(self.ret)

    def normalize_obs(self, obs):
        return np.clip((obs - self.obs_rms.mean) / np.sqrt(self.obs_rms.var + self.epsilon), -self.clip_obs,
                       self.clip_obs)

    def normalize_reward(self, reward):
        return np.clip(reward / np.sqrt(self.ret_rms.var + self.epsilon), -self.clip_reward, self.clip_reward)

    def reset(self, obs):
        """vec_normalize.py reset (0.x): zero returns, one ret_rms update on them, normalise."""
        self.ret = np.zeros(self.ret.shape[0])
        if self.training:
            self._update_reward(self.ret)
        return self.normalize_obs(obs)

    def step(self, obs, rews, news):
        """vec_normalize.py step_wait: -> (normalised obs, normalised rewards) as float64."""
        if self.training:
            self.obs_rms.update(obs)
        obs = self.normalize_obs(obs)
        if self.training:
            self._update_reward(rews)
        rews = self.normalize_reward(rews)
        self.ret[news] = 0
        return obs, rews
