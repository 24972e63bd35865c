"""Philox4x32-10 and the synthetic environments, restated in numpy.

Test infrastructure only (see oracle/__init__.py).  The reference's envs are
gym/ALE/MuJoCo processes (env.py:7-12) that cannot run here; the build uses
synthetic device envs whose streams are defined below and mirrored bit-for-bit
by ppo-exploration_amd/csrc/env.hip.  Frame-stack / auto-reset layout follows
the reference's Atari wrapper stack (.ipynb_checkpoints/env-checkpoint.py:15-17:
VecFrameStack(4) + VecTransposeImage -> (N, 4, 84, 84) uint8, newest frame last,
stack zeroed on episode reset).
"""
import numpy as np

M0, M1, W0, W1 = np.uint32(0xD2511F53), np.uint32(0xCD9E8D57), np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised over broadcastable uint32 arrays; returns 4 uint32 arrays."""
    c0, c1, c2, c3 = (np.asarray(c, np.uint64) for c in (c0, c1, c2, c3))
    k0 = np.uint64(k0)
    k1 = np.uint64(k1)
    mask = np.uint64(0xFFFFFFFF)
    for _ in range(10):
        p0 = np.uint64(M0) * c0
        p1 = np.uint64(M1) * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & mask
        hi1, lo1 = p1 >> np.uint64(32), p1 & mask
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & mask, lo1, (hi0 ^ c3 ^ k1) & mask, lo0
        k0 = (k0 + np.uint64(W0)) & mask
        k1 = (k1 + np.uint64(W1)) & mask
    return tuple(x.astype(np.uint32) for x in (c0, c1, c2, c3))


def u01(x):
    return (np.asarray(x, np.uint32) >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)


FRAME = 84 * 84          # bytes per frame
FRAME_BLOCKS = FRAME // 16  # 441 philox blocks of 16 bytes
EVENT_BLOCK = 0xFFFFFFFF
RESET_ACTION = 0xFFFFFFFF


def _key(seed):
    return seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF


def atari_frame(seed, env_ids, step, actions):
    """(len(env_ids), 84*84) uint8: counter (block, env, step, action)."""
    k0, k1 = _key(seed)
    env_ids = np.asarray(env_ids, np.uint32)[:, None]
    acts = np.asarray(actions, np.uint32)[:, None]
    blocks = np.arange(FRAME_BLOCKS, dtype=np.uint32)[None, :]
    w = philox4x32_10(blocks, env_ids, np.uint32(step), acts, k0, k1)
    b = np.stack(w, axis=-1).astype("<u4").view(np.uint8)  # (n, 441, 16)
    return b.reshape(len(env_ids), FRAME)


def events(seed, env_ids, step, actions, p_reward, p_done):
    k0, k1 = _key(seed)
    w = philox4x32_10(np.uint32(EVENT_BLOCK), np.asarray(env_ids, np.uint32), np.uint32(step),
                      np.asarray(actions, np.uint32), k0, k1)
    rew = (u01(w[0]) < np.float32(p_reward)).astype(np.float32)
    done = u01(w[1]) < np.float32(p_done)
    return rew, done


class SyntheticAtari:
    """Numpy twin of the device env (csrc/env.hip ppox_atari_env_*).  step k
    (1-based) draws the new frame and the reward/done events from counter
    (., env, k, action); reset draws frame (., env, 0, RESET_ACTION)."""

    def __init__(self, n_envs, seed, n_actions=4, p_reward=0.02, p_done=1e-3, env_offset=0):
        self.num_envs, self.seed, self.n_actions = n_envs, seed, n_actions
        self.p_reward, self.p_done = p_reward, p_done
        self.env_ids = np.arange(env_offset, env_offset + n_envs)
        self.k = 0
        self.obs = None

    def reset(self):
        self.k = 0
        self.obs = np.zeros((self.num_envs, 4, 84, 84), np.uint8)
        self.obs[:, 3] = atari_frame(self.seed, self.env_ids, 0, np.full(self.num_envs, RESET_ACTION)).reshape(
            self.num_envs, 84, 84)
        return self.obs.copy()

    def step(self, actions):
        self.k += 1
        a = np.asarray(actions).astype(np.int64).reshape(self.num_envs).astype(np.uint32)
        f = atari_frame(self.seed, self.env_ids, self.k, a).reshape(self.num_envs, 84, 84)
        rew, done = events(self.seed, self.env_ids, self.k, a, self.p_reward, self.p_done)
        nxt = np.empty_like(self.obs)
        nxt[:, :3] = self.obs[:, 1:]
        nxt[done, :3] = 0
        nxt[:, 3] = f
        self.obs = nxt
        return nxt.copy(), rew, done, [{} for _ in range(self.num_envs)]
