#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by RUNNING the reference.

Test infrastructure only.  This script imports BoogaQ/PPO-exploration from
/root/reference (read-only; it exists only in the build container, never on the
GPU box) and records inputs + outputs of the functions on the hot path as small
.npz files.  No reference source is copied: the reference is imported and
called, and only arrays are written.

  buffer.py, util.py, models.py, logger.py import cleanly.
  ppo.py imports gym / stable_baselines3 / mujoco_py at module level
  (ppo.py:2,20; env.py:1-2).  None of them is installed; the minimal
  sys.modules entries below only satisfy those import statements (a
  `spaces` namespace and an empty `VecEnv` base class).  Nothing the
  algorithm computes comes from them: the environment is a FakeVec defined
  here whose outputs are recorded into the fixtures, so the oracle replays
  exactly the same env stream.  (SURVEY.md §8c documents this recipe.)

Run:  python tests/golden/make_golden.py        (skips if /root/reference absent)
"""
import os
import sys
import types
import importlib.util

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------
# import plumbing
# --------------------------------------------------------------------------
def _install_import_stubs():
    """Satisfy ppo.py's third-party import statements (not its computation)."""
    class VecEnv:  # ppo.py:20 uses it only for isinstance()
        pass

    gym = types.ModuleType("gym")
    gym.spaces = types.SimpleNamespace()
    sys.modules.setdefault("gym", gym)
    sys.modules.setdefault("gym.spaces", types.ModuleType("gym.spaces"))
    sys.modules.setdefault("mujoco_py", types.ModuleType("mujoco_py"))
    sb3 = types.ModuleType("stable_baselines3")
    common = types.ModuleType("stable_baselines3.common")
    vec = types.ModuleType("stable_baselines3.common.vec_env")
    base = types.ModuleType("stable_baselines3.common.vec_env.base_vec_env")
    cmd = types.ModuleType("stable_baselines3.common.cmd_util")
    base.VecEnv = VecEnv
    for name in ("SubprocVecEnv", "VecFrameStack", "VecTransposeImage", "VecNormalize"):
        setattr(vec, name, type(name, (), {}))
    cmd.make_atari_env = cmd.make_vec_env = lambda *a, **k: None
    for m in (sb3, common, vec, base, cmd):
        sys.modules.setdefault(m.__name__, m)
    return VecEnv


def import_reference():
    sys.dont_write_bytecode = True
    if REF not in sys.path:
        sys.path.insert(0, REF)
    VecEnv = _install_import_stubs()
    import util, buffer, models, logger  # noqa: E401
    import ppo
    return types.SimpleNamespace(util=util, buffer=buffer, models=models, logger=logger,
                                 ppo=ppo, VecEnv=VecEnv)


# Space duck types: the reference dispatches on __class__.__name__
# (models.py:20, buffer.py:38, util.py:53).
class Discrete:
    def __init__(self, n):
        self.n = n
        self.shape = ()


class Box:
    def __init__(self, shape):
        self.shape = tuple(shape)


def make_fakevec(VecEnv, n_envs, obs_dim, action_space, seed, done_p=0.05, obs_shape=None, frames=False):
    """Action-independent env with a PRIVATE RandomState (does not touch np's
    global RNG, so the reference's own np.random consumption is undisturbed).
    frames=True: (4, 84, 84) frame stacks of integer pixel values 0..255 as float32 (what
    the reference feeds the NatureCNN: VecFrameStack frames through torch.FloatTensor),
    made of 7x7-pixel blocks so the recorded fixture compresses."""
    shape = obs_shape if obs_shape is not None else (obs_dim,)

    class FakeVec(VecEnv):
        def __init__(self):
            self.num_envs = n_envs
            self.observation_space = Box(shape)
            self.action_space = action_space
            self.rs = np.random.RandomState(seed)
            self.trace = {"obs": [], "rew": [], "done": []}

        def _obs(self):
            if frames:
                blocks = self.rs.randint(0, 256, size=(n_envs, 4, 12, 12))
                return np.repeat(np.repeat(blocks, 7, axis=2), 7, axis=3).astype(np.float32)
            return self.rs.randn(n_envs, *shape).astype(np.float32)

        def reset(self):
            o = self._obs()
            self.trace["obs"].append(o.copy())
            return o

        def step(self, actions):
            o = self._obs()
            r = (self.rs.rand(n_envs) < 0.3).astype(np.float32) * self.rs.rand(n_envs).astype(np.float32)
            d = self.rs.rand(n_envs) < done_p
            infos = [{"episode": {"r": float(i), "l": 1}} if d[i] else {} for i in range(n_envs)]
            self.trace["obs"].append(o.copy())
            self.trace["rew"].append(r.copy())
            self.trace["done"].append(d.copy())
            return o, r, d, infos

        def unnormalize_obs(self, obs):
            return obs

    return FakeVec()


def save(name, **arrays):
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **arrays)
    print("wrote", os.path.relpath(path, OUT), sum(a.nbytes for a in map(np.asarray, arrays.values())), "B")


# --------------------------------------------------------------------------
# (1) GAE, one stream: RolloutStorage.compute_returns_and_advantages
#     buffer.py:203-230, called as ppo.py:196 (last_value = V(s_{T-1}))
# --------------------------------------------------------------------------
def gen_gae(R):
    import torch
    cases = [  # (T, N, gamma, lam, done_p, seed)
        (1, 1, 0.99, 0.95, 0.0, 0),
        (5, 3, 0.99, 0.95, 0.3, 1),
        (128, 8, 0.99, 0.95, 0.02, 2),
        (16, 33, 0.999, 0.95, 0.1, 3),
        (64, 64, 0.99, 1.0, 0.05, 4),
        (32, 17, 0.9, 0.0, 0.5, 5),
        (7, 5, 0.99, 0.95, 1.0, 6),       # every step terminal
        (256, 16, 0.997, 0.9, 0.001, 7),
    ]
    out = {}
    for k, (T, N, g, lam, dp, seed) in enumerate(cases):
        rs = np.random.RandomState(100 + seed)
        st = R.buffer.RolloutStorage(T, N, Box((2,)), Discrete(3), gae_lam=lam, gamma=g)
        rew = (rs.randn(T, N) * 2).astype(np.float32)
        val = (rs.randn(T, N) * 3).astype(np.float32)
        done = rs.rand(T, N) < dp
        for t in range(T):
            st.add(np.zeros((N, 2), np.float32), np.zeros((N, 1)), rew[t].copy(),
                   torch.from_numpy(val[t].copy()), done[t], torch.zeros(N, 1))
        last_v = (rs.randn(N) * 3).astype(np.float32)
        last_done = done[-1]  # ppo.py:196 passes the dones of the last env step
        st.compute_returns_and_advantages(torch.from_numpy(last_v), dones=last_done)
        p = f"c{k}_"
        out.update({p + "T": np.int64(T), p + "N": np.int64(N), p + "gamma": np.float64(g),
                    p + "lam": np.float64(lam), p + "rewards": rew, p + "values": val,
                    p + "dones": done, p + "last_value": last_v, p + "last_done": last_done,
                    p + "advantages": st.advantages.copy(), p + "returns": st.returns.copy()})
    out["ncases"] = np.int64(len(cases))
    save("gae_single", **out)


# --------------------------------------------------------------------------
# (2) GAE, two streams: IntrinsicStorage (buffer.py:321-362)
# --------------------------------------------------------------------------
def gen_gae_dual(R):
    import torch
    R.logger.record = lambda *a, **k: None  # buffer.py:335 side effect not needed
    cases = [(1, 1, 0.99, 0.99, 0.95, 0.0, 0), (9, 4, 0.99, 0.999, 0.95, 0.2, 1),
             (128, 16, 0.99, 0.99, 0.95, 0.01, 2), (33, 7, 0.999, 0.9, 1.0, 0.1, 3),
             (64, 32, 0.97, 0.995, 0.8, 0.05, 4)]
    out = {}
    for k, (T, N, g, ig, lam, dp, seed) in enumerate(cases):
        rs = np.random.RandomState(200 + seed)
        st = R.buffer.IntrinsicStorage(T, N, Box((2,)), Discrete(3), gae_lam=lam, gamma=g, int_gamma=ig)
        st.reset()  # IntrinsicStorage.__init__ nulls its int arrays (buffer.py:285)
        rew = (rs.randn(T, N)).astype(np.float32)
        irew = np.abs(rs.randn(T, N)).astype(np.float32)
        val = (rs.randn(T, N) * 2).astype(np.float32)
        ival = (rs.randn(T, N)).astype(np.float32)
        done = rs.rand(T, N) < dp
        for t in range(T):
            st.add(np.zeros((N, 2), np.float32), np.zeros((N, 1)), rew[t].copy(), irew[t].copy(),
                   torch.from_numpy(val[t].copy()), torch.from_numpy(ival[t].copy()), done[t],
                   torch.zeros(N, 1))
        lv = rs.randn(N).astype(np.float32)
        liv = rs.randn(N).astype(np.float32)
        st.compute_returns_and_advantages(torch.from_numpy(lv), torch.from_numpy(liv), done[-1])
        p = f"c{k}_"
        out.update({p + "T": np.int64(T), p + "N": np.int64(N), p + "gamma": np.float64(g),
                    p + "int_gamma": np.float64(ig), p + "lam": np.float64(lam),
                    p + "rewards": rew, p + "int_rewards": irew, p + "values": val,
                    p + "int_values": ival, p + "dones": done, p + "last_value": lv,
                    p + "last_int_value": liv, p + "last_done": done[-1],
                    p + "advantages": st.advantages.copy(), p + "returns": st.returns.copy(),
                    p + "int_advantages": st.int_advantages.copy(),
                    p + "int_returns": st.int_returns.copy()})
    out["ncases"] = np.int64(len(cases))
    save("gae_dual", **out)


# --------------------------------------------------------------------------
# (3) RunningMeanStd sequences (util.py:9-44) and normalize_obs (ppo.py:111-118)
# --------------------------------------------------------------------------
def gen_rms(R):
    rs = np.random.RandomState(300)
    out = {}
    # a) feature vectors, float32 batches of varying size (obs_rms path, ppo.py:392)
    rms = R.util.RunningMeanStd()
    batches = [(rs.randn(n, 6) * 3 + 1).astype(np.float32) for n in (4, 1, 17, 64, 3)]
    for i, b in enumerate(batches):
        rms.update(b)
        out[f"f32_b{i}"] = b
        out[f"f32_mean{i}"] = np.asarray(rms.mean, np.float64)
        out[f"f32_var{i}"] = np.asarray(rms.var, np.float64)
        out[f"f32_count{i}"] = np.float64(rms.count)
    out["f32_n"] = np.int64(len(batches))
    # b) uint8 frames (Atari last frame, 84x84 flattened to 7056 features)
    rms = R.util.RunningMeanStd()
    frames = [rs.randint(0, 256, size=(n, 7056)).astype(np.uint8) for n in (8, 5)]
    for i, b in enumerate(frames):
        rms.update(b)
        out[f"u8_b{i}"] = b
        out[f"u8_mean{i}"] = np.asarray(rms.mean, np.float64)
        out[f"u8_var{i}"] = np.asarray(rms.var, np.float64)
        out[f"u8_count{i}"] = np.float64(rms.count)
    out["u8_n"] = np.int64(len(frames))
    # c) scalar stream (int_rew_rms, ppo.py:396): shape () state, (N,) batches
    rms = R.util.RunningMeanStd()
    for i in range(6):
        b = np.abs(rs.randn(16)).astype(np.float32) * (i + 1)
        rms.update(b)
        out[f"sc_b{i}"] = b
        out[f"sc_mean{i}"] = np.asarray(rms.mean, np.float64)
        out[f"sc_var{i}"] = np.asarray(rms.var, np.float64)
        out[f"sc_count{i}"] = np.float64(rms.count)
    out["sc_n"] = np.int64(6)
    # d) normalize_obs with the state from (a): BaseAlgorithm.normalize_obs
    alg = types.SimpleNamespace(obs_rms=R.util.RunningMeanStd())
    for b in batches:
        alg.obs_rms.update(b)
    x = (rs.randn(32, 6) * 10).astype(np.float32)
    out["norm_in"] = x
    out["norm_mean"] = np.asarray(alg.obs_rms.mean)
    out["norm_var"] = np.asarray(alg.obs_rms.var)
    out["norm_out"] = R.ppo.BaseAlgorithm.normalize_obs(alg, x)
    save("rms", **out)


# --------------------------------------------------------------------------
# (4) get(): swap_and_flatten + np.random.permutation minibatching
#     buffer.py:41-52, 137, 233-267 — including the construction-time randn
# --------------------------------------------------------------------------
def gen_get(R):
    import torch
    out = {}
    for k, (T, N, D, B, E, seed) in enumerate([(8, 3, 2, 5, 3, 11), (4, 4, 3, None, 2, 12),
                                               (16, 5, 1, 16, 2, 13)]):
        np.random.seed(seed)
        st = R.buffer.RolloutStorage(T, N, Box((D,)), Discrete(4))  # draws randn(16, D)
        obs = np.arange(T * N * D, dtype=np.float32).reshape(T, N, D)
        for t in range(T):
            st.add(obs[t], np.full((N, 1), t), np.zeros(N, np.float32),
                   torch.arange(N, dtype=torch.float32) + 100 * t, np.zeros(N, bool),
                   torch.full((N, 1), float(t)))
        st.compute_returns_and_advantages(torch.zeros(N), dones=np.zeros(N, bool))
        p = f"c{k}_"
        out[p + "cfg"] = np.array([T, N, D, -1 if B is None else B, E, seed], np.int64)
        mb = 0
        for e in range(E):
            for batch in st.get(B):
                out[p + f"obs{mb}"] = batch.observations.numpy()
                out[p + f"act{mb}"] = batch.actions.numpy()
                out[p + f"oldv{mb}"] = batch.old_values.numpy()
                out[p + f"oldlp{mb}"] = batch.old_log_probs.numpy()
                out[p + f"adv{mb}"] = batch.advantages.numpy()
                out[p + f"ret{mb}"] = batch.returns.numpy()
                mb += 1
        out[p + "nmb"] = np.int64(mb)
        out[p + "A"] = st.A.copy()
    save("get_perm", **out)


# --------------------------------------------------------------------------
# (4b) SimHash count bonus (buffer.py:188-200) through RolloutStorage.add with
#      sim_hash=True: keys of A.obs, a count table persisting across reset(),
#      rewards mutated in env-index order.  Duplicated rows force collisions
#      within one step.
# --------------------------------------------------------------------------
def gen_simhash(R):
    import torch
    out = {}
    for k, (T, N, D, rollouts, seed) in enumerate([(5, 16, 2, 2, 31), (4, 64, 6, 3, 32), (3, 7, 1, 2, 33)]):
        np.random.seed(seed)
        st = R.buffer.RolloutStorage(T, N, Box((D,)), Discrete(2), sim_hash=True)  # draws A = randn(16, D)
        rs = np.random.RandomState(seed + 100)
        p = f"s{k}_"
        out[p + "cfg"] = np.array([T, N, D, rollouts, seed], np.int64)
        out[p + "A"] = st.A.copy()
        obs_all, rin_all, rout_all = [], [], []
        for r in range(rollouts):
            st.reset()
            for t in range(T):
                obs = rs.randn(N, D).astype(np.float32)
                dup = rs.rand(N) < 0.5
                obs[dup] = obs[rs.randint(0, max(1, N // 4), dup.sum())]
                rew = rs.randn(N).astype(np.float32)
                obs_all.append(obs.copy())
                rin_all.append(rew.copy())
                st.add(obs, np.zeros((N, 1)), rew, torch.zeros(N), np.zeros(N, bool), torch.zeros(N, 1))
                rout_all.append(st.rewards[t].copy())
        out[p + "obs"] = np.stack(obs_all)
        out[p + "rew_in"] = np.stack(rin_all)
        out[p + "rew_out"] = np.stack(rout_all)
        out[p + "n_keys"] = np.int64(len(st.count_table))
    save("simhash", **out)


# --------------------------------------------------------------------------
# (5) One full PPO.train() (ppo.py:200-259) on fixed weights: losses, dL/dlogits,
#     dL/dvalues per minibatch, post-update weights.  Discrete and Box.
# --------------------------------------------------------------------------
def _record_logger(R):
    rec = {}
    R.logger.record = lambda k, v: rec.__setitem__(k, v)
    R.logger.configure = lambda *a, **k: None
    R.logger.dump = lambda *a, **k: None
    return rec


def _net_grad_hooks(net, store):
    def fwd_hook(mod, inp, outp):
        outs = outp if isinstance(outp, tuple) else (outp,)
        store["inputs"].append(inp[0].detach().clone())
        grads = []
        store["grads"].append(grads)
        for o in outs:
            if o.requires_grad:
                o.register_hook(lambda g, grads=grads: grads.append(g.detach().clone()))
    return net.register_forward_hook(fwd_hook)


def gen_train(R):
    import torch
    out = {}
    cases = [  # name, action_space, obs_dim, n_envs, nstep, batch, epochs, hidden, seed, kwargs
        ("disc2", Discrete(2), 4, 4, 16, 16, 2, 32, 21, {}),
        ("disc4sat", Discrete(4), 5, 3, 8, 12, 1, 16, 22, {"sat": True}),
        ("box2", Box((2,)), 3, 4, 8, 8, 2, 16, 23, {}),
        ("disc18", Discrete(18), 6, 2, 12, 24, 1, 16, 24, {}),
        # BASELINE config 1 (CartPole-v1 shape): 8 envs x 128 steps, MLP hidden 128, the
        # reference's default batch 128 and 10 epochs (80 optimizer steps); batches not recorded
        ("cartpole", Discrete(2), 4, 8, 128, 128, 10, 128, 25, {"no_batches": True, "defaults": True}),
    ]
    for name, aspace, D, N, T, B, E, H, seed, kw in cases:
        rec = _record_logger(R)
        np.random.seed(seed)
        torch.manual_seed(seed)
        env = make_fakevec(R.VecEnv, N, D, aspace, seed=1000 + seed)
        R.ppo.make_env = lambda env_id, n_envs=4, env=env: env
        if kw.get("defaults"):  # the reference's own defaults (ppo.py:139-153) for the rest
            alg = R.ppo.PPO(env_id="Fake-v0", nstep=T, batch_size=B, n_epochs=E, hidden_size=H)
        else:
            alg = R.ppo.PPO(env_id="Fake-v0", nstep=T, batch_size=B, n_epochs=E, hidden_size=H,
                            max_grad_norm=0.5, ent_coef=0.01, vf_coef=1.0)
        if kw.get("sat"):
            with torch.no_grad():  # push the actor into softmax saturation (eps clamp)
                alg.policy.net.actor[-1].weight.mul_(60.0)
        init = {k: v.detach().clone().numpy() for k, v in alg.policy.net.state_dict().items()}
        alg.collect_samples()
        st = alg.rollout
        store = {"inputs": [], "grads": []}
        h = _net_grad_hooks(alg.policy.net, store)
        # capture per-minibatch batches too (the inputs of train's loss)
        batches = []
        orig_get = st.get

        def get_rec(bs, orig_get=orig_get):
            for b in orig_get(bs):
                batches.append(b)
                yield b
        st.get = get_rec
        if aspace.__class__.__name__ == "Box":
            # Box path goes through forward_continuous, not forward: hook the actor/critic
            h.remove()
            store = {"inputs": [], "grads": []}
            hs = []
            for sub in (alg.policy.net.actor, alg.policy.net.critic):
                hs.append(_net_grad_hooks(sub, store))
        alg.train()
        p = name + "_"
        out[p + "cfg"] = np.array([D, N, T, B, E, H, seed, aspace.n if hasattr(aspace, "n") else -aspace.shape[0]],
                                  np.int64)
        for k, v in init.items():
            out[p + "w0_" + k] = v
        for k, v in alg.policy.net.state_dict().items():
            out[p + "w1_" + k] = v.detach().numpy()
        tr = env.trace
        out[p + "env_obs"] = np.stack(tr["obs"])
        out[p + "env_rew"] = np.stack(tr["rew"])
        out[p + "env_done"] = np.stack(tr["done"])
        # rollout after collect (before get() flattened it we cannot see it; use batches)
        if not kw.get("no_batches"):
            for i, b in enumerate(batches):
                for f in b._fields:
                    out[p + f"mb{i}_{f}"] = getattr(b, f).numpy()
            for i, gs in enumerate(store["grads"]):
                for j, g in enumerate(gs):
                    out[p + f"mb{i}_grad{j}"] = g.numpy()
        out[p + "nmb"] = np.int64(len(batches))
        out[p + "np_state_after"] = np.random.get_state()[1].copy()
        for k in ("train/entropy_loss", "train/policy_gradient_loss", "train/value_loss", "train/total_loss"):
            out[p + k.split("/")[1]] = np.float64(rec[k])
    save("train_ppo", **out)


# --------------------------------------------------------------------------
# (6) PPO_RND: collect (warm-up + normalize_obs + rnd.int_reward + int_rew_rms
#     scaling, ppo.py:367-407) and train (ppo.py:409-502, incl. randn<0.25 gate)
# --------------------------------------------------------------------------
def gen_rnd(R):
    import torch
    out = {}
    rec = _record_logger(R)
    R.buffer.logger.record = R.logger.record
    D, N, T, B, E, H, IH, seed = 5, 4, 8, 16, 2, 16, 16, 31
    np.random.seed(seed)
    torch.manual_seed(seed)
    env = make_fakevec(R.VecEnv, N, D, Discrete(3), seed=2000 + seed)
    R.ppo.make_env = lambda env_id, n_envs=4: env
    alg = R.ppo.PPO_RND(env_id="Fake-v0", nstep=T, batch_size=B, n_epochs=E, hidden_size=H,
                        int_hidden_size=IH, rnd_start=3, max_grad_norm=0.5)
    init = {k: v.detach().clone().numpy() for k, v in alg.policy.net.state_dict().items()}
    rinit = {k: v.detach().clone().numpy() for k, v in alg.rnd.state_dict().items()}
    alg.collect_samples()  # first iteration: 2 warm-up steps then RND
    it1 = {"int_rewards": alg.rollout.int_rewards.copy(), "rewards": alg.rollout.rewards.copy(),
           "int_values": alg.rollout.int_values.copy(), "values": alg.rollout.values.copy(),
           "adv": alg.rollout.advantages.copy(), "iadv": alg.rollout.int_advantages.copy(),
           "obs_mean": np.asarray(alg.obs_rms.mean), "obs_var": np.asarray(alg.obs_rms.var),
           "obs_count": np.float64(alg.obs_rms.count), "ir_mean": np.asarray(alg.int_rew_rms.mean),
           "ir_var": np.asarray(alg.int_rew_rms.var), "ir_count": np.float64(alg.int_rew_rms.count)}
    alg.train()
    p = "rnd_"
    out[p + "cfg"] = np.array([D, N, T, B, E, H, IH, seed, 3], np.int64)
    for k, v in init.items():
        out[p + "w0_" + k] = v
    for k, v in rinit.items():
        out[p + "r0_" + k] = v
    for k, v in alg.policy.net.state_dict().items():
        out[p + "w1_" + k] = v.detach().numpy()
    for k, v in alg.rnd.state_dict().items():
        out[p + "r1_" + k] = v.detach().numpy()
    for k, v in it1.items():
        out[p + "it1_" + k] = v
    tr = env.trace
    out[p + "env_obs"] = np.stack(tr["obs"])
    out[p + "env_rew"] = np.stack(tr["rew"])
    out[p + "env_done"] = np.stack(tr["done"])
    for k in ("train/intrinsic_loss", "train/entropy_loss", "train/policy_gradient_loss",
              "train/value_loss", "train/total_loss"):
        out[p + k.split("/")[1]] = np.float64(rec[k])
    out[p + "mean_int_reward"] = np.float64(rec["rollout/mean_int_reward"])
    out[p + "np_state_after"] = np.random.get_state()[1].copy()
    save("train_rnd", **out)


# --------------------------------------------------------------------------
# (7) PPO_ICM: collect (int reward mix, ppo.py:603-649) + train (ppo.py:651-713)
# --------------------------------------------------------------------------
def gen_icm(R):
    import torch
    out = {}
    for name, aspace in (("icm_disc", Discrete(3)), ("icm_box", Box((2,)))):
        rec = _record_logger(R)
        D, N, T, B, E, H, IH, seed = 4, 3, 8, 12, 2, 16, 8, 41
        np.random.seed(seed)
        torch.manual_seed(seed)
        env = make_fakevec(R.VecEnv, N, D, aspace, seed=3000 + seed)
        R.ppo.make_env = lambda env_id, n_envs=4, env=env: env
        alg = R.ppo.PPO_ICM(env_id="Fake-v0", nstep=T, batch_size=B, n_epochs=E, hidden_size=H,
                            int_hidden_size=IH, max_grad_norm=0.5, int_rew_integration=0.1)
        init = {k: v.detach().clone().numpy() for k, v in alg.policy.net.state_dict().items()}
        iinit = {k: v.detach().clone().numpy() for k, v in alg.intrinsic_module.state_dict().items()}
        alg.collect_samples()
        roll = {"rewards": alg.rollout.rewards.copy(), "adv": alg.rollout.advantages.copy(),
                "actions": alg.rollout.actions.copy()}
        alg.train()
        p = name + "_"
        out[p + "cfg"] = np.array([D, N, T, B, E, H, IH, seed], np.int64)
        for k, v in init.items():
            out[p + "w0_" + k] = v
        for k, v in iinit.items():
            out[p + "i0_" + k] = v
        for k, v in alg.policy.net.state_dict().items():
            out[p + "w1_" + k] = v.detach().numpy()
        for k, v in alg.intrinsic_module.state_dict().items():
            out[p + "i1_" + k] = v.detach().numpy()
        for k, v in roll.items():
            out[p + "roll_" + k] = v
        tr = env.trace
        out[p + "env_obs"] = np.stack(tr["obs"])
        out[p + "env_rew"] = np.stack(tr["rew"])
        out[p + "env_done"] = np.stack(tr["done"])
        for k in ("train/entropy_loss", "train/policy_gradient_loss", "train/value_loss",
                  "train/total_loss", "train/icm_loss", "rollout/mean_int_reward"):
            out[p + k.split("/")[1]] = np.float64(rec[k])
    save("train_icm", **out)


# --------------------------------------------------------------------------
# (8) NatureCNN actor-critic architecture (.ipynb_checkpoints/models-checkpoint.py:48-90)
# --------------------------------------------------------------------------
def gen_cnn(R):
    import torch
    spec = importlib.util.spec_from_file_location(
        "models_checkpoint", os.path.join(REF, ".ipynb_checkpoints", "models-checkpoint.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    torch.manual_seed(51)
    net = mod.CnnActorCritic(4, 4)
    rs = np.random.RandomState(52)
    x = rs.randint(0, 256, size=(3, 4, 84, 84)).astype(np.uint8)
    with torch.no_grad():
        logits, value = net(torch.from_numpy(x.astype(np.float32)))
    out = {"x": x, "logits": logits.numpy(), "value": value.numpy()}
    # weights are NOT stored (7.8 MB): the oracle re-creates them from the same
    # torch seed + module order; per-tensor checksums pin that init.
    for k, v in net.state_dict().items():
        out["wsum_" + k] = np.float64(v.double().sum())
        out["wabs_" + k] = np.float64(v.double().abs().sum())
        out["whead_" + k] = v.flatten()[:16].numpy()
    out["param_count"] = np.int64(sum(p.numel() for p in net.parameters()))
    save("cnn", **out)


# --------------------------------------------------------------------------
# (9) One PPO iteration of the NatureCNN (the benchmarked Atari path): the live
#     ppo.PPO (ppo.py:121-259) with the checkpoint CnnActorCritic
#     (.ipynb_checkpoints/models-checkpoint.py:48-90) as policy.net.  Policy.act /
#     evaluate are net-agnostic for Discrete (models.py:30-73: self.net(obs) ->
#     (logits, values)), so only the net and its Adam are swapped after construction.
#     Frames are integer-valued float32 (4, 84, 84) stacks.  Recorded: the rollout after
#     collect (obs as uint8), the init checksums (the net is re-created from its torch
#     seed), post-train() weights (full small tensors, a fixed index sample of the large
#     ones + whole-tensor update sums), the loss scalars and numpy's RNG state.
# --------------------------------------------------------------------------
def _load_checkpoint_models():
    spec = importlib.util.spec_from_file_location(
        "models_checkpoint", os.path.join(REF, ".ipynb_checkpoints", "models-checkpoint.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def weight_sample_index(numel, k):
    """Fixed sample of flat indices of a large tensor (also recomputed by the tests)."""
    if numel <= 8192:
        return np.arange(numel, dtype=np.int64)
    return np.sort(np.random.RandomState(1000 + k).choice(numel, 8192, replace=False)).astype(np.int64)


def gen_cnn_train(R):
    import torch
    ck = _load_checkpoint_models()
    out = {}
    # env seeds chosen so the recorded trajectory is well-conditioned: the same program in
    # float64 (oracle, train_dtype=float64) lands within rtol 2e-5 / atol 2e-6 of the reference's
    # float32 weights (test_oracle_golden.test_cnn_fixture_is_well_conditioned).  With raw 0..255
    # pixels some trajectories are not (a ratio crossing a clip boundary, a saturated softmax):
    # there the reference's own f32 result is 10-400x further than that from exact arithmetic,
    # and no other f32 implementation can be held to it.
    for name, A, N, T, B, E, seed, net_seed, env_seed in (("cnn4", 4, 4, 16, 24, 2, 61, 62, 15061),
                                                          ("cnn18", 18, 2, 16, 12, 1, 63, 64, 6063)):
        rec = _record_logger(R)
        np.random.seed(seed)
        torch.manual_seed(seed)
        env = make_fakevec(R.VecEnv, N, None, Discrete(A), seed=env_seed, obs_shape=(4, 84, 84), frames=True)
        R.ppo.make_env = lambda env_id, n_envs=4, env=env: env
        alg = R.ppo.PPO(env_id="Fake-v0", nstep=T, batch_size=B, n_epochs=E)  # reference defaults otherwise
        torch.manual_seed(net_seed)
        net = ck.CnnActorCritic(4, A)
        alg.policy.net = net
        alg.optimizer = torch.optim.Adam(net.parameters(), lr=alg.lr)
        init = {k: v.detach().clone() for k, v in net.state_dict().items()}
        alg.collect_samples()
        st = alg.rollout
        p = name + "_"
        out[p + "cfg"] = np.array([N, T, B, E, A, seed, net_seed], np.int64)
        out[p + "obs"] = st.observations.astype(np.uint8)                   # (T, N, 4, 84, 84), integer-valued
        assert np.array_equal(out[p + "obs"].astype(np.float32), st.observations)
        for f in ("actions", "rewards", "values", "masks", "action_log_probs", "advantages", "returns"):
            out[p + "roll_" + f] = np.asarray(getattr(st, f)).copy()
        out[p + "last_obs"] = np.asarray(alg.last_obs).astype(np.uint8)
        alg.train()
        for k, (key, v0) in enumerate(init.items()):
            v1 = net.state_dict()[key].detach()
            out[p + "wsum0_" + key] = np.float64(v0.double().sum())
            out[p + "whead0_" + key] = v0.flatten()[:16].numpy()
            idx = weight_sample_index(v1.numel(), k)
            out[p + "w1idx_" + key] = idx
            out[p + "w1_" + key] = v1.flatten().numpy()[idx]
            d = (v1 - v0).double()
            out[p + "dsum_" + key] = np.float64(d.sum())
            out[p + "dabs_" + key] = np.float64(d.abs().sum())
        for k in ("train/entropy_loss", "train/policy_gradient_loss", "train/value_loss", "train/total_loss"):
            out[p + k.split("/")[1]] = np.float64(rec[k])
        out[p + "np_state_after"] = np.random.get_state()[1].copy()
        # the same iteration with train() in float64 (oracle; collect in f32 on the replayed
        # frames, as test_oracle_golden.test_cnn_fixture_is_well_conditioned re-runs it): the
        # exact-arithmetic losses the GPU test bounds the product's entropy against
        out.update(_cnn_f64_losses(out, p))
    save("train_cnn", **out)


def _cnn_f64_losses(f, p):
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
    sys.path.insert(0, os.path.dirname(OUT))
    from oracle import models as OM
    from oracle.algos import OraclePPO
    from replay_env import ReplayVecEnv, Discrete as RDiscrete
    N, T, B, E, A, seed, net_seed = (int(x) for x in f[p + "cfg"])
    obs = np.concatenate([f[p + "obs"], f[p + "last_obs"][None]])
    env = ReplayVecEnv(obs, f[p + "roll_rewards"], f[p + "roll_masks"].astype(bool), RDiscrete(A))
    state = np.random.get_state()
    np.random.seed(seed)
    torch.manual_seed(net_seed)
    alg = OraclePPO(env, nstep=T, batch_size=B, n_epochs=E, net=OM.NatureCNN(4, A), train_dtype=torch.float64)
    alg.collect()
    alg.train()
    np.random.set_state(state)
    out = {}
    for key, st in (("total_loss", "loss"), ("policy_gradient_loss", "pl"), ("value_loss", "vl"),
                    ("entropy_loss", "el")):
        out[p + "f64_" + key] = np.float64(alg.stats[st])
    return out


# --------------------------------------------------------------------------
# (9a) The same NatureCNN PPO iteration at the size the benchmark dispatches: 128 envs x
#      128 steps, ONE minibatch of 16,384 rows per epoch, 2 epochs (ppo.py:200-259 with
#      models-checkpoint.py:48-90).  At this batch the product runs its training-size kernel
#      forms (sg2 fc forward, the solo persistent conv2 dgrad, the split heads' hidden layer,
#      multi-slab split-K weight gradients).  The frames are not stored (462 MB): the env is
#      the Philox synthetic Atari env restated in oracle/philox.py (the numpy twin of the
#      device env, action-dependent counters), so the GPU test regenerates them bitwise on the
#      device from the recorded actions; a crc32 per step pins that.  The same iteration is
#      also run in float64 by the oracle on the reference's recorded rollout, so the test can
#      bound the product's error against exact arithmetic, next to the reference's own.
# --------------------------------------------------------------------------
def gen_cnn_train_big(R):
    import zlib
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
    from oracle.philox import SyntheticAtari
    from oracle import models as OM
    from oracle.algos import OraclePPO
    ck = _load_checkpoint_models()
    out = {}
    name, A, N, T, B, E, seed, net_seed, env_seed, p_done = "big", 4, 128, 128, 16384, 2, 71, 72, 17071, 5e-3

    class PhiloxFakeVec(R.VecEnv):
        """oracle.philox.SyntheticAtari with float32 observations (what the reference feeds its
        NatureCNN); no episode infos (the test checks the training update, not logging)."""

        def __init__(self):
            self.env = SyntheticAtari(N, env_seed, n_actions=A, p_done=p_done)
            self.num_envs = N
            self.observation_space = Box((4, 84, 84))
            self.action_space = Discrete(A)
            self.crc = []

        def _rec(self, o):
            self.crc.append(zlib.crc32(np.ascontiguousarray(o).tobytes()))
            return o.astype(np.float32)

        def reset(self):
            return self._rec(self.env.reset())

        def step(self, actions):
            o, r, d, _ = self.env.step(actions)
            return self._rec(o), r, d, [{} for _ in range(N)]

        def unnormalize_obs(self, obs):
            return obs

    rec = _record_logger(R)
    np.random.seed(seed)
    torch.manual_seed(seed)
    env = PhiloxFakeVec()
    R.ppo.make_env = lambda env_id, n_envs=4, env=env: env
    alg = R.ppo.PPO(env_id="Fake-v0", nstep=T, batch_size=B, n_epochs=E)  # reference defaults otherwise
    torch.manual_seed(net_seed)
    net = ck.CnnActorCritic(4, A)
    alg.policy.net = net
    alg.optimizer = torch.optim.Adam(net.parameters(), lr=alg.lr)
    init = {k: v.detach().clone() for k, v in net.state_dict().items()}
    alg.collect_samples()
    st = alg.rollout
    p = name + "_"
    out[p + "cfg"] = np.array([N, T, B, E, A, seed, net_seed, env_seed], np.int64)
    out[p + "p_done"] = np.float64(p_done)
    out[p + "obs_crc"] = np.array(env.crc, np.uint32)                      # reset + T steps
    roll = {}
    for f in ("actions", "rewards", "values", "masks", "action_log_probs", "advantages", "returns"):
        roll[f] = np.asarray(getattr(st, f)).copy()
        out[p + "roll_" + f] = roll[f]
    obs_ref = np.asarray(st.observations).copy()                          # (T, N, 4, 84, 84) f32
    alg.train()
    for k, (key, v0) in enumerate(init.items()):
        v1 = net.state_dict()[key].detach()
        out[p + "wsum0_" + key] = np.float64(v0.double().sum())
        out[p + "whead0_" + key] = v0.flatten()[:16].numpy()
        # the whole initial tensor: orthogonal_ runs LAPACK's QR, whose last bits differ between
        # CPUs, so the GPU test starts from these exact values instead of re-creating them
        out[p + "init_" + key] = v0.numpy()
        idx = weight_sample_index(v1.numel(), k)
        out[p + "w1idx_" + key] = idx
        out[p + "w1_" + key] = v1.flatten().numpy()[idx]
        d = (v1 - v0).double()
        out[p + "dsum_" + key] = np.float64(d.sum())
        out[p + "dabs_" + key] = np.float64(d.abs().sum())
    for k in ("train/entropy_loss", "train/policy_gradient_loss", "train/value_loss", "train/total_loss"):
        out[p + k.split("/")[1]] = np.float64(rec[k])
    out[p + "np_state_after"] = np.random.get_state()[1].copy()

    # the same train() in float64 (oracle, test infrastructure) on the reference's recorded
    # rollout: same initial weights, same permutations (numpy seeded as the reference's run)
    np.random.seed(seed)
    torch.manual_seed(net_seed)
    onet = OM.NatureCNN(4, A)
    for key, v in onet.state_dict().items():
        assert torch.equal(v, init[key]), key
    oalg = OraclePPO(PhiloxFakeVec(), nstep=T, batch_size=B,
                     n_epochs=E, net=onet, train_dtype=torch.float64)
    ro = oalg.rollout
    ro.obs[:] = obs_ref
    ro.actions[:] = roll["actions"].reshape(ro.actions.shape)
    ro.rewards[:], ro.values[:], ro.masks[:] = roll["rewards"], roll["values"], roll["masks"]
    ro.log_probs[:] = roll["action_log_probs"].reshape(ro.log_probs.shape)
    ro.pos = T
    ro.finish(roll["values"][T - 1], roll["masks"][T - 1])
    assert np.array_equal(ro.adv, roll["advantages"]) and np.array_equal(ro.ret, roll["returns"])
    oalg.train()
    assert np.array_equal(np.random.get_state()[1], out[p + "np_state_after"])
    for k, (key, v) in enumerate(onet.state_dict().items()):
        out[p + "w64_" + key] = v.flatten().numpy()[out[p + "w1idx_" + key]]
        out[p + "d64abs_" + key] = np.float64((v - init[key].double()).abs().sum())
    for key, stk in (("total_loss", "loss"), ("policy_gradient_loss", "pl"), ("value_loss", "vl"),
                     ("entropy_loss", "el")):
        out[p + "f64_" + key] = np.float64(oalg.stats[stk])
        print(f"  {key}: ref {float(out[p + key]):.9g}  f64 {oalg.stats[stk]:.9g}  "
              f"rel {abs(float(out[p + key]) - oalg.stats[stk]) / abs(oalg.stats[stk]):.3g}")
    del oalg
    for key in init:
        w, w64 = out[p + "w1_" + key].astype(np.float64), out[p + "w64_" + key]
        print(f"  {key}: max |ref - f64| {np.abs(w - w64).max():.3g}")

    # the FIRST minibatch's raw gradient (loss.backward(), before clip_grad_norm_ / Adam) at the
    # initial weights, by the oracle in float32 (torch-CPU: the reference's own arithmetic) and
    # float64, sampled like the weights: the GPU test compares the product's per-layer gradient
    # error with the reference's (a diagnostic finer than the post-Adam weights)
    from oracle.algos import _tensors, ppo_loss
    for dt, tag in ((torch.float32, "g32_"), (torch.float64, "g64_")):
        np.random.seed(seed)
        torch.manual_seed(net_seed)
        gnet = OM.NatureCNN(4, A).to(dt)
        galg = OraclePPO(PhiloxFakeVec(), nstep=T, batch_size=B, n_epochs=E, net=gnet, train_dtype=dt)
        ro = galg.rollout
        ro.obs[:] = obs_ref
        ro.actions[:] = roll["actions"].reshape(ro.actions.shape)
        ro.rewards[:], ro.values[:], ro.masks[:] = roll["rewards"], roll["values"], roll["masks"]
        ro.log_probs[:] = roll["action_log_probs"].reshape(ro.log_probs.shape)
        ro.pos = T
        ro.finish(roll["values"][T - 1], roll["masks"][T - 1])
        _idx, mb = next(ro.minibatches(B))
        mb = _tensors(mb, dt)
        v, _, lp, ent = OM.evaluate(gnet, mb["observations"], mb["actions"], False, dt)
        with torch.no_grad():  # the first minibatch's forward outputs, in minibatch order
            logits = gnet.heads(mb["observations"])[0]
        out[p + "mb0_v" + tag[1:3]] = v.detach().double().numpy()
        out[p + "mb0_logits" + tag[1:3]] = logits.double().numpy()
        loss, _, _, _ = ppo_loss(v, lp, ent, mb, galg.clip, galg.ent_coef, galg.vf_coef)
        loss.backward()
        for k, (key, prm) in enumerate(gnet.named_parameters()):
            out[p + tag + key] = prm.grad.detach().double().flatten().numpy()[out[p + "w1idx_" + key]]
        del galg, ro, mb
    for key in init:
        g32, g64 = out[p + "g32_" + key], out[p + "g64_" + key]
        print(f"  grad {key}: max |g32 - g64| / max |g64| {np.abs(g32 - g64).max() / np.abs(g64).max():.3g}")
    save("train_cnn_big", **out)


# --------------------------------------------------------------------------
# (9b) logger CSV schema (logger.py:13-58, 195-234): configure(log_to_file=True) and
#      three dumps whose later ones bring new keys (the header is rewritten and the
#      earlier rows padded); the stdout table of the first dump is recorded too.
# --------------------------------------------------------------------------
def gen_logger(R):
    import io
    import tempfile
    import contextlib
    lg = importlib.reload(R.logger)  # earlier generators replaced record/dump/configure
    dumps = [
        {"time/total timesteps": 512, "time/total_time": 1.25},
        {"time/total timesteps": 1024, "rollout/ep_rew_mean": 3.5, "rollout/num_episodes": 7,
         "time/total_time": 2.5, "train/entropy_loss": -1.3862, "train/policy_gradient_loss": -0.0125,
         "train/value_loss": 0.5, "train/total_loss": 0.48},
        {"Progress": "66.67%", "time/total timesteps": 1536, "rollout/mean_int_reward": 0.03125,
         "train/icm_loss": 0.25, "time/total_time": 3.75},
    ]
    with tempfile.TemporaryDirectory() as d:
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            lg.configure("PPO", "Fake-v0", log_to_file=True, folder=d)
        lg.Logger.CURRENT.outputs[0].file = buf   # stdout table into the buffer
        tables = []
        for kv in dumps:
            start = len(buf.getvalue())
            for k, v in kv.items():
                lg.record(k, v)
            lg.dump(step=0)
            tables.append(buf.getvalue()[start:])
        folder = os.path.join(d, "PPO", "Fake-v0")
        (csv_name,) = os.listdir(folder)
        text = open(os.path.join(folder, csv_name)).read()
    out = {"n_dumps": np.int64(len(dumps)), "csv": np.array(text), "table0": np.array(tables[0]),
           "table1": np.array(tables[1])}
    for i, kv in enumerate(dumps):
        out[f"d{i}_keys"] = np.array(list(kv.keys()))
        out[f"d{i}_vals"] = np.array([repr(v) for v in kv.values()])
    save("logger", **out)


# --------------------------------------------------------------------------
# (10) ES-NSRA pieces: FeedForwardNetwork.predict (evolution_strategies.py:50-63),
#      EvolutionStrategy._update_weights (:224-246), get_kNN (:273-289),
#      calc_noveltiy_distribution (:291-297).  evolution_strategies.py imports gym and
#      pybulletgym at module level (:8-9); the stubs below only satisfy those imports and
#      gym.make (called by __init__, :121) — evaluate()/get_behavior_char() need MuJoCo
#      and are not recorded.
# --------------------------------------------------------------------------
def gen_es(R):
    class FakeEnv:
        def __init__(self, obs_dim, act_dim):
            self.observation_space = Box((obs_dim,))
            self.action_space = Box((act_dim,))

    gym = sys.modules["gym"]
    gym.make = lambda env_id: FakeEnv(8, 2)
    sys.modules.setdefault("pybulletgym", types.ModuleType("pybulletgym"))
    import evolution_strategies as ES
    out = {}
    # predict: f64 arctan MLP, tanh head (Box)
    np.random.seed(21)
    net = ES.FeedForwardNetwork(FakeEnv(8, 2), hidden_sizes=[16, 12])
    obs = np.random.randn(20, 8)
    out["pred_w0"], out["pred_w1"], out["pred_w2"] = [w.copy() for w in net.get_weights()]
    out["pred_obs"] = obs
    out["pred_act"] = np.stack([net.predict(o) for o in obs]).reshape(20, -1)
    # _update_weights on a recorded population (numpy RNG: layer-major per member, :176-186)
    for tag, novelty, npar in (("a", 0.37, 0.5), ("b", 1.0, 0.8)):
        np.random.seed(5 if tag == "a" else 6)
        es = ES.EvolutionStrategy("Swimmer-v3", hidden_sizes=[16, 12], population_size=40, sigma=0.1,
                                  learning_rate=0.01, decay=0.9995, novelty_param=npar)
        w_before = [w.copy() for w in es.get_weights()]
        pop = es._get_population()
        rewards = np.random.randn(40) * 3 + 1
        es._update_weights(rewards, pop, novelty)
        for i in range(3):
            out[f"upd_{tag}_w{i}_before"] = w_before[i]
            out[f"upd_{tag}_w{i}_after"] = es.get_weights()[i].copy()
            out[f"upd_{tag}_pop{i}"] = np.array([p[i] for p in pop])
        out[f"upd_{tag}_rewards"] = rewards
        out[f"upd_{tag}_meta"] = np.array([novelty, npar, 0.01, 40, 0.1, es.learning_rate])
    # kNN novelty distance: sum of the S nearest Euclidean distances (sklearn NearestNeighbors)
    np.random.seed(9)
    for n in (1, 3, 10, 57):
        arch = [np.random.randn(1, 2) for _ in range(n)]
        bc = np.random.randn(1, 2)
        S = min(10, n)
        es.K = 10
        out[f"knn_{n}_archive"] = np.concatenate(arch)
        out[f"knn_{n}_bc"] = bc
        out[f"knn_{n}_dist"] = np.array(es.get_kNN(arch, bc, S))
    nov = np.abs(np.random.randn(2)) + 0.01
    out["probs_in"] = nov
    out["probs_out"] = np.array(es.calc_noveltiy_distribution(list(nov)))
    save("es", **out)

def main():
    if not os.path.isdir(REF):
        print("reference not present; fixtures are committed — nothing to do")
        return 0
    R = import_reference()
    if len(sys.argv) > 1:  # regenerate selected fixtures only, e.g. `simhash`
        for name in sys.argv[1:]:
            globals()["gen_" + name](R)
        return 0
    gen_gae(R)
    gen_gae_dual(R)
    gen_rms(R)
    gen_get(R)
    gen_simhash(R)
    gen_train(R)
    gen_rnd(R)
    gen_icm(R)
    gen_cnn(R)
    gen_cnn_train(R)
    gen_logger(R)
    gen_es(R)
    return 0


if __name__ == "__main__":
    sys.exit(main())
