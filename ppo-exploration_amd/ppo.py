"""PPO, PPO+RND and PPO+ICM on MI355X — the reference's algorithm API
(reference: ppo.py / algorithms.py:22-756) over the libppox hot path.

    PPO(env_id=..., lr=3e-4, nstep=128, batch_size=128, n_epochs=10, ...)
        .collect_samples()  (alias collect_rollouts)   ppo.py:166-198
        .train()                                       ppo.py:200-259
        .learn(total_timesteps, log_interval, reward_target=None, log_to_file=False)

Keyword arguments and defaults are the reference's; added keywords:
n_envs (the reference hard-codes 4, ppo.py:52), seed, device, env (a device env
object; default: the synthetic env for env_id), quiet.

Per iteration on each rank:
  collect: T x [net forward (rocBLAS + MFMA convs) -> ppox_categorical_sample ->
            ppox_*_env_step writing slot t+1]            (+ RND / ICM rewards)
  GAE:     ppox_gae / ppox_gae_dual (bit-identical to buffer.py:203-230)
  train:   per epoch one numpy permutation (buffer.py:239) + ppox_minibatch_adv_stats;
           per minibatch ppox_gather_rows -> forward -> ppox_ppo_loss_partials
           -> [all-reduce 4 KB] -> ppox_ppo_loss_backward -> backward into the flat
           grad bucket -> [all-reduce] -> ppox_grad_sumsq + ppox_adam_step.
There is no CPU fallback: every step needs libppox.so and a GPU.
"""
import os
import time
from collections import deque

import numpy as np
import torch
import torch.nn.functional as F

import logger
import native
import convs
import icm as icm_native
from buffer import IntrinsicStorage, RolloutStorage
from dist import DistContext, owned_minibatch_indices, owned_minibatch_positions, shard_range
from env import DeviceAtariEnv, make_env
from phases import traced
from models import CnnActorCritic, FlatParams, IntrinsicCuriosityModule, MlpNetwork, RndNetwork
from util import ActionConverter, RunningMeanStd


def _is_image(space):
    return len(space.shape) == 3


_TRAIN_PRIO = native.ab_env("PPOX_TRAIN_PRIO", "0") == "1"
_prio_streams = {}


class _train_stream:
    """PPOX_TRAIN_PRIO=1: the update's main-stream work on a high-priority stream (the weight
    gradients' side stream keeps the default priority), ordered after / before the caller's stream."""

    def __init__(self, device):
        self.on = _TRAIN_PRIO and device.type == "cuda"
        self.device = device

    def __enter__(self):
        if not self.on:
            return
        s = _prio_streams.get(self.device)
        if s is None:
            s = _prio_streams[self.device] = torch.cuda.Stream(device=self.device, priority=-1)
        self.prev = torch.cuda.current_stream(self.device)
        s.wait_stream(self.prev)
        self.ctx = torch.cuda.stream(s)
        self.ctx.__enter__()

    def __exit__(self, *exc):
        if not self.on:
            return False
        s = torch.cuda.current_stream(self.device)
        self.ctx.__exit__(*exc)
        self.prev.wait_stream(s)
        return False


def icm_loss_sharded(icm, x, acts, pos, B, beta, ctx):
    """ICM loss of one GLOBAL minibatch whose rows are spread over ranks (ppo.py:684-692):
    pairs are consecutive rows of the permuted minibatch, (row j, row j+1), j < B-1,
    whatever rank owns them.  x / acts: this rank's owned rows (permutation order),
    pos: their positions in the minibatch.  Encoder features and actions are summed
    into global positions (all-reduce of B x h f32 + B actions), each rank evaluates
    the pairs whose first row it owns, and the feature gradient is all-reduced back to
    the owners — so the gradients equal the single-process ones.  Backpropagates into
    the ICM parameters' .grad and returns this rank's share of the loss (sum over ranks
    = the reference's icm_loss)."""
    h = icm.feature_size
    phi = icm.state_encoder(x)
    npair = B - 1

    def pair_loss(s_ft, n_ft, a_s):  # a_s: the action taken at the pair's first row
        a_hat = icm.inverse_model(torch.cat((s_ft, n_ft), 1))
        n_hat = icm.forward_model(torch.cat((s_ft, icm.encode_action(a_s)), 1))
        fwd = ((n_hat - n_ft) ** 2).sum() / (npair * h)                # F.mse_loss, mean over (B-1) x h
        if icm.discrete:
            inv = F.cross_entropy(a_hat, a_s, reduction="sum") / npair
        else:
            inv = ((a_hat - a_s) ** 2).sum() / (npair * a_hat.shape[1])
        return (1 - beta) * inv + beta * fwd

    if not ctx.enabled:
        # one process: the rows are the minibatch in order, so the pairs are two slices (no
        # gathers: torch's indexing backward on ROCm took ~190 us per minibatch of 2048)
        a = acts.reshape(-1).long() if icm.discrete else acts.float()
        loss = pair_loss(phi[:-1], phi[1:], a[:-1])
        loss.backward()
        return loss.detach()
    full = torch.zeros(B, h, dtype=phi.dtype, device=phi.device)
    full[pos] = phi.detach()
    ctx.all_reduce_(full)
    if icm.discrete:
        a_full = torch.zeros(B, dtype=torch.int64, device=phi.device)
        a_full[pos] = acts.reshape(-1).long()
    else:
        a_full = torch.zeros(B, acts.shape[-1], dtype=torch.float32, device=phi.device)
        a_full[pos] = acts.float()
    ctx.all_reduce_(a_full)
    j = pos[pos < B - 1]
    # the pairs' features as leaves; their gradients are scattered back with index_add_ (each
    # of j, j + 1 holds distinct rows, so each row adds at most two terms: the same sums as
    # autograd's indexing backward, without its slow kernel)
    s_ft = full[j].requires_grad_(True)
    n_ft = full[j + 1].requires_grad_(True)
    loss = pair_loss(s_ft, n_ft, a_full[j])
    loss.backward()
    g = torch.zeros_like(full)
    if s_ft.grad is not None:
        g.index_add_(0, j, s_ft.grad)
    if n_ft.grad is not None:
        g.index_add_(0, j + 1, n_ft.grad)
    g = ctx.all_reduce_(g)
    if phi.shape[0]:
        phi.backward(g[pos])
    return loss.detach()


class Policy:
    """models.py:15-124 interface (act / evaluate) over a device network."""

    def __init__(self, env, hidden_size, intrinsic_model=False):
        self.env = env
        self.action_type = env.action_space.__class__.__name__
        self.action_dim = env.action_space.n if self.action_type == "Discrete" else env.action_space.shape[0]
        self.intrinsic = intrinsic_model
        shape = env.observation_space.shape
        if _is_image(env.observation_space):
            self.net = CnnActorCritic(shape[0], self.action_dim, intrinsic=intrinsic_model)
        else:
            self.net = MlpNetwork(shape[0], self.action_dim, hidden_size, intrinsic=intrinsic_model)

    def parameters(self):
        return self.net.parameters()

    def _dist(self, out):
        if self.action_type == "Discrete":
            return torch.distributions.Categorical(F.softmax(out, dim=-1))
        mean = out.tanh()
        return torch.distributions.Normal(mean, torch.exp(self.net.action_log_std.expand_as(mean)))

    def act(self, obs):
        """models.py:30-50 / 75-99."""
        out, v, iv = self.net(torch.as_tensor(obs, device=self.net.action_log_std.device
                                              if hasattr(self.net, "action_log_std") else None))
        d = self._dist(out)
        a = d.sample()
        lp = d.log_prob(a)
        return (a, v, iv, lp) if self.intrinsic else (a, v, lp)

    def evaluate(self, obs, actions):
        """models.py:52-73 / 101-124."""
        out, v, iv = self.net(obs)
        d = self._dist(out)
        if self.action_type == "Discrete":
            lp = d.log_prob(actions.flatten()).unsqueeze(1)
        else:
            lp = d.log_prob(actions)
        return (v, iv, lp, d.entropy()) if self.intrinsic else (v, lp, d.entropy())


# (A/B) PPOX_SHARED_GPU_STREAMS=1: ranks sharing a GPU keep the backward's side stream;
# PPOX_DENSE_EARLY=0: the fc + heads bucket's all-reduce starts after the whole backward, from the main stream
SHARED_GPU_STREAMS = native.ab_env("PPOX_SHARED_GPU_STREAMS", "0") == "1"
DENSE_EARLY = native.ab_env("PPOX_DENSE_EARLY", "1") != "0"


class BaseAlgorithm:
    """ppo.py:22-118."""

    def __init__(self, env_id, lr, nstep, batch_size, n_epochs, gamma, gae_lam, clip_range, ent_coef, vf_coef,
                 max_grad_norm, n_envs=4, seed=0, device=None, env=None, quiet=False):
        self.env_id = env_id
        self.dist = DistContext.current()
        self.device = torch.device(device or "cuda")
        native.lib()  # fail loudly: no GPU / no libppox => no product path
        if self.device.type == "cuda" and self.dist.enabled:
            # ranks sharing one GPU (the 8-rank tests on a one-GPU box) run the backward on one stream: with the
            # side stream, 8 processes x (main, side, collective streams) oversubscribe the hardware queues, and
            # there about one 8-rank run in two had one corrupted rank pass (open); one rank per GPU
            # keeps the side stream
            idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
            if (convs.BWD_STREAMS and not SHARED_GPU_STREAMS
                    and self.dist.ranks_on_device(torch.device("cuda", idx)) > 1):
                convs.BWD_STREAMS = False
        self.num_envs = n_envs
        self.env_offset, self.local_envs = shard_range(n_envs, self.dist.rank, self.dist.world)
        self.seed = seed
        self.env = env if env is not None else make_env(env_id, n_envs=self.local_envs, seed=seed,
                                                        env_offset=self.env_offset, device=self.device)
        self.state_dim = self.env.observation_space.shape[0]
        self.action_converter = ActionConverter(self.env.action_space)
        self.discrete = self.action_converter.action_type == "Discrete"
        self.n_actions = self.action_converter.num_actions
        self.lr, self.nstep, self.batch_size, self.n_epochs = lr, nstep, batch_size, n_epochs
        self.gamma, self.gae_lam, self.clip_range = gamma, gae_lam, clip_range
        self.ent_coef, self.vf_coef, self.max_grad_norm = ent_coef, vf_coef, max_grad_norm
        self._ep_info_buffer = deque(maxlen=50)
        self._pending_episodes = None  # a collect's (returns, lengths) host copy, booked on first read
        self._ep_host = None
        self._n_updates = 0
        self.num_timesteps = 0
        self._num_episodes = 0
        self.quiet = quiet
        self.obs_rms = RunningMeanStd(device=self.device)
        self._sample_counter = 0
        self._started = False

    # ---------------------------------------------------------------- helpers
    def _attach_convs(self):
        if isinstance(self.policy.net, CnnActorCritic):
            convs.attach(self.policy.net, self.flat)

    def _new_rollout(self, cls, **kw):
        return cls(self.nstep, self.local_envs, self.env.observation_space, self.env.action_space,
                   device=self.device, **kw)

    def _alloc_train_state(self):
        d = self.device
        self.loss_partials = torch.zeros(native.LOSS_PARTIALS * 8, dtype=torch.float64, device=d)
        self.loss_accum = torch.zeros(8, dtype=torch.float64, device=d)
        if not self.discrete:
            self.dls_partials = torch.zeros(native.LOSS_PARTIALS * self.n_actions, dtype=torch.float64, device=d)
            self.dls = torch.zeros(self.n_actions, device=d)

    def _loss_grads(self, od, vd, ivd, idx, roll, stats, B_global, int_vf_coef, scale):
        """K4 for one minibatch: partial sums -> all-reduce -> backward to the head outputs
        (ppo.py:216-238).  Discrete: Categorical kernels; Box: Normal kernels, whose
        dL/d(action_log_std) goes straight into the flat gradient (before its all-reduce).
        Returns (d_out, d_value, d_int_value or None)."""
        Bl, A, T, N = idx.numel(), self.n_actions, self.nstep, self.local_envs
        if self.discrete:
            native.ppo_loss_partials(od, vd, ivd, Bl, A, idx, T, N, roll, stats, self.clip_range, self.loss_partials)
        else:
            ls = self.policy.net.action_log_std.detach()
            native.ppo_box_loss_partials(od, ls, vd, ivd, Bl, A, idx, T, N, roll, stats, self.clip_range,
                                         self.loss_partials)
        self.dist.all_reduce_(self.loss_partials)
        dout, dv = torch.empty_like(od), torch.empty_like(vd)
        div = torch.empty_like(ivd) if ivd is not None else None
        if self.discrete:
            native.ppo_loss_backward(od, vd, ivd, Bl, A, idx, T, N, roll, stats, self.clip_range, self.loss_partials,
                                     B_global, self.ent_coef, self.vf_coef, int_vf_coef, scale, dout, dv, div,
                                     self.loss_accum)
        else:
            native.ppo_box_loss_backward(od, ls, vd, ivd, Bl, A, idx, T, N, roll, stats, self.clip_range,
                                         self.loss_partials, B_global, self.ent_coef, self.vf_coef, int_vf_coef,
                                         scale, dout, self.dls_partials, self.dls, dv, div, self.loss_accum)
            g = self.policy.net.action_log_std.grad
            g.add_(self.dls.view_as(g))
        return dout, dv, div

    def _empty_outputs(self, intrinsic=False):
        """Zero-row head outputs (out, value, int value) for a rank that owns no rows of a minibatch."""
        z = torch.zeros(0, device=self.device)
        return torch.zeros(0, self.n_actions, device=self.device), z, (z if intrinsic else None)

    def _fwd_train(self, obs):
        """Training forward of the policy net -> (out, v, iv, ctx).  NatureCNN nets on the
        libppox trunk take the explicit path (models.CnnActorCritic.forward_train: no
        autograd graph, grads accumulated straight into the flat buffer); others autograd."""
        net = self.policy.net
        if getattr(net, "conv_impl", None) is not None and hasattr(net, "forward_train"):
            return net.forward_train(obs)
        out, v, iv = net(obs)
        return out, v, iv, None

    def _train_obs(self, ro, idx):
        """Minibatch observations for the policy's training forward: the rows left in the
        rollout (convs.RolloutRows: the split conv1 forward and weight-gradient kernels read
        them through idx, no gather) when the NatureCNN trunk runs conv1 in split math on uint8
        frames; otherwise the gathered rows (buffer.py:97-109)."""
        net = self.policy.net
        cv = getattr(net, "conv_impl", None)
        obs = ro.observations
        if (cv is not None and hasattr(net, "forward_train") and obs.dtype == torch.uint8 and obs.dim() == 5
                and cv.uses_split("fwd", 1) and cv.uses_split("wgrad", 1)):
            return convs.RolloutRows(obs, idx)
        return ro._gather(obs, idx)

    def _zero_policy_grad(self, rows):
        """The explicit NatureCNN backward overwrites every policy gradient (models.py
        CnnActorCritic.backward_train), so the flat buffer is zeroed only for autograd nets
        or a minibatch with no rows on this rank (its all-reduce contribution is zero)."""
        net = self.policy.net
        if rows == 0 or getattr(net, "conv_impl", None) is None or not hasattr(net, "backward_train"):
            self.flat.zero_grad()

    def _bwd_reduce(self, ctx, out, v, iv, dout, dv, div=None, has_rows=True):
        """Backward into the flat grad bucket + its all-reduce over ranks.  On the explicit
        NatureCNN path at world > 1 the bucket is reduced in two pieces: the fc + head part
        (flat params after the convs, 96 % of the bytes) asynchronously as soon as backward_train
        has produced it, overlapping the conv backward, then the conv part."""
        net = self.policy.net
        if self.dist.enabled and getattr(net, "conv_impl", None) is not None and hasattr(net, "backward_train"):
            # the collective sequence depends only on state every rank shares (world size and the
            # net type), never on this rank's row count: a rank with no rows of the minibatch
            # issues the same two all-reduces on its zeroed bucket (otherwise the ranks mismatch)
            n0 = (net.feature_extractor[7].weight.data_ptr() - self.flat.data.data_ptr()) // 4
            work = []
            start = lambda: work.append(self.dist.all_reduce_async_(self.flat.grad[n0:]))  # noqa: E731
            if has_rows:
                net.backward_train(ctx, dout, dv, div, dense_ready=start if DENSE_EARLY else None)
            if not (has_rows and DENSE_EARLY):
                start()
            for w in work:  # (the communicator's reductions run one at a time, in issue order)
                w.wait()
            self.dist.all_reduce_(self.flat.grad[:n0])
            return
        if has_rows:
            self._bwd_train(ctx, out, v, iv, dout, dv, div)
        self.dist.all_reduce_(self.flat.grad)

    def _bwd_train(self, ctx, out, v, iv, dout, dv, div=None, extra=None):
        """Backward of _fwd_train's outputs (+ an optional extra scalar loss with its own graph)."""
        if ctx is not None:
            self.policy.net.backward_train(ctx, dout, dv, div)
            if extra is not None:
                torch.autograd.backward([extra])
            return
        tensors, grads = [out, v], [dout, dv]
        if iv is not None and div is not None:
            tensors.append(iv)
            grads.append(div)
        if extra is not None:
            tensors.append(extra)
            grads.append(None)
        torch.autograd.backward(tensors, grads)

    def _ensure_started(self):
        if not self._started:
            self.env.reset_into(self.rollout.obs_slots[0])
            self._started = True
        else:
            self.rollout.obs_slots[0].copy_(self.rollout.obs_slots[self.nstep])

    def _sample_actions(self, out, t):
        ro = self.rollout
        if self.discrete:
            native.categorical_sample(out, self.local_envs, self.n_actions, self.env_offset, self.seed,
                                      self._sample_counter, ro.actions[t], ro.log_probs[t])
        else:  # Normal(tanh(mu), exp(action_log_std)) (models.py:42-45), Philox + Box-Muller
            native.normal_sample(out.contiguous(), self.policy.net.action_log_std.detach(), self.local_envs,
                                 self.n_actions, self.env_offset, self.seed, self._sample_counter, ro.actions[t],
                                 ro.log_probs[t])
        self._sample_counter += 1

    @traced("episodes")
    def _finish_episodes(self):
        """Episode bookkeeping of one rollout over ALL envs (ppo.py:180-183, 98-109): every rank
        gathers the (T, N_global) episode returns / lengths, so num_episodes, ep_info_buffer and
        the reward_target decision of learn() are identical on every rank (the reference's
        step-then-env order: row-major over (t, env)).  The gather is enqueued here; the host
        reads it only when ep_info_buffer / num_episodes are next read (the reference's own
        readers: the log line, learn()'s reward_target test) — not here, where a device->host
        copy would stall the host behind the whole collect and delay train()'s first launches."""
        ro = self.rollout
        ret = self.dist.all_gather_cat(ro.done_ret, dim=1)
        ln = self.dist.all_gather_cat(ro.done_len, dim=1)
        # an earlier collect nobody read (consecutive collects): its copy landed long ago, so this is
        # host work only, beside this collect's kernels
        self._book_episodes()
        host = self._ep_host
        if host is None or host[0].shape != ret.shape:
            pin = self.device.type == "cuda"
            host = self._ep_host = (torch.empty(ret.shape, dtype=ret.dtype, pin_memory=pin),
                                    torch.empty(ln.shape, dtype=ln.dtype, pin_memory=pin))
        host[0].copy_(ret, non_blocking=True)
        host[1].copy_(ln, non_blocking=True)
        ev = torch.cuda.Event() if self.device.type == "cuda" else None
        if ev is not None:
            ev.record()
        self._pending_episodes = (host[0], host[1], ev)

    def _book_episodes(self):
        if self._pending_episodes is None:
            return
        h_ret, h_ln, ev = self._pending_episodes
        self._pending_episodes = None
        if ev is not None:
            ev.synchronize()
        ret, ln = h_ret.numpy(), h_ln.numpy()
        fin = ~np.isnan(ret)
        r_fin, l_fin = ret[fin], ln[fin]  # row-major over (t, env), as the reference appends
        n_fin = int(r_fin.size)
        self._num_episodes += n_fin
        # the buffer keeps its last maxlen entries: appending only the last maxlen finished
        # episodes leaves it exactly as appending all of them (thousands per rollout at 4096
        # envs: the per-episode host loop cost ~47 ms per iteration with the GPU idle)
        k = min(n_fin, self._ep_info_buffer.maxlen)
        if k:
            for x, y in zip(r_fin[-k:], l_fin[-k:]):
                self._ep_info_buffer.append({"r": float(x), "l": int(y)})

    @property
    def ep_info_buffer(self):
        """deque(maxlen=50) of the last finished episodes' {"r", "l"} (ppo.py:98-109)."""
        self._book_episodes()
        return self._ep_info_buffer

    @property
    def num_episodes(self):
        self._book_episodes()
        return self._num_episodes

    @num_episodes.setter
    def num_episodes(self, v):
        self._num_episodes = v

    def _batch(self, total):
        """Minibatch size: batch_size=None is one full-rollout minibatch (buffer.py:248-249)."""
        return total if self.batch_size is None else int(self.batch_size)

    def _epoch_minibatches(self, total):
        """One global numpy permutation (buffer.py:239) -> per-minibatch (local idx, global size)."""
        perm = np.random.permutation(total)
        bs = self._batch(total)
        sizes = [min(bs, total - s) for s in range(0, total, bs)]
        # pinned staging: a pageable host->device copy blocks the host until the stream
        # drains, idling the GPU while the next epoch's permutation is drawn
        perm_dev = self._h2d(perm)
        if not self.dist.enabled:
            offs = np.concatenate([[0], np.cumsum(sizes)])
            return perm_dev, perm_dev, offs, sizes
        local, offs = owned_minibatch_indices(perm, self.nstep, self.env_offset, self.local_envs, bs)
        self._epoch_pos = self._h2d(owned_minibatch_positions(perm, self.nstep, self.env_offset, self.local_envs, bs))
        return perm_dev, self._h2d(local), offs, sizes

    def _h2d(self, a):
        t = torch.from_numpy(np.ascontiguousarray(a))
        if self.device.type == "cuda":
            t = t.pin_memory()
        return t.to(self.device, non_blocking=True)

    def _global_advantages(self, ro, intrinsic=False):
        adv = self.dist.all_gather_cat(ro.advantages, dim=1)
        iadv = self.dist.all_gather_cat(ro.int_advantages, dim=1) if intrinsic else None
        return adv, iadv

    def _record_train(self, extra=None):
        acc = self.loss_accum.cpu().numpy()
        n = max(acc[5], 1.0)
        logger.record("train/entropy_loss", acc[2] / n)
        logger.record("train/policy_gradient_loss", acc[0] / n)
        logger.record("train/value_loss", acc[1] / n)
        logger.record("train/total_loss", (acc[3] + (extra or 0.0)) / n)
        return acc

    def normalize_obs(self, obs):
        """ppo.py:111-118 -> f32 device tensor (rows, features)."""
        x = obs.reshape(obs.shape[0], -1)
        # a never-updated shape-() RunningMeanStd normalises by broadcasting, as numpy does in
        # the reference: give it its per-feature (identical-valued) state first
        self.obs_rms._features(x.shape[1])
        out = torch.empty(x.shape, dtype=torch.float32, device=self.device)
        native.normalize_obs(x, x.shape[0], x.shape[1], x.stride(0), self.obs_rms.mean, self.obs_rms.var, out)
        return out

    def update_info_buffer(self, infos, dones=None):
        for info in infos:
            ep = info.get("episode")
            if ep is not None:
                self.ep_info_buffer.extend([ep])

    # ------------------------------------------------------------------ learn
    def _log_iteration(self, start_time, extra=None):
        logger.record("time/total timesteps", self.num_timesteps)
        if len(self.ep_info_buffer) > 0:
            logger.record("rollout/ep_rew_mean", float(np.mean([e["r"] for e in self.ep_info_buffer])))
            logger.record("rollout/num_episodes", self.num_episodes)
        if extra:
            for k, v in extra.items():
                logger.record(k, v)
        el = time.time() - start_time
        logger.record("time/total_time", el)
        logger.record("time/env_steps_per_s", self.num_timesteps / max(el, 1e-9))
        logger.dump(step=self.num_timesteps)

    def _learn(self, algo_name, total_timesteps, log_interval, reward_target, log_to_file, progress=False):
        if self.dist.rank == 0:
            logger.configure(algo_name, self.env_id, log_to_file, quiet=self.quiet)
        else:
            logger.configure(algo_name, self.env_id, False, quiet=True)
        start = time.time()
        it = 0
        while self.num_timesteps < total_timesteps:
            prog = round(self.num_timesteps / total_timesteps * 100, 2)
            self.collect_samples()
            it += 1
            if log_interval is not None and it % log_interval == 0:
                self._log_iteration(start, {"Progress": f"{prog}%"} if progress else None)
            self.train()
            if reward_target is not None and len(self.ep_info_buffer) and \
                    np.mean([e["r"] for e in self.ep_info_buffer]) > reward_target:
                self._log_iteration(start)
                break
        return self

    def collect_rollouts(self):
        """north_star name for collect_samples (ppo.py:80 docstring)."""
        return self.collect_samples()


class PPO(BaseAlgorithm):
    """ppo.py:121-308."""

    def __init__(self, *, env_id, lr=3e-4, nstep=128, batch_size=128, n_epochs=10, gamma=0.99, gae_lam=0.95,
                 clip_range=0.2, ent_coef=.01, vf_coef=1, max_grad_norm=0.2, hidden_size=128, sim_hash=False,
                 sil=False, n_envs=4, seed=0, device=None, env=None, quiet=False):
        if sil:
            raise NotImplementedError("self-imitation (sil=True) is broken in the reference "
                                      "(sil_module.py:14 vs buffer.py:406) and out of scope")
        super().__init__(env_id, lr, nstep, batch_size, n_epochs, gamma, gae_lam, clip_range, ent_coef, vf_coef,
                         max_grad_norm, n_envs=n_envs, seed=seed, device=device, env=env, quiet=quiet)
        self.policy = Policy(self.env, hidden_size)
        self.rollout = self._new_rollout(RolloutStorage, gae_lam=gae_lam, gamma=gamma, sim_hash=sim_hash)
        self.flat = FlatParams(self.policy.net, self.device)
        self._attach_convs()
        self.optimizer = self.flat
        self.sim_hash, self.sil = sim_hash, sil
        self._alloc_train_state()
        self.last_obs = None
        # the collect step loop as one captured graph (PPOX_COLLECT_GRAPH=0: eager launches)
        self._collect_graph_enabled = native.ab_env("PPOX_COLLECT_GRAPH", "1") != "0"
        self._cgraph = None
        self._ctables = None

    def _collect_graph_ok(self):
        return (self._collect_graph_enabled and isinstance(self.env, DeviceAtariEnv) and self.discrete
                and not self.rollout.do_hash and getattr(self.policy.net, "conv_impl", None) is not None
                and self.device.type == "cuda")

    def _collect_steps_eager(self):
        ro, net = self.rollout, self.policy.net
        for t in range(self.nstep):
            with torch.no_grad():
                out, v, _ = net(ro.obs_slots[t])
            self._sample_actions(out, t)
            ro.values[t].copy_(v)
            self.env.step_into(ro.obs_slots[t], ro.obs_slots[t + 1], ro.actions[t], ro.rewards[t], ro.masks[t],
                               ro.done_ret[t], ro.done_len[t])
            if ro.do_hash:                                  # rollout.add -> sim_hash(last_obs), buffer.py:176
                ro.sim_hash(ro.obs_slots[t], ro.rewards[t])
            self.num_timesteps += self.num_envs

    def _collect_step_dc(self, t):
        """Step t of the collect loop with both Philox counters read on the device
        (self._ctr = [sample counter, env step] at the rollout's start)."""
        ro = self.rollout
        # the value straight into the rollout row, the pass's amax table one of the graph's pre-zeroed ones
        out, v, _ = self.policy.net(ro.obs_slots[t], value_out=ro.values[t],
                                    table=self._ctables[t] if self._ctables is not None else None)
        native.categorical_sample_dc(out, self.local_envs, self.n_actions, self.env_offset, self.seed, self._ctr[0:1],
                                     t, ro.actions[t], ro.log_probs[t])
        if v.data_ptr() != ro.values[t].data_ptr():
            ro.values[t].copy_(v)
        self.env.step_into_dc(ro.obs_slots[t], ro.obs_slots[t + 1], ro.actions[t], ro.rewards[t], ro.masks[t],
                              ro.done_ret[t], ro.done_len[t], self._ctr[1:2], t + 1)

    def _collect_graphed(self):
        """ppo.py:174-194 as one hipGraph replay: the first collect runs eagerly (packing the
        weights, warming the library GEMMs) and then captures the nstep steps; every later
        collect refreshes the packed weight forms (train moved the weights), writes the two
        Philox counters to the device and replays — the same launches, counters and results
        as the eager loop (test_collect_graph_matches_eager), without ~20 host launches per step."""
        T, env = self.nstep, self.env
        if self._cgraph is None:
            self._collect_steps_eager()
            self._ctr = torch.zeros(2, dtype=torch.int64, device=self.device)
            # one amax table per step, zeroed by one fill per rollout instead of a fill node per step
            self._ctables = torch.zeros((T, convs.AM_ROWS, native.AMAX_SLOTS), dtype=torch.int32, device=self.device)
            g = torch.cuda.CUDAGraph()
            with torch.no_grad(), torch.cuda.graph(g):
                for t in range(T):
                    self._collect_step_dc(t)
            self._cgraph = g
            return
        self.policy.net.conv_impl.pack(self.local_envs)
        self._ctr[0].fill_(self._sample_counter)
        self._ctr[1].fill_(env.k)
        self._ctables.zero_()
        self._cgraph.replay()
        self._sample_counter += T
        env.k += T
        self.num_timesteps += T * self.num_envs

    @traced("collect")
    def collect_samples(self):
        ro = self.rollout
        self._ensure_started()
        ro.reset()
        if self._collect_graph_ok():
            self._collect_graphed()
        else:
            self._collect_steps_eager()
        ro.pos, ro.full = self.nstep, True
        # ppo.py:196 bootstraps with V(s_{T-1}) and the last step's dones
        ro.compute_returns_and_advantages(ro.values[self.nstep - 1], ro.masks[self.nstep - 1])
        self._finish_episodes()
        self.last_obs = ro.obs_slots[self.nstep]
        return True

    def _minibatch(self, idx, adv_stats, B_global, scale=1.0, extra_backward=None):
        """Forward + fused loss + backward into the flat grad bucket (no step)."""
        ro = self.rollout
        Bl = idx.numel()
        net = self.policy.net
        self._zero_policy_grad(Bl)
        ctx = out = v = None
        if Bl > 0:
            out, v, _, ctx = self._fwd_train(self._train_obs(ro, idx))
            out_d, v_d = out.detach().contiguous(), v.detach().contiguous()
        else:
            out_d, v_d, _ = self._empty_outputs()
        dout, dv, _ = self._loss_grads(out_d, v_d, None, idx, ro.tensors(), adv_stats, B_global, 0.0, scale)
        if extra_backward is None:
            self._bwd_reduce(ctx, out, v, None, dout, dv, has_rows=Bl > 0)
            return
        if Bl > 0:
            self._bwd_train(ctx, out, v, None, dout, dv, extra=extra_backward)
        self.dist.all_reduce_(self.flat.grad)

    @traced("train")
    def train(self):
        with _train_stream(self.device):
            self._train()

    def _train(self):
        ro = self.rollout
        total = self.nstep * self.num_envs
        self.loss_accum.zero_()
        adv, _ = self._global_advantages(ro)
        bs = self._batch(total)
        stats = torch.empty((total + bs - 1) // bs, 4, dtype=torch.float64, device=self.device)
        for _ in range(self.n_epochs):
            perm_dev, local, offs, sizes = self._epoch_minibatches(total)
            native.minibatch_adv_stats(adv, None, perm_dev, total, bs, self.nstep, self.num_envs, stats)
            for k, B in enumerate(sizes):
                idx = local[offs[k]:offs[k + 1]]
                self._minibatch(idx, stats[k], B)
                self.flat.adam_step(self.lr, self.max_grad_norm)
        self._record_train()
        self._n_updates += self.n_epochs

    def learn(self, total_timesteps, log_interval, reward_target=None, log_to_file=False):
        name = "PPO_SimHash" if self.sim_hash else ("PPO_SIL" if self.sil else "PPO")
        return self._learn(name, total_timesteps, log_interval, reward_target, log_to_file)


class PPO_RND(BaseAlgorithm):
    """ppo.py:310-543.  On image envs the RND nets read the normalised LAST frame
    (the checkpoint's RND input, .ipynb_checkpoints/ppo-checkpoint.py:290)."""

    def __init__(self, *, env_id, lr=3e-4, nstep=128, batch_size=128, n_epochs=10, gamma=0.99, int_gamma=0.99,
                 gae_lam=0.95, clip_range=0.2, ent_coef=.01, vf_coef=0.5, int_vf_coef=0.5, max_grad_norm=0.2,
                 hidden_size=128, int_hidden_size=128, int_lr=3e-4, rnd_start=1e+3, n_envs=4, seed=0, device=None,
                 env=None, quiet=False):
        super().__init__(env_id, lr, nstep, batch_size, n_epochs, gamma, gae_lam, clip_range, ent_coef, vf_coef,
                         max_grad_norm, n_envs=n_envs, seed=seed, device=device, env=env, quiet=quiet)
        self.policy = Policy(self.env, hidden_size, intrinsic_model=True)
        self.image = _is_image(self.env.observation_space)
        self.rnd_features = 84 * 84 if self.image else self.state_dim
        self.rnd = RndNetwork(self.rnd_features, hidden_size=int_hidden_size)
        self.rollout = self._new_rollout(IntrinsicStorage, gae_lam=gae_lam, gamma=gamma, int_gamma=int_gamma)
        self.flat = FlatParams(self.policy.net, self.device)
        self._attach_convs()
        self.rnd_flat = FlatParams(self.rnd, self.device)
        self.optimizer, self.rnd_optimizer = self.flat, self.rnd_flat
        self.int_lr, self.rnd_start, self.int_vf_coef = int_lr, rnd_start, int_vf_coef
        self.int_rew_rms = RunningMeanStd(device=self.device)
        self._alloc_train_state()

    def _rnd_input(self, obs):
        """(N, F) view of the features RND sees: last frame (image) or the obs vector (rows of
        _rnd_rows hold the last frame only)."""
        if self.image:
            return obs[:, obs.shape[1] - 1].reshape(obs.shape[0], -1)
        return obs.reshape(obs.shape[0], -1)

    @traced("collect")
    def collect_samples(self):
        ro = self.rollout
        self._ensure_started()
        ro.reset()
        net = self.policy.net
        for t in range(self.nstep):
            with torch.no_grad():
                out, v, iv = net(ro.obs_slots[t])
            self._sample_actions(out, t)
            ro.values[t].copy_(v)
            ro.int_values[t].copy_(iv)
            self.env.step_into(ro.obs_slots[t], ro.obs_slots[t + 1], ro.actions[t], ro.rewards[t], ro.masks[t],
                               ro.done_ret[t], ro.done_len[t])
            self.num_timesteps += self.num_envs
            if (self.num_timesteps / self.num_envs) < self.rnd_start:        # ppo.py:390-392
                ro.int_rewards[t].zero_()
                self._update_obs_rms(self._rnd_input(ro.obs_slots[t]))
            else:                                                              # ppo.py:394-398
                with torch.no_grad():
                    ir = self.rnd.int_reward(self.normalize_obs(self._rnd_input(ro.obs_slots[t + 1])))
                self._scale_int_rewards(ir)
                ro.int_rewards[t].copy_(ir)
        ro.pos, ro.full = self.nstep, True
        T1 = self.nstep - 1
        ro.compute_returns_and_advantages(ro.values[T1], ro.int_values[T1], ro.masks[T1])
        self._finish_episodes()
        return True

    def _rnd_rows(self, ro, idx):
        """The minibatch rows RND trains on: on images only their last frame is gathered (7 KB
        of each 28 KB frame stack; the policy reads its rows in place), else the whole rows."""
        if not self.image:
            return ro._gather(ro.observations, idx)
        obs = ro.observations
        T, N = obs.shape[0], obs.shape[1]
        last = obs[:, :, 3]  # (T, N, 84, 84) view, frame stacks 4 * 7056 bytes apart
        out = torch.empty((idx.numel(), 1) + tuple(last.shape[2:]), dtype=obs.dtype, device=self.device)
        native.gather_rows(last, T, N, last[0, 0].numel() * last.element_size(), obs[0, 0].numel() * obs.element_size(),
                           idx, idx.numel(), out)
        return out

    def _update_obs_rms(self, x):
        if not self.dist.enabled:
            self.obs_rms.update(x)
            return
        # exact across ranks: gather every rank's rows (rank order == env order)
        self.obs_rms.update(self.dist.all_gather_cat(x.contiguous(), dim=0))

    def _scale_int_rewards(self, ir):
        ir = ir.contiguous()
        full = self.dist.all_gather_cat(ir, dim=0) if self.dist.enabled else ir
        native.rms_scale_int_rewards(full, self.int_rew_rms.mean, self.int_rew_rms.var, self.int_rew_rms.count)
        self.int_rew_rms.count = full.numel() + self.int_rew_rms.count
        if self.dist.enabled:
            ir.copy_(full[self.env_offset:self.env_offset + self.local_envs])
        elif full.data_ptr() != ir.data_ptr():
            ir.copy_(full)

    def train_rnd(self, obs, B_global=None):
        """ppo.py:487-502.  MSE(pred, target) over the GLOBAL minibatch: this rank's squared
        errors summed and divided by the global row count B_global, so the all-reduced gradient
        is the reference's mean over all B rows (a per-rank mean would weight ranks' rows
        unequally).  obs None: this rank owns no rows (it still joins the all-reduce)."""
        if obs is None or obs.shape[0] == 0:
            x = torch.zeros(0, self.rnd_features, device=self.device)
        else:
            x = self.normalize_obs(self._rnd_input(obs))
        p, tgt = self.rnd(x)
        n = p.numel() if B_global is None else int(B_global)
        loss = F.mse_loss(p, tgt, reduction="sum") / n
        self.rnd_flat.zero_grad()
        loss.backward()
        self.dist.all_reduce_(self.rnd_flat.grad)
        self.rnd_flat.adam_step(self.int_lr, self.max_grad_norm)

    @traced("train")
    def train(self):
        ro = self.rollout
        total = self.nstep * self.num_envs
        self.loss_accum.zero_()
        adv, iadv = self._global_advantages(ro, intrinsic=True)
        bs = self._batch(total)
        stats = torch.empty((total + bs - 1) // bs, 4, dtype=torch.float64, device=self.device)
        net = self.policy.net
        roll = ro.tensors()
        for _ in range(self.n_epochs):
            perm_dev, local, offs, sizes = self._epoch_minibatches(total)
            native.minibatch_adv_stats(adv, iadv, perm_dev, total, bs, self.nstep, self.num_envs, stats)
            for k, B in enumerate(sizes):
                idx = local[offs[k]:offs[k + 1]]
                Bl = idx.numel()
                self._zero_policy_grad(Bl)
                ctx = out = v = iv = None
                if Bl > 0:
                    out, v, iv, ctx = self._fwd_train(self._train_obs(ro, idx))
                    od, vd, ivd = out.detach().contiguous(), v.detach().contiguous(), iv.detach().contiguous()
                else:  # no rows of this minibatch on this rank: zero contributions, same collectives
                    od, vd, ivd = self._empty_outputs(intrinsic=True)
                dout, dv, div = self._loss_grads(od, vd, ivd, idx, roll, stats[k], B, self.int_vf_coef, 1.0)
                self._bwd_reduce(ctx, out, v, iv, dout, dv, div, has_rows=Bl > 0)
                if np.random.randn() < 0.25:                                   # ppo.py:468-469
                    # (RND's own parameters: beside the policy's Adam step on a side stream in one
                    # process, joined before the next minibatch)
                    side = convs.side_stream(self.device, 1) if convs.BWD_STREAMS and not self.dist.enabled \
                        else None
                    if side is None:
                        self.flat.adam_step(self.lr, self.max_grad_norm)
                        self.train_rnd(self._rnd_rows(ro, idx) if Bl > 0 else None, B)
                    else:
                        convs.fork(side)
                        with torch.cuda.stream(side):
                            self.train_rnd(self._rnd_rows(ro, idx) if Bl > 0 else None, B)
                        self.flat.adam_step(self.lr, self.max_grad_norm)
                        convs.join(side)
                else:
                    self.flat.adam_step(self.lr, self.max_grad_norm)
        acc = self._record_train()
        logger.record("train/intrinsic_loss", acc[4] / max(acc[5], 1.0))
        self._n_updates += self.n_epochs

    def learn(self, total_timesteps, log_interval, reward_target=None, log_to_file=False):
        return self._learn("RND", total_timesteps, log_interval, reward_target, log_to_file)


class PPO_ICM(BaseAlgorithm):
    """ppo.py:546-756.  Quirks kept: beta is fixed at 0.2 (ppo.py:600); the
    rollout uses the default gamma 0.99 (ppo.py:591); ICM pairs are consecutive
    rows of the permuted minibatch (ppo.py:684).  On image envs the ICM MLP reads
    the flattened frame stack (input 4*84*84)."""

    def __init__(self, *, env_id, lr=3e-4, int_lr=3e-4, nstep=128, batch_size=128, n_epochs=10, gamma=0.99,
                 gae_lam=0.95, clip_range=0.2, ent_coef=.01, vf_coef=0.5, max_grad_norm=0.2, hidden_size=128,
                 int_hidden_size=32, int_rew_integration=0.05, beta=0.2, policy_weight=1, n_envs=4, seed=0,
                 device=None, env=None, quiet=False):
        super().__init__(env_id, lr, nstep, batch_size, n_epochs, gamma, gae_lam, clip_range, ent_coef, vf_coef,
                         max_grad_norm, n_envs=n_envs, seed=seed, device=device, env=env, quiet=quiet)
        self.int_rew_integration = int_rew_integration
        self.policy = Policy(self.env, hidden_size)
        self.rollout = self._new_rollout(RolloutStorage, gae_lam=gae_lam)
        icm_in = int(np.prod(self.env.observation_space.shape))
        self.intrinsic_module = IntrinsicCuriosityModule(icm_in, self.action_converter, hidden_size=int_hidden_size)
        self.flat = FlatParams(self.policy.net, self.device)
        self._attach_convs()
        self.icm_flat = FlatParams(self.intrinsic_module, self.device)
        self.optimizer, self.icm_optimizer = self.flat, self.icm_flat
        # image observations: the ICM on libppox kernels (icm.py, csrc/icm.hip); PPOX_ICM_NATIVE=0
        # keeps the torch module (A/B, tests)
        self._icm_native = None
        if os.environ.get("PPOX_ICM_NATIVE", "1") != "0" and icm_native.supported(
                self.intrinsic_module, self.icm_flat, self.env.observation_space.shape, self.rollout.obs_slots.dtype):
            self._icm_native = icm_native.NativeIcm(self.intrinsic_module, self.icm_flat, icm_in)
        self.int_lr = int_lr
        self.policy_weight = policy_weight
        self.beta = 0.2
        self._alloc_train_state()
        self.icm_accum = torch.zeros(1, dtype=torch.float64, device=self.device)
        # At world > 1 the K11 minibatch and its collectives (feature / action / feature-gradient
        # exchange, the ICM gradient all-reduce) run on the main stream after the policy's, in
        # program order on one communicator.  PPOX_ICM_SIDE_DIST=1 (opt-in, never run on more than
        # one GPU) runs them on the side stream beside the policy minibatch as in one process, on a
        # communicator of their own (DistContext.subgroup): two communicators' collectives then
        # run concurrently, which RCCL guarantees to progress only when both fit on the GPU at once.
        self._icm_side_dist = native.ab_env("PPOX_ICM_SIDE_DIST", "0") == "1"
        self._icm_dist = (self.dist.subgroup() if self.dist.enabled and self._icm_native is not None
                          and self._icm_side_dist else self.dist)
        # the collect loop (policy + env + K11 curiosity reward) as one captured graph, as PPO's
        # (PPOX_COLLECT_GRAPH=0: eager launches)
        self._collect_graph_enabled = native.ab_env("PPOX_COLLECT_GRAPH", "1") != "0"
        self._cgraph = None
        self._ctables = None
        self._ir_sum = torch.zeros((), dtype=torch.float64, device=self.device)

    def _collect_graph_ok(self):
        return (self._collect_graph_enabled and self._icm_native is not None and isinstance(self.env, DeviceAtariEnv)
                and self.discrete and getattr(self.policy.net, "conv_impl", None) is not None
                and self.device.type == "cuda")

    def _icm_collect_step_dc(self, t, nat, eta):
        """Step t of the collect loop with device-resident Philox counters (as PPO._collect_step_dc)
        plus the K11 curiosity reward; phi(s_t) is in tag c0 / c1 by the parity of t."""
        ro = self.rollout
        # the value straight into the rollout row, the pass's amax table one of the graph's pre-zeroed ones
        out, v, _ = self.policy.net(ro.obs_slots[t], value_out=ro.values[t],
                                    table=self._ctables[t] if self._ctables is not None else None)
        native.categorical_sample_dc(out, self.local_envs, self.n_actions, self.env_offset, self.seed, self._ctr[0:1],
                                     t, ro.actions[t], ro.log_probs[t])
        if v.data_ptr() != ro.values[t].data_ptr():
            ro.values[t].copy_(v)
        self.env.step_into_dc(ro.obs_slots[t], ro.obs_slots[t + 1], ro.actions[t], ro.rewards[t], ro.masks[t],
                              ro.done_ret[t], ro.done_len[t], self._ctr[1:2], t + 1)
        if t == 0:
            nat.encode(ro.obs_slots[0], "c0")
        f = nat._buf("c0_phi" if t % 2 == 0 else "c1_phi", (self.local_envs, icm_native.H))
        f_next = nat.encode(ro.obs_slots[t + 1], "c1" if t % 2 == 0 else "c0")[1]
        ir = nat._buf("ir", (self.local_envs,))
        nat.int_reward(f, f_next, ro.actions[t], ro.rewards[t], eta, ir)
        self._ir_sum += ir.double().mean()

    def _icm_x(self, obs):
        x = obs.reshape(obs.shape[0], int(np.prod(obs.shape[1:])))
        if x.dtype == torch.uint8 and x.is_cuda and x.is_contiguous() and x.numel() % 16 == 0:
            return native.u8_to_f32(x)
        return x.float()

    @traced("collect")
    def collect_samples(self):
        ro = self.rollout
        self._ensure_started()
        ro.reset()
        if self._collect_graph_ok() and self._cgraph is not None:
            # replay: refresh the packed weight forms (train moved the weights), the counters
            T, env = self.nstep, self.env
            self.policy.net.conv_impl.pack(self.local_envs)
            self._icm_native.pack()
            self._ctr[0].fill_(self._sample_counter)
            self._ctr[1].fill_(env.k)
            self._ir_sum.zero_()
            self._ctables.zero_()
            self._cgraph.replay()
            self._sample_counter += T
            env.k += T
            self.num_timesteps += T * self.num_envs
        else:
            self._collect_eager()
            if self._collect_graph_ok():  # capture after the first (eager) rollout
                self._ctr = torch.zeros(2, dtype=torch.int64, device=self.device)
                self._ctables = torch.zeros((self.nstep, convs.AM_ROWS, native.AMAX_SLOTS), dtype=torch.int32,
                                            device=self.device)
                g = torch.cuda.CUDAGraph()
                nat, eta = self._icm_native, self.int_rew_integration
                with torch.no_grad(), torch.cuda.graph(g):
                    for t in range(self.nstep):
                        self._icm_collect_step_dc(t, nat, eta)
                self._cgraph = g
        logger.record("rollout/mean_int_reward", float(self._ir_sum.item()) / self.nstep)
        ro.pos, ro.full = self.nstep, True
        ro.compute_returns_and_advantages(ro.values[self.nstep - 1], ro.masks[self.nstep - 1])
        self._finish_episodes()
        return True

    def _collect_eager(self):
        ro = self.rollout
        net = self.policy.net
        ir_sum = self._ir_sum
        ir_sum.zero_()
        eta = self.int_rew_integration
        icm = self.intrinsic_module
        f_next = None  # phi(s_{t+1}) of the previous step = phi(s_t) of this one (same rows, same math)
        nat = self._icm_native
        for t in range(self.nstep):
            with torch.no_grad():
                out, v, _ = net(ro.obs_slots[t])
            self._sample_actions(out, t)
            ro.values[t].copy_(v)
            self.env.step_into(ro.obs_slots[t], ro.obs_slots[t + 1], ro.actions[t], ro.rewards[t], ro.masks[t],
                               ro.done_ret[t], ro.done_len[t])
            self.num_timesteps += self.num_envs
            if nat is not None:  # ppo.py:629-631 on K11: encoder + forward model + reward mix, 3 launches
                if f_next is None:
                    f_next = nat.encode(ro.obs_slots[t], "c0")[1]
                f = f_next
                f_next = nat.encode(ro.obs_slots[t + 1], "c1" if t % 2 == 0 else "c0")[1]
                ir = nat._buf("ir", (self.local_envs,))
                nat.int_reward(f, f_next, ro.actions[t], ro.rewards[t], eta, ir)
                ir_sum += ir.double().mean()
                continue
            with torch.no_grad():                                              # ppo.py:629-630
                f = icm.state_encoder(self._icm_x(ro.obs_slots[t])) if f_next is None else f_next
                f_next = icm.state_encoder(self._icm_x(ro.obs_slots[t + 1]))
                ir = icm.int_reward_features(f, f_next, ro.actions[t])
            ro.rewards[t].copy_((1 - eta) * ro.rewards[t] + eta * ir)
            ir_sum += ir.double().mean()

    @traced("train")
    def train(self):
        ro = self.rollout
        total = self.nstep * self.num_envs
        self.loss_accum.zero_()
        self.icm_accum.zero_()
        adv, _ = self._global_advantages(ro)
        bs = self._batch(total)
        stats = torch.empty((total + bs - 1) // bs, 4, dtype=torch.float64, device=self.device)
        net, icm = self.policy.net, self.intrinsic_module
        roll = ro.tensors()
        for _ in range(self.n_epochs):
            perm_dev, local, offs, sizes = self._epoch_minibatches(total)
            native.minibatch_adv_stats(adv, None, perm_dev, total, bs, self.nstep, self.num_envs, stats)
            for k, B in enumerate(sizes):
                idx = local[offs[k]:offs[k + 1]]
                Bl = idx.numel()
                if self._icm_native is not None:
                    self._minibatch_native_icm(idx, stats[k], B, roll, offs[k], offs[k + 1])
                    continue
                self._zero_policy_grad(Bl)
                self.icm_flat.zero_grad()
                obs = ro._gather(ro.observations, idx)
                ctx = out = v = None
                if Bl > 0:
                    out, v, _, ctx = self._fwd_train(obs)
                    od, vd = out.detach().contiguous(), v.detach().contiguous()
                else:  # no rows of this minibatch on this rank: zero contributions, same collectives
                    od, vd, _ = self._empty_outputs()
                dout, dv, _ = self._loss_grads(od, vd, None, idx, roll, stats[k], B, 0.0, float(self.policy_weight))
                # ICM on consecutive rows of the (owned part of the) permuted minibatch (ppo.py:684-688)
                rows = (idx % self.nstep) * self.local_envs + idx // self.nstep
                if self.discrete:
                    acts = ro.actions.reshape(-1)[rows]
                else:
                    acts = ro.actions.reshape(-1, self.n_actions)[rows]
                x = self._icm_x(obs)
                if Bl > 0:
                    self._bwd_train(ctx, out, v, None, dout, dv)
                # pairs (row j, row j+1) of the permuted minibatch; each row is encoded once
                # (the reference encodes s and s' separately: same rows, same math) and at
                # world > 1 the pairs cross rank boundaries (icm_loss_sharded)
                pos = self._epoch_pos[offs[k]:offs[k + 1]] if self.dist.enabled else \
                    torch.arange(Bl, device=self.device)
                self.icm_accum += icm_loss_sharded(icm, x, acts, pos, B, self.beta, self.dist).double()
                self.dist.all_reduce_(self.flat.grad)
                self.dist.all_reduce_(self.icm_flat.grad)
                self.flat.adam_step(self.lr, self.max_grad_norm)               # ppo.py:697-698
                self.icm_flat.adam_step(self.int_lr, None)                     # ppo.py:699 (no clipping)
        icm_mean = float(self.dist.all_reduce_(self.icm_accum).item())
        acc = self._record_train(extra=icm_mean)
        logger.record("train/icm_loss", icm_mean / max(acc[5], 1.0))
        self._n_updates += self.n_epochs

    def _minibatch_native_icm(self, idx, adv_stats, B, roll, o0, o1):
        """One minibatch with the ICM on K11 kernels: the policy as PPO's minibatch (rollout rows
        read in place, overlapped gradient all-reduce), then the ICM loss of the same rows
        (ppo.py:684-688) straight off the rollout frames, its all-reduce and both Adam steps."""
        ro = self.rollout
        Bl = idx.numel()
        # the ICM (independent of the policy: its own parameters, the same frames) runs on a
        # side stream beside the policy's forward / loss / backward in one process; at world > 1
        # only with PPOX_ICM_SIDE_DIST=1 (its collectives then on their own communicator,
        # self._icm_dist, issued in the same program order on every rank), else after the policy
        side = (convs.side_stream(self.device, 1)
                if convs.BWD_STREAMS and (not self.dist.enabled or self._icm_side_dist) else None)
        pos = self._epoch_pos[o0:o1] if self.dist.enabled else None
        idist = self._icm_dist
        if side is not None:
            convs.fork(side)
            with torch.cuda.stream(side):
                self._icm_native.train_minibatch(convs.RolloutRows(ro.observations, idx), ro.actions, pos, B,
                                                 self.beta, idist, self.icm_accum)
                idist.all_reduce_(self.icm_flat.grad)
        self._zero_policy_grad(Bl)
        ctx = out = v = None
        if Bl > 0:
            out, v, _, ctx = self._fwd_train(self._train_obs(ro, idx))
            od, vd = out.detach().contiguous(), v.detach().contiguous()
        else:
            od, vd, _ = self._empty_outputs()
        dout, dv, _ = self._loss_grads(od, vd, None, idx, roll, adv_stats, B, 0.0, float(self.policy_weight))
        self._bwd_reduce(ctx, out, v, None, dout, dv, has_rows=Bl > 0)
        if side is None:
            self._icm_native.train_minibatch(convs.RolloutRows(ro.observations, idx), ro.actions, pos, B,
                                             self.beta, idist, self.icm_accum)
            idist.all_reduce_(self.icm_flat.grad)
        else:
            convs.join(side)
        self.flat.adam_step(self.lr, self.max_grad_norm)                       # ppo.py:697-698
        self.icm_flat.adam_step(self.int_lr, None)                             # ppo.py:699 (no clipping)

    def learn(self, total_timesteps, log_interval=5, reward_target=None, log_to_file=False):
        return self._learn("ICM", total_timesteps, log_interval, reward_target, log_to_file, progress=True)
