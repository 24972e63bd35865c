"""Data-parallel context: one process per GPU, envs sharded by index.

The reference is single-process (no DP).  Here rank g owns envs
[g*N/G, (g+1)*N/G).  The update stays EXACTLY the single-GPU update: every rank
draws the same global numpy permutation (same seed), processes the rows of each
global minibatch it owns, and the only per-minibatch exchanges are a 4 KB
all-reduce of the loss partial sums (global advantage moments are all-gathered
once per rollout) and the all-reduce of the flat gradient bucket.  On ROCm the
torch "nccl" backend is RCCL over xGMI; CPU tests use "gloo".
"""
import atexit
import os
import warnings

import numpy as np
import torch
import torch.distributed as tdist


# the per-minibatch all-reduces through native code (csrc/dp.cpp) instead of torch.distributed
NATIVE_DP = os.environ.get("PPOX_NATIVE_DP", "1") != "0"
_dp_comm = None
_native_off = False  # set once the RCCL library could not be found (torch's collectives then)


def shutdown():
    """Destroy the process's native RCCL communicator (a stream sync, then ncclCommDestroy).  Call before
    torch.distributed.destroy_process_group(); also registered with atexit when the communicator is made, so
    it never lives into the exit-time destructors (a profiled run left it alive and died with SIGSEGV in
    __cxa_finalize).  Returns the destroy's status (0, or None when there was none)."""
    global _dp_comm
    comm, _dp_comm = _dp_comm, None
    return comm.close() if comm is not None else None


def _self_check(comm, device, world, rank):
    """At creation: the communicator sums across every rank.  Integer-valued floats (exact sums) through the
    blocking and the asynchronous form, checked against the closed-form totals and against torch's own
    collective over the same ranks; a mismatch raises — there is no silent fallback."""
    i = torch.arange(4099, device=device, dtype=torch.float32)
    x = (i.remainder(7) + 1) * (rank + 1)
    y = torch.full((17,), float(rank + 1), dtype=torch.float64, device=device)
    ones = torch.ones(1024, device=device)
    comm.all_reduce_(x)
    comm.all_reduce_(y, wait=False)
    comm.wait()
    comm.all_reduce_(ones)
    tri = world * (world + 1) / 2
    ref = (i.remainder(7) + 1) * (rank + 1)
    tdist.all_reduce(ref)
    ok = (torch.equal(x, (i.remainder(7) + 1) * tri) and torch.equal(x, ref) and bool((y == tri).all())
          and bool((ones == world).all()))
    if not ok:
        raise RuntimeError(f"native RCCL communicator self-check failed on rank {rank} of {world}: the all-reduce "
                           "does not sum across the ranks")


class _NativeWork:
    def __init__(self, comm):
        self.comm = comm

    def wait(self):
        self.comm.wait()


class DistContext:
    def __init__(self, rank=0, world=1, group=None):
        self.rank, self.world, self.group = rank, world, group

    @property
    def enabled(self):
        return self.world > 1

    @classmethod
    def current(cls):
        if tdist.is_available() and tdist.is_initialized():
            return cls(tdist.get_rank(), tdist.get_world_size())
        return cls()

    def ranks_on_device(self, device):
        """How many ranks of this context drive the same GPU as this one (host name, visible-device lists and
        device index compared over an all_gather: a collective, every rank calls it in the same order).  1 in
        the deployed layout (one process per GPU); more when the ranks of a test share one device."""
        if not self.enabled:
            return 1
        import socket
        key = "|".join([socket.gethostname()] + [os.environ.get(v, "") for v in
                                                  ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES",
                                                   "CUDA_VISIBLE_DEVICES")] + [str(device.index)])
        keys = [None] * self.world
        tdist.all_gather_object(keys, key, group=self.group)
        return keys.count(key)

    def subgroup(self):
        """A context over the same ranks on a communicator of its own (a collective call: every rank
        makes it, in the same order).  Its collectives are ordered only among themselves, so they
        can run on a side stream beside this context's (PPO_ICM's curiosity-module exchange beside
        the policy's loss and gradient all-reduces) without queueing behind them."""
        if not (tdist.is_available() and tdist.is_initialized()):
            return self
        return DistContext(self.rank, self.world, group=tdist.new_group(ranks=list(range(self.world))))

    def _native(self, t):
        """The process's native RCCL communicator (native.DpComm) when `t` can go through it: the default
        group on the RCCL backend, a float32 / float64 device tensor (PPOX_NATIVE_DP=0: torch's collectives
        throughout).  A subgroup() context (PPO_ICM's opt-in side-stream exchange) stays on torch's
        collectives: on a native communicator of its own, beside the default group's, the dp-forced PPO_ICM
        iteration ran 544 ms against 243 (profiles/r05g).  Created on first use: a collective call, made by
        every rank at its first such all-reduce, in the same order."""
        global _dp_comm, _native_off
        if (self.group is not None or not NATIVE_DP or _native_off or not t.is_cuda
                or t.dtype not in (torch.float32, torch.float64) or not t.is_contiguous()):
            return None
        comm = _dp_comm
        if comm is None:
            if tdist.get_backend() != "nccl":
                return None
            import native
            try:
                path = native.rccl_path()
            except ImportError as e:  # a torch build on the system RCCL: torch's collectives throughout
                warnings.warn(f"native RCCL exchange off ({e}); using torch.distributed's collectives")
                _native_off = True
                return None

            def bcast(b):
                buf = torch.tensor(list(b), dtype=torch.uint8, device=t.device)
                tdist.broadcast(buf, 0)
                return bytes(buf.cpu().numpy())
            comm = native.DpComm(tdist.get_world_size(), tdist.get_rank(), t.device.index, bcast, rccl=path)
            _dp_comm = comm
            atexit.register(shutdown)
            _self_check(comm, t.device, comm.world, comm.rank)
        return comm

    def all_reduce_(self, t):
        if self.enabled:
            comm = self._native(t)
            if comm is not None:
                return comm.all_reduce_(t)
            tdist.all_reduce(t, op=tdist.ReduceOp.SUM, group=self.group)
        return t

    def all_reduce_async_(self, t):
        """Start a SUM all-reduce of `t` ordered after the work already on the current
        stream; returns the work handle (None at world 1).  Call .wait() before reading t:
        the then-current stream waits for it."""
        if self.enabled:
            comm = self._native(t)
            if comm is not None:
                comm.all_reduce_(t, wait=False)
                return _NativeWork(comm)
            return tdist.all_reduce(t, op=tdist.ReduceOp.SUM, group=self.group, async_op=True)
        return None

    def all_gather_cat(self, t, dim):
        """Concatenate every rank's `t` along `dim` in rank order."""
        if not self.enabled:
            return t
        parts = [torch.empty_like(t) for _ in range(self.world)]
        tdist.all_gather(parts, t.contiguous(), group=self.group)
        return torch.cat(parts, dim=dim)

    def all_gather_rows(self, t, counts):
        """Concatenate every rank's rows in rank order when rank r holds counts[r] of them (ragged
        shards: all_gather needs equal sizes, so each rank sends max(counts) rows, zero-padded)."""
        if not self.enabled:
            return t
        m = max(counts)
        if t.shape[0] != counts[self.rank]:
            raise ValueError(f"rank {self.rank} holds {t.shape[0]} rows, counts says {counts[self.rank]}")
        pad = t.new_zeros((m,) + tuple(t.shape[1:]))
        pad[:t.shape[0]] = t
        parts = [torch.empty_like(pad) for _ in range(self.world)]
        tdist.all_gather(parts, pad, group=self.group)
        return torch.cat([p[:c] for p, c in zip(parts, counts)], dim=0)

    def barrier(self):
        if self.enabled:
            tdist.barrier(group=self.group)


def init_from_env(backend=None):
    """Initialise the default process group from torchrun's env vars (no-op at world 1)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1 or tdist.is_initialized():
        return DistContext.current()
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    tdist.init_process_group(backend=backend)
    return DistContext.current()


def shard_range(n_envs, rank, world):
    if n_envs % world:
        raise ValueError(f"n_envs={n_envs} must be divisible by world size {world}")
    per = n_envs // world
    return rank * per, per


def owned_minibatch_indices(perm, T, env_lo, n_local, batch_size):
    """Split the GLOBAL env-major permutation into per-minibatch LOCAL indices.

    perm holds flat indices i = n*T + t over all envs; this rank owns envs
    [env_lo, env_lo + n_local).  Returns (local_flat_indices int64, offsets) where
    minibatch k's owned rows are local[offsets[k]:offsets[k+1]], in permutation
    order, re-based to the local flat index (n - env_lo)*T + t.
    """
    perm = np.asarray(perm, dtype=np.int64)
    total = perm.shape[0]
    env = perm // T
    own = (env >= env_lo) & (env < env_lo + n_local)
    local = perm[own] - env_lo * T
    mb_of = (np.nonzero(own)[0] // batch_size)
    n_mb = (total + batch_size - 1) // batch_size
    counts = np.bincount(mb_of, minlength=n_mb)
    offsets = np.concatenate([[0], np.cumsum(counts)])
    return local, offsets


def owned_minibatch_positions(perm, T, env_lo, n_local, batch_size):
    """Positions inside their global minibatch (0..B-1) of the rows owned_minibatch_indices
    returns, in the same order."""
    perm = np.asarray(perm, dtype=np.int64)
    env = perm // T
    own = np.nonzero((env >= env_lo) & (env < env_lo + n_local))[0]
    return own - (own // batch_size) * batch_size
