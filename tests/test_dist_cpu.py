"""Data-parallel decomposition on CPU (gloo, world size 2): the sharded update must
equal the single-process update.  No GPU needed."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as tdist
import torch.multiprocessing as mp

from dist import DistContext, owned_minibatch_indices, shard_range
from oracle import algos as OA


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,T,N,B", [(2, 8, 6, 10), (4, 16, 8, 32), (3, 5, 9, 7), (8, 128, 64, 1000)])
def test_owned_indices_partition_the_global_minibatches(world, T, N, B):
    rs = np.random.RandomState(world * 100 + T)
    perm = rs.permutation(T * N)
    n_mb = -(-T * N // B)
    per_rank = []
    for r in range(world):
        lo, n_local = shard_range(N, r, world)
        local, offs = owned_minibatch_indices(perm, T, lo, n_local, B)
        assert len(offs) == n_mb + 1
        per_rank.append((lo, local, offs))
    for k in range(n_mb):
        glob = perm[k * B:(k + 1) * B]
        got = []
        for lo, local, offs in per_rank:
            rows = local[offs[k]:offs[k + 1]] + lo * T
            # rows of a rank keep the permutation order
            pos = [int(np.nonzero(glob == x)[0][0]) for x in rows]
            assert pos == sorted(pos)
            got.extend(rows.tolist())
        assert sorted(got) == sorted(glob.tolist())


def test_shard_range_rejects_ragged():
    with pytest.raises(ValueError):
        shard_range(10, 0, 3)


# --- the per-rank loss decomposition, restated on torch-CPU ------------------
def _rank_step(rows, logits_fn, roll, stats, clip, ent_coef, vf_coef, B_glob, ctx):
    """What one rank does per minibatch: forward on its rows, loss partial sums,
    all-reduce, then gradients scaled by the GLOBAL minibatch size."""
    z, v = logits_fn(rows)
    mean, std = stats
    adv = (torch.tensor(roll["adv"][rows]) - mean) / (std + 1e-8)
    d = torch.distributions.Categorical(torch.softmax(z, -1))
    lp = d.log_prob(torch.tensor(roll["act"][rows]).double())
    ratio = torch.exp(lp - torch.tensor(roll["lp"][rows]))
    surr = torch.min(adv * ratio, adv * torch.clamp(ratio, 1 - clip, 1 + clip))
    ret = torch.tensor(roll["ret"][rows])
    ov = torch.tensor(roll["v"][rows])
    vc = ov + (v - ov).clamp(-clip, clip)
    e1, e2 = ((ret - v) ** 2), ((ret - vc) ** 2)
    part = torch.stack([e1.sum(), e2.sum()]).detach().double()
    ctx.all_reduce_(part)
    vl1, vl2 = float(part[0] / B_glob), float(part[1] / B_glob)
    wA = 0.5 if vl1 == vl2 else float(vl1 > vl2)
    wB = 0.5 if vl1 == vl2 else float(vl2 > vl1)
    loss = (-surr.sum() + vf_coef * (wA * e1.sum() + wB * e2.sum()) - ent_coef * d.entropy().sum()) / B_glob
    return loss


def _worker(rank, world, port, out_q, seed):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = DistContext.current()
    T, N, A, B = 8, 8, 3, 24
    lo, n_local = shard_range(N, rank, world)
    rs = np.random.RandomState(seed)
    roll = {"act": rs.randint(0, A, T * N), "lp": np.log(rs.dirichlet(np.ones(A), T * N).max(-1)).astype(np.float32),
            "adv": rs.randn(T * N).astype(np.float32), "ret": rs.randn(T * N).astype(np.float32),
            "v": rs.randn(T * N).astype(np.float32), "obs": rs.randn(T * N, 5).astype(np.float32)}
    torch.manual_seed(seed)
    net = torch.nn.Linear(5, A + 1)
    perm = rs.permutation(T * N)
    local, offs = owned_minibatch_indices(perm, T, lo, n_local, B)
    # all_gather_cat: rank order == env order
    g = ctx.all_gather_cat(torch.arange(n_local, dtype=torch.float32) + lo, dim=0)
    assert torch.equal(g, torch.arange(N, dtype=torch.float32))
    grads = []
    for k in range(len(offs) - 1):
        gl = perm[k * B:(k + 1) * B]
        a = torch.tensor(roll["adv"][gl]).double()
        stats = (float(a.mean()), float(a.std()))
        rows = local[offs[k]:offs[k + 1]] + lo * T
        net.zero_grad()

        def fwd(r):
            o = net(torch.tensor(roll["obs"][r]))
            return o[:, :A], o[:, A]
        loss = _rank_step(rows, fwd, roll, stats, 0.2, 0.01, 0.5, len(gl), ctx)
        loss.backward()
        flat = torch.cat([p.grad.reshape(-1) for p in net.parameters()])
        ctx.all_reduce_(flat)
        grads.append(flat.numpy().copy())
    # ranks sharing a GPU (the backward's side stream is dropped then: DESIGN.md §5): same index -> both, own -> 1
    shared = (ctx.ranks_on_device(torch.device("cuda", 0)), ctx.ranks_on_device(torch.device("cuda", rank)))
    out_q.put((rank, (grads, shared)))
    tdist.destroy_process_group()


def test_two_rank_gradients_equal_single_process():
    world, seed = 2, 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, seed)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] == (world, 1) for r in res.values()), {k: r[1] for k, r in res.items()}
    res = {k: r[0] for k, r in res.items()}
    # single process reference: full global minibatches
    T, N, A, B = 8, 8, 3, 24
    rs = np.random.RandomState(seed)
    roll = {"act": rs.randint(0, A, T * N), "lp": np.log(rs.dirichlet(np.ones(A), T * N).max(-1)).astype(np.float32),
            "adv": rs.randn(T * N).astype(np.float32), "ret": rs.randn(T * N).astype(np.float32),
            "v": rs.randn(T * N).astype(np.float32), "obs": rs.randn(T * N, 5).astype(np.float32)}
    torch.manual_seed(seed)
    net = torch.nn.Linear(5, A + 1)
    perm = rs.permutation(T * N)
    for k in range(-(-T * N // B)):
        gl = perm[k * B:(k + 1) * B]
        net.zero_grad()
        o = net(torch.tensor(roll["obs"][gl]))
        z, v = o[:, :A], o[:, A]
        d = torch.distributions.Categorical(torch.softmax(z, -1))
        lp = d.log_prob(torch.tensor(roll["act"][gl]).double())
        mb = {"advantages": torch.tensor(roll["adv"][gl]), "old_log_probs": torch.tensor(roll["lp"][gl]),
              "returns": torch.tensor(roll["ret"][gl]), "old_values": torch.tensor(roll["v"][gl])}
        loss, *_ = OA.ppo_loss(v, lp, d.entropy(), mb, 0.2, 0.01, 0.5)
        loss.backward()
        ref = torch.cat([p.grad.reshape(-1) for p in net.parameters()]).numpy()
        for r in range(world):
            np.testing.assert_allclose(res[r][k], ref, rtol=2e-5, atol=1e-7)


def _icm_worker(rank, world, port, out_q, discrete, seed):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ppo import icm_loss_sharded
        icm, x, a, owner = _icm_case(discrete, seed)
        mine = np.nonzero(owner == rank)[0]  # positions this rank owns, in minibatch order
        pos = torch.from_numpy(mine)
        loss = icm_loss_sharded(icm, x[pos], a[pos], pos, x.shape[0], 0.2, DistContext.current())
        g = torch.cat([p.grad.reshape(-1) for p in icm.parameters()])
        tdist.all_reduce(g)
        out_q.put((rank, float(loss), g.numpy()))
    finally:
        tdist.destroy_process_group()


def _icm_case(discrete, seed):
    from models import IntrinsicCuriosityModule
    from util import ActionConverter
    import env as E
    torch.manual_seed(seed)
    rs = np.random.RandomState(seed)
    B, F_, A = 23, 10, 3
    space = E.Discrete(A) if discrete else E.Box((A,))
    icm = IntrinsicCuriosityModule(F_, ActionConverter(space), hidden_size=8)
    x = torch.tensor(rs.randn(B, F_).astype(np.float32))
    a = torch.tensor(rs.randint(0, A, B)) if discrete else torch.tensor(rs.randn(B, A).astype(np.float32))
    owner = rs.randint(0, 2, B)  # a random, interleaved row ownership
    return icm, x, a, owner


@pytest.mark.parametrize("discrete", [True, False])
def test_icm_sharded_pairs_equal_single_process(discrete):
    """PPO_ICM pairs (row j, row j+1) of the permuted minibatch (ppo.py:684-692) across two
    ranks with interleaved row ownership == the one-process loss and gradients."""
    import torch.nn.functional as F
    seed = 17
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_icm_worker, args=(r, 2, port, q, discrete, seed)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (l, g)) for r, l, g in (q.get(timeout=120) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
    icm, x, a, _ = _icm_case(discrete, seed)
    a_hat, nf, nfh = icm(x[:-1], x[1:], a[:-1])
    inv = F.cross_entropy(a_hat, a[:-1].long()) if discrete else F.mse_loss(a_hat, a[:-1])
    loss = 0.8 * inv + 0.2 * F.mse_loss(nf, nfh)
    loss.backward()
    ref = torch.cat([p.grad.reshape(-1) for p in icm.parameters()]).numpy()
    np.testing.assert_allclose(res[0][0] + res[1][0], loss.item(), rtol=1e-5)
    for r in range(2):
        np.testing.assert_allclose(res[r][1], ref, rtol=1e-4, atol=1e-6)
