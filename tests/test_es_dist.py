"""ES-NSRA sharded generation (BASELINE config 5, evolution_strategies.py:184-199, 217-239,
299-385): members sharded by index over ranks, fitness all-gathered in member order, the
update's partial P^T c all-reduced.  W ranks over gloo must reproduce one process: the
first generation's fitness vector bitwise (later ones to 1e-10: the update's sum is split at the
shard boundaries, so the weights differ by ~1e-16), the same novelty schedule and brain choices,
and the weights within 1e-12.

CPU (world 2 / 4, no GPU): the class's host logic with the device kernels stood in for by their
oracle restatements (oracle/es.py: the same Philox perturbations, episodes and P^T c) — the
collectives, the ragged shard bookkeeping and the host RNG are what is under test here.
GPU (world 2, gloo, both ranks on cuda:0; RCCL cannot put two ranks on one device): the product
kernels at P = 10,000, the C5 population."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_device(native):
    """Replace the ES entry points of `native` by CPU restatements (oracle/es.py) on CPU tensors."""
    from oracle import es as O

    def split(flat, sizes):
        out, off = [], 0
        for a, b in zip(sizes[:-1], sizes[1:]):
            out.append(flat[off:off + a * b].reshape(a, b))
            off += a * b
        return out

    def es_evaluate(w, eps, sigma, P, D, H1, H2, A, T, env_seed, xi, fit, bc=None, stream=None):
        wn, sizes = w.numpy(), [D, H1, H2, A]
        flats = [wn + sigma * eps[p].numpy() for p in range(P)] if eps is not None else [wn]
        f, b = O.evaluate([split(x, sizes) for x in flats], env_seed, T)
        fit.copy_(torch.from_numpy(f))
        if bc is not None:
            bc.copy_(torch.from_numpy(b))

    native.lib = lambda: None
    native.es_env_noise = lambda T, D, env_seed, xi, stream=None: xi.zero_()
    native.es_noise = lambda P, n, m0, gen, seed, eps, stream=None: eps.copy_(
        torch.from_numpy(O.perturbations(seed, gen, np.arange(m0, m0 + P), n)))
    native.es_evaluate = es_evaluate
    native.es_update_workspace_bytes = lambda P, n: 8
    native.es_update = lambda eps, coef, P, n, ws, out, stream=None: out.copy_(
        torch.from_numpy(coef.numpy() @ eps.numpy()))


def _run_es(P, hidden, T, gens, device):
    """One ES run; returns (fitness per generation, (brain, novelty, novelty_param) per generation,
    final weights)."""
    import evolution_strategies as ES
    np.random.seed(5)
    es = ES.EvolutionStrategy("Swimmer-v3", hidden_sizes=list(hidden), population_size=P, sigma=0.1,
                              learning_rate=0.02, seed=9, episode_len=T, device=device)
    fits, sched = [], []
    get_rewards, update = es._get_rewards, es._update_weights

    def rec_rewards(pool, population):
        r = get_rewards(pool, population)
        fits.append(r.copy())
        return r

    def rec_update(rewards, population, novelty=None):
        sched.append((novelty, float(es.novelty_param)))
        return update(rewards, population, novelty)
    es._get_rewards, es._update_weights = rec_rewards, rec_update
    es.run(gens, log_interval=10 ** 9)
    return np.stack(fits), sched, [w.copy() for w in es.weights], float(es.novelty_param)


def _rank(rank, world, port, q, P, hidden, T, gens, cpu):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "ppo-exploration_amd"))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as tdist
    if not cpu:
        torch.cuda.set_device(0)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import native
        if cpu:
            _oracle_device(native)
        q.put((rank, _run_es(P, hidden, T, gens, "cpu" if cpu else "cuda")))
    except Exception as e:  # surface the failure to the parent
        import traceback
        q.put((rank, traceback.format_exc() + repr(e)))
    finally:
        tdist.destroy_process_group()


def _compare(world, P, hidden, T, gens, cpu):
    if cpu:
        import native
        saved = {k: getattr(native, k) for k in ("lib", "es_env_noise", "es_noise", "es_evaluate",
                                                  "es_update_workspace_bytes", "es_update")}
        _oracle_device(native)
        try:
            one = _run_es(P, hidden, T, gens, "cpu")
        finally:
            for k, v in saved.items():
                setattr(native, k, v)
    else:
        one = _run_es(P, hidden, T, gens, "cuda")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q, P, hidden, T, gens, cpu)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=600) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    f1, s1, w1, nu1 = one
    for r in range(world):
        got = res[r]
        if isinstance(got, str):
            raise AssertionError(f"rank {r}: {got}")
        f, s, w, nu = got
        # generation 0 evaluates the same weights everywhere: its fitness vector (all-gathered in member
        # order) is bitwise the one process's; from then the weights differ by the update's split sum
        # (~1e-16), so later fitness agrees to that
        assert np.array_equal(f[0], f1[0]), f"rank {r}: generation-0 fitness differs"
        np.testing.assert_allclose(f, f1, rtol=1e-10, atol=1e-10 * np.abs(f1).max())
        assert [x[1] for x in s] == [x[1] for x in s1] and nu == nu1, f"rank {r}: novelty schedule differs"
        np.testing.assert_allclose([x[0] for x in s], [x[0] for x in s1], rtol=1e-10)  # the chosen brain's novelty
        for a, b in zip(w, w1):
            np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-12 * np.abs(b).max())


@pytest.mark.parametrize("world,P", [(2, 24), (4, 24), (2, 23), (4, 30)])
def test_es_sharded_generation_equals_one_process_cpu(world, P):
    """P % world != 0 (23 over 2, 30 over 4): ragged shards, the padded all-gather."""
    _compare(world, P, (8, 6), 12, 4, cpu=True)


@pytest.mark.gpu
def test_es_sharded_generation_equals_one_process_gpu():
    """The product kernels (ppox_es_noise / _evaluate / _update) at the C5 population P = 10,000
    (Swimmer shape, 64 x 64 policy), two ranks of 5,000 members on one GPU."""
    _compare(2, 10000, (64, 64), 200, 3, cpu=False)
