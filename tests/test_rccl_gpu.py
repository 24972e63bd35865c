"""RCCL (torch's "nccl" backend on ROCm) on a one-rank communicator, with the data-parallel code
paths forced on: owned-row minibatches, the loss-partials all-reduce, the two-piece gradient
all-reduce started asynchronously from the backward's side stream, all_gather_cat of the
rollout statistics, PPO_ICM's feature / action / feature-gradient exchange (float32 and int32
all-reduces) and PPO_RND's gathered obs_rms.  The update must equal the single-process one —
every collective is a sum over one rank.  The float all-reduces of the default group run on the
native communicator (native.DpComm, csrc/dp.cpp), the rest on torch's.  The driver's multi-GPU
runs (one rank per GPU) use this backend; RCCL cannot put two ranks on one device, so this is the
RCCL coverage one GPU allows (the 2-rank decomposition itself is tests/test_dist_gpu.py, over gloo)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CFG = dict(env_id="BreakoutNoFrameskip-v4", n_envs=8, nstep=16, batch_size=48, n_epochs=2, seed=5, quiet=True)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _train(algo, cfg):
    import logger
    import ppo
    np.random.seed(11)
    torch.manual_seed(11)
    kw = dict(rnd_start=0) if algo == "PPO_RND" else {}
    alg = getattr(ppo, algo)(**cfg, **kw)
    logger.configure(algo, cfg["env_id"], quiet=True)
    alg.collect_samples()
    alg.train()
    w = [alg.flat.data[:alg.flat.n].cpu().numpy()]
    for extra in ("icm_flat", "rnd_flat"):
        if hasattr(alg, extra):
            fl = getattr(alg, extra)
            w.append(fl.data[:fl.n].cpu().numpy())
    return np.concatenate(w), alg.loss_accum.cpu().numpy(), alg.dist.enabled


def _rank(port, algo, cfg, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "ppo-exploration_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as tdist
    torch.cuda.set_device(0)
    try:
        tdist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        import dist
        import native
        dist.DistContext.enabled = property(lambda self: True)  # the world > 1 code paths on one rank
        res = _train(algo, cfg)
        # the per-minibatch all-reduces went through the native communicator (csrc/dp.cpp)
        comm = dist._dp_comm
        assert comm is not None and comm.world == 1, "native RCCL communicator not used"
        x = torch.arange(1000, dtype=torch.float64, device="cuda")
        y = x.clone()
        comm.all_reduce_(y)
        z = torch.full((4097,), 0.5, device="cuda")
        comm.all_reduce_(z, wait=False)
        comm.wait()
        assert torch.equal(x, y) and bool((z == 0.5).all())
        try:
            comm.all_reduce_(torch.zeros(4, dtype=torch.int32, device="cuda"))
            raise AssertionError("int32 accepted")
        except TypeError:
            pass
        # one asynchronous reduction at a time: the second before the join is refused
        comm.all_reduce_(z, wait=False)
        try:
            comm.all_reduce_(z, wait=False)
            raise AssertionError("second asynchronous reduction accepted")
        except native.NativeError:
            pass
        comm.wait()
        # a blocking reduction on another stream is ordered after the asynchronous one and the blocking one
        # before it (csrc/dp.cpp order_after_last)
        s2 = torch.cuda.Stream()
        with torch.cuda.stream(s2):
            u = torch.full((1 << 20,), 2.0, device="cuda")
            comm.all_reduce_(u)
        torch.cuda.current_stream().wait_stream(s2)
        assert bool((u == 2.0).all())
        # the creation self-check ran: it is the communicator's first reduction, so a wrong sum would have raised
        # inside the first train(); destroy before the process group goes (exit-time SIGSEGV)
        assert dist.shutdown() == 0 and dist._dp_comm is None and comm.handle is None
        q.put(res)
    except Exception as e:  # surface the failure to the parent
        q.put(repr(e))
    finally:
        if tdist.is_initialized():
            tdist.destroy_process_group()


@pytest.mark.parametrize("algo", ["PPO", "PPO_ICM", "PPO_RND"])
def test_rccl_one_rank_matches_single_process(algo):
    w_one, acc_one, enabled = _train(algo, CFG)
    assert not enabled
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rank, args=(_port(), algo, CFG, q))
    p.start()
    res = q.get(timeout=240)
    p.join(timeout=60)
    if isinstance(res, str):
        raise AssertionError(res)
    w, acc, enabled = res
    assert enabled
    np.testing.assert_allclose(acc, acc_one, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(w, w_one, rtol=1e-6, atol=1e-7)
