"""Host-side profile of one PPO train() (dev tool): cProfile of the Python / ctypes launch path
at a given shape, top functions by own time.  Usage: python tools/probes/host_profile.py [envs] [batch] [algo] [dist]
("dist": the data-parallel branches on over a one-rank RCCL communicator, as bench.py --force-dist)"""
import cProfile
import os
os.environ.setdefault("PPOX_AB", "1")  # this tool switches kernel forms / gates (native.ab_env)
import pstats
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "ppo-exploration_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ppo  # noqa: E402


def main():
    envs = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    bs = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    algo = sys.argv[3] if len(sys.argv) > 3 else "ppo"
    if len(sys.argv) > 4 and sys.argv[4] == "dist":
        import socket
        import torch.distributed as tdist
        import dist
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(sk.getsockname()[1]))
        sk.close()
        torch.cuda.set_device(0)
        tdist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        dist.DistContext.enabled = property(lambda self: True)
    np.random.seed(0)
    torch.manual_seed(0)
    cls = {"ppo": ppo.PPO, "icm": ppo.PPO_ICM, "rnd": ppo.PPO_RND}[algo]
    alg = cls(env_id="BreakoutNoFrameskip-v4", n_envs=envs, nstep=128, batch_size=bs, n_epochs=2, seed=1, quiet=True)
    alg.collect_samples()
    alg.train()
    torch.cuda.synchronize()
    alg.collect_samples()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    alg.train()
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    n_mb = 2 * (envs * 128 // bs)
    print(f"minibatches {n_mb}; total host s {st.total_tt:.3f} = {1e6 * st.total_tt / n_mb:.0f} us per minibatch")
    st.sort_stats("tottime").print_stats(45)


if __name__ == "__main__":
    main()
