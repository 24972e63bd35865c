"""cProfile of the collect loop's host side (dev tool): where the per-step host time of
collect_samples() goes at a launch-bound env count.  Usage: python tools/collect_cprofile.py [envs]"""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-exploration_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ppo  # noqa: E402


def main():
    envs = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    np.random.seed(0)
    torch.manual_seed(0)
    alg = ppo.PPO(env_id="BreakoutNoFrameskip-v4", n_envs=envs, nstep=128, batch_size=envs * 4, n_epochs=1, seed=1,
                  quiet=True)
    alg.collect_samples()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    alg.collect_samples()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
