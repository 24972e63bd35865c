"""cProfile of one PPO train() at the per-rank shape: where the host time per minibatch goes
(dev tool).  Usage: python tools/host_prof.py [envs] [batch]"""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-exploration_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import logger  # noqa: E402
import ppo  # noqa: E402

envs = int(sys.argv[1]) if len(sys.argv) > 1 else 512
bs = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
np.random.seed(0)
torch.manual_seed(0)
logger.configure("PPO", "BreakoutNoFrameskip-v4", quiet=True)
alg = ppo.PPO(env_id="BreakoutNoFrameskip-v4", n_envs=envs, nstep=128, batch_size=bs, n_epochs=10, seed=1, quiet=True)
alg.collect_samples()
alg.train()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
alg.train()
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(35)
