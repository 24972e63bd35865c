"""List the torch ops (and the Python lines that issue them) launched per PPO minibatch at
the per-rank shape — finds library kernels between the libppox launches (dev tool)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "ppo-exploration_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import logger  # noqa: E402
import ppo  # noqa: E402

algo = sys.argv[1] if len(sys.argv) > 1 else "PPO"
cls = getattr(ppo, algo)
np.random.seed(0)
torch.manual_seed(0)
logger.configure(algo, "BreakoutNoFrameskip-v4", quiet=True)
alg = cls(env_id="BreakoutNoFrameskip-v4", n_envs=512, nstep=128, batch_size=2048, n_epochs=1, quiet=True)
alg.collect_samples()
alg.train()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    alg.train()
    torch.cuda.synchronize()
print(prof.key_averages(group_by_stack_n=4).table(sort_by="cuda_time_total", row_limit=40, max_name_column_width=60))
