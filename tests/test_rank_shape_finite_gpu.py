"""The per-rank training shape in ONE process, many minibatches (round 6): PPO_ICM at 512 envs x 128 steps,
minibatch 2,048 (the 8-GPU per-rank shape of BASELINE configs 1 / 4), its epoch repeated on one rollout; after
every minibatch the policy and ICM gradients must be finite.  The 8-rank C4 test (8 processes sharing one GPU)
saw non-finite conv gradients in about one rank pass in 100-200; this is the same kernels and stream layout
without co-tenancy, ~600 passes.  Reference: ppo.py:651-713 (the PPO_ICM minibatch loop)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_per_rank_shape_gradients_stay_finite():
    import ppo
    np.random.seed(3)
    torch.manual_seed(3)
    alg = ppo.PPO_ICM(env_id="BreakoutNoFrameskip-v4", n_envs=512, nstep=128, batch_size=2048, n_epochs=1, seed=3,
                      quiet=True)
    alg.collect_samples()
    bad = []
    step = alg.icm_flat.adam_step
    count = [0]

    def icm_step(*a, **k):
        ok = bool(torch.isfinite(alg.flat.grad).all()) and bool(torch.isfinite(alg.icm_flat.grad).all())
        if not ok:
            bad.append(count[0])
        count[0] += 1
        return step(*a, **k)
    alg.icm_flat.adam_step = icm_step
    epochs = int(os.environ.get("PPOX_STRESS_EPOCHS", "18"))  # (tools/gpu.sh cstress: longer, beside other load)
    for _ in range(epochs):
        alg.train()
    assert count[0] == epochs * 32
    assert not bad, f"non-finite gradients at minibatches {bad} of {count[0]}"
