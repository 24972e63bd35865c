"""Running moments and observation normalisation restated in numpy.

Test infrastructure only (see oracle/__init__.py).

Reference: util.py:9-44 (RunningMeanStd: batch mean/var over axis 0,
Chan et al. parallel merge into float64 state, count starts at epsilon=1e-4)
and ppo.py:111-118 (normalize_obs: clip((x-mean)/sqrt(var+1e-10), -5, 5) as
float64).
"""
import numpy as np


class RunningMoments:
    """util.py:9-18 state: mean f64 zeros(shape), var f64 ones(shape), count=eps."""

    def __init__(self, epsilon=1e-4, shape=()):
        self.mean = np.zeros(shape, np.float64)
        self.var = np.ones(shape, np.float64)
        self.count = epsilon

    def update(self, arr):
        """util.py:20-28: moments over axis 0 in numpy's own reduction dtype."""
        arr = np.asarray(arr)
        self.merge(np.mean(arr, axis=0), np.var(arr, axis=0), arr.shape[0])

    def merge(self, bmean, bvar, bcount):
        """util.py:30-44 (Chan parallel combination)."""
        d = bmean - self.mean
        n = self.count + bcount
        mean = self.mean + d * bcount / n
        m2 = self.var * self.count + bvar * bcount + np.square(d) * self.count * bcount / (self.count + bcount)
        self.mean, self.var, self.count = mean, m2 / (self.count + bcount), bcount + self.count


def normalize_obs(obs, mean, var):
    """ppo.py:117 — float64 result."""
    return np.clip((obs - mean) / np.sqrt(var + 1e-10), -5, 5).astype(float)
