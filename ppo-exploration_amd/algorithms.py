"""The reference imports its algorithms from `algorithms` (main.py:5), a byte-identical copy
of ppo.py.  Same classes here."""
from ppo import BaseAlgorithm, Policy, PPO, PPO_ICM, PPO_RND  # noqa: F401
