"""oracle/ — CPU restatement of the BoogaQ/PPO-exploration hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product:
only tests/, __graft_entry__.smoke() and bench.py's `cpu_baseline` leg may
import it, and only as the checker (or as the timed CPU baseline).  The
product path (ppo-exploration_amd/) never imports it and fails loudly when
its HIP library is missing.

Every function cites the reference file:line whose behaviour it restates.
The restatement is pinned by tests/golden/*.npz, which were produced by
running the reference itself (tests/golden/make_golden.py).
"""
