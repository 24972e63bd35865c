"""GAE(lambda) restated in numpy with the reference's exact dtype promotions.

Test infrastructure only (see oracle/__init__.py).

Reference: buffer.py:203-230 (RolloutStorage, one stream) and
buffer.py:321-362 (IntrinsicStorage, extrinsic + non-episodic intrinsic).

Promotion facts the reference code produces (numpy, Python-float scalars are
"weak"):
  * gamma * next_value            -> float32 multiply with f32(gamma)
  * (...) * next_non_terminal     -> float64 (1.0 - done is float64)
  * r + (...) - v                 -> float64
  * gamma * lam                   -> Python float (f64) product
  * carry = delta + ((gl * nnt) * carry)   float64 carry
  * advantages[t] = f32(carry);  returns = adv + values (float32)
  * intrinsic stream: everything float32, f32(int_gamma * lam) multiplier.
"""
import numpy as np


def _nnt(flags):
    return 1.0 - np.asarray(flags).astype(np.float64)


def gae_single(rewards, values, step_dones, last_value, last_done, gamma, lam):
    """buffer.py:217-230.  step_dones[t] = done flag stored by add() at step t
    (ppo.py:192 passes `dones` as the mask); last_value = V(s_{T-1}) (ppo.py:196).
    Returns (advantages f32 (T,N), returns f32 (T,N))."""
    rewards = np.asarray(rewards, np.float32)
    values = np.asarray(values, np.float32)
    T, N = rewards.shape
    g32 = np.float32(gamma)
    gl = float(gamma) * float(lam)
    adv = np.zeros((T, N), np.float32)
    carry = np.zeros(N, np.float64)
    for t in range(T - 1, -1, -1):
        if t == T - 1:
            nnt = _nnt(last_done)
            nv = np.asarray(last_value, np.float32).reshape(N)
        else:
            nnt = _nnt(step_dones[t + 1])
            nv = values[t + 1]
        gv = g32 * nv                                         # f32
        delta = (rewards[t].astype(np.float64) + gv.astype(np.float64) * nnt) \
            - values[t].astype(np.float64)
        carry = delta + (gl * nnt) * carry
        adv[t] = carry.astype(np.float32)
    return adv, adv + values


def gae_intrinsic(int_rewards, int_values, last_int_value, int_gamma, lam):
    """Intrinsic stream of buffer.py:343-362: no done mask, float32 throughout."""
    ir = np.asarray(int_rewards, np.float32)
    iv = np.asarray(int_values, np.float32)
    T, N = ir.shape
    ig32 = np.float32(int_gamma)
    igl32 = np.float32(float(int_gamma) * float(lam))
    iadv = np.zeros((T, N), np.float32)
    carry = None
    for t in range(T - 1, -1, -1):
        niv = np.asarray(last_int_value, np.float32).reshape(N) if t == T - 1 else iv[t + 1]
        d = (ir[t] + ig32 * niv) - iv[t]
        carry = (d + np.float32(0.0)) if carry is None else (d + igl32 * carry)
        iadv[t] = carry
    return iadv, iadv + iv


def gae_dual(rewards, int_rewards, values, int_values, step_dones, last_value,
             last_int_value, last_done, gamma, int_gamma, lam):
    """IntrinsicStorage.compute_returns_and_advantages (buffer.py:321-362)."""
    a, r = gae_single(rewards, values, step_dones, last_value, last_done, gamma, lam)
    ia, ir = gae_intrinsic(int_rewards, int_values, last_int_value, int_gamma, lam)
    return a, r, ia, ir
