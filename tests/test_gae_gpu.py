"""K1 GAE on the GPU through the C ABI vs the golden fixtures and the oracle.
Bit-exact (np.array_equal) at every size."""
import numpy as np
import pytest
import torch

from oracle import gae as G

pytestmark = pytest.mark.gpu


def _dev(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.cuda()


def _run_single(rew, val, done, lv, ld, gamma, lam):
    import native
    T, N = rew.shape
    adv = torch.empty(T, N, device="cuda")
    ret = torch.empty(T, N, device="cuda")
    native.gae(_dev(rew), _dev(val), _dev(done, torch.uint8), _dev(lv), _dev(ld, torch.uint8),
               gamma, lam, adv, ret)
    torch.cuda.synchronize()
    return adv.cpu().numpy(), ret.cpu().numpy()


def test_gae_golden(golden):
    f = golden("gae_single")
    for k in range(int(f["ncases"])):
        p = f"c{k}_"
        adv, ret = _run_single(f[p + "rewards"], f[p + "values"], f[p + "dones"], f[p + "last_value"],
                               f[p + "last_done"], float(f[p + "gamma"]), float(f[p + "lam"]))
        assert np.array_equal(adv, f[p + "advantages"]), p
        assert np.array_equal(ret, f[p + "returns"]), p


def test_gae_dual_golden(golden):
    import native
    f = golden("gae_dual")
    for k in range(int(f["ncases"])):
        p = f"c{k}_"
        T, N = f[p + "rewards"].shape
        outs = [torch.empty(T, N, device="cuda") for _ in range(4)]
        native.gae_dual(_dev(f[p + "rewards"]), _dev(f[p + "values"]), _dev(f[p + "dones"], torch.uint8),
                        _dev(f[p + "last_value"]), _dev(f[p + "last_done"], torch.uint8),
                        _dev(f[p + "int_rewards"]), _dev(f[p + "int_values"]), _dev(f[p + "last_int_value"]),
                        float(f[p + "gamma"]), float(f[p + "int_gamma"]), float(f[p + "lam"]), *outs)
        torch.cuda.synchronize()
        for o, key in zip(outs, ("advantages", "returns", "int_advantages", "int_returns")):
            assert np.array_equal(o.cpu().numpy(), f[p + key]), (p, key)


@pytest.mark.parametrize("T,N", [(128, 4096), (128, 131072 + 4), (128, 131072), (3, 5), (1, 200000), (16, 262144),
                                 (8, 262144 + 2), (4, 131071)])
def test_gae_random_vs_oracle(T, N):
    """Covers every lane width (1 env/lane, float2 lanes from N = 131,072, float4 lanes from
    262,144; odd N falls back to 1 env/lane) and ragged N."""
    rs = np.random.RandomState(T * 7 + N)
    rew = (rs.rand(T, N) < 0.02).astype(np.float32) + rs.randn(T, N).astype(np.float32) * 0.1
    val = rs.randn(T, N).astype(np.float32)
    done = rs.rand(T, N) < 0.01
    lv = rs.randn(N).astype(np.float32)
    ld = done[-1]
    adv, ret = _run_single(rew, val, done, lv, ld, 0.99, 0.95)
    eadv, eret = G.gae_single(rew, val, done, lv, ld, 0.99, 0.95)
    assert np.array_equal(adv, eadv)
    assert np.array_equal(ret, eret)


def test_gae_dual_random_vs_oracle():
    import native
    T, N = 128, 131072
    rs = np.random.RandomState(5)
    a = [rs.randn(T, N).astype(np.float32) for _ in range(4)]
    done = rs.rand(T, N) < 0.01
    lv, liv = rs.randn(N).astype(np.float32), rs.randn(N).astype(np.float32)
    outs = [torch.empty(T, N, device="cuda") for _ in range(4)]
    native.gae_dual(_dev(a[0]), _dev(a[1]), _dev(done, torch.uint8), _dev(lv), _dev(done[-1], torch.uint8),
                    _dev(a[2]), _dev(a[3]), _dev(liv), 0.99, 0.999, 0.95, *outs)
    torch.cuda.synchronize()
    exp = G.gae_dual(a[0], a[2], a[1], a[3], done, lv, liv, done[-1], 0.99, 0.999, 0.95)
    for o, e in zip(outs, exp):
        assert np.array_equal(o.cpu().numpy(), e)
