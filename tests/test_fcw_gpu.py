"""The fc forward in 256 x 128 tiles (csrc/dconv.hip fcw_kernel, round 5): ppox_nature_fc_fwd on PX h3 from
PPOX_FCW_MIN rows (default 8192), the sg2 form's hi / lo accumulator pair per 32 x 32 tile.  Held to float64:
no larger than twice the error of torch's f32 GEMM and of the sg2 form on the same planes (PPOX_FCW=0), its
amax the output's, bitwise run to run, nothing written past the batch.  Reference layer: .ipynb_checkpoints/models-checkpoint.py:58-59 (Linear(3136, 512) + ReLU)."""
import os

import numpy as np
import pytest
import torch

from test_ddgrad2_gpu import _planes, _split_exp, _values

pytestmark = pytest.mark.gpu


def _fwd(h3p, E, B, qf, b, form):
    import native
    env = {"PPOX_FCW": "1" if form == "wide" else "0", "PPOX_FCW_MIN": "1"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        f = torch.full((B + 1, 512), 7.0, device="cuda")
        am = native.amax_table(1, "cuda")[0]
        native.nature_fc_fwd(h3p, B, qf, b, f, amax_f=am, h3_exp=torch.tensor([E], dtype=torch.int32, device="cuda"))
        torch.cuda.synchronize()
        return f, float(am.cpu().numpy().view(np.float32).max())
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("B", [1, 255, 256, 257, 2048, 9001, 16384])
def test_fc_fwd_wide_vs_fp64(B):
    import native
    torch.manual_seed(B)
    W = torch.randn(512, 3136, device="cuda") * 0.02
    b = torch.randn(512, device="cuda") * 0.1
    h3n = torch.relu(torch.randn(B, 7, 7, 64, device="cuda")) * torch.rand(B, 7, 7, 64, device="cuda")
    E = _split_exp(float(h3n.abs().max()))
    h3p = _planes(h3n, E)
    h3v = _values(h3p, E)
    n = native.nature_fc_pack_elems()
    qf, qd = torch.empty(n, dtype=torch.int16, device="cuda"), torch.empty(n, dtype=torch.int16, device="cuda")
    native.nature_fc_pack(W, qf, qd)
    fw, amw = _fwd(h3p, E, B, qf, b, "wide")
    fs, _ = _fwd(h3p, E, B, qf, b, "sg2")
    assert bool((fw[B] == 7.0).all()), "nothing written past the batch"
    f = fw[:B]
    assert amw == float(f.max())
    h3 = h3v.permute(0, 3, 1, 2).reshape(B, 3136)  # the reference's Flatten order
    ref = torch.relu(h3.double() @ W.double().t() + b.double())
    scale = ref.abs().max()
    e_w = float((f.double() - ref).abs().max() / scale)
    e_s = float((fs[:B].double() - ref).abs().max() / scale)
    e_f = float((torch.relu(torch.addmm(b, h3, W.t())).double() - ref).abs().max() / scale)
    assert e_w <= 2 * max(e_f, e_s) + 1e-7, (e_w, e_f, e_s)


def test_fc_fwd_wide_is_deterministic():
    import native
    torch.manual_seed(3)
    B = 4096
    W = torch.randn(512, 3136, device="cuda") * 0.02
    b = torch.randn(512, device="cuda") * 0.1
    h3n = torch.relu(torch.randn(B, 7, 7, 64, device="cuda"))
    E = _split_exp(float(h3n.abs().max()))
    h3p = _planes(h3n, E)
    n = native.nature_fc_pack_elems()
    qf, qd = torch.empty(n, dtype=torch.int16, device="cuda"), torch.empty(n, dtype=torch.int16, device="cuda")
    native.nature_fc_pack(W, qf, qd)
    a = _fwd(h3p, E, B, qf, b, "wide")
    c = _fwd(h3p, E, B, qf, b, "wide")
    assert torch.equal(a[0], c[0]) and a[1] == c[1]


@pytest.mark.parametrize("B", [1024, 2048, 3000, 8191])
def test_fc_fwd_wide_splitk_vs_fp64(B):
    """the small-batch form (PPOX_FCW_SK_MIN .. PPOX_FCW_MIN rows): the 256 x 128 tiles split 8 ways over K into
    slabs, summed in order with bias + ReLU + the fused actor head by fc_fwd_sk_reduce_actor — against float64,
    the sg2 split-K form (PPOX_FCW=0) and torch's f32 GEMM; logits as the same reduce computes them from f"""
    import native
    torch.manual_seed(B)
    W = torch.randn(512, 3136, device="cuda") * 0.02
    b = torch.randn(512, device="cuda") * 0.1
    wa, ba = torch.randn(4, 512, device="cuda") * 0.05, torch.randn(4, device="cuda") * 0.1
    h3n = torch.relu(torch.randn(B, 7, 7, 64, device="cuda")) * torch.rand(B, 7, 7, 64, device="cuda")
    E = _split_exp(float(h3n.abs().max()))
    h3p = _planes(h3n, E)
    h3v = _values(h3p, E)
    n = native.nature_fc_pack_elems()
    qf, qd = torch.empty(n, dtype=torch.int16, device="cuda"), torch.empty(n, dtype=torch.int16, device="cuda")
    native.nature_fc_pack(W, qf, qd)
    outs = {}
    for form, v in (("wide", "1"), ("sg2", "0")):
        old = os.environ.get("PPOX_FCW")
        os.environ["PPOX_FCW"] = v
        try:
            ws = torch.empty(native.nature_fc_fwd_splitk_workspace_bytes(B), dtype=torch.uint8, device="cuda")
            f = torch.full((B + 1, 512), 7.0, device="cuda")
            lg = torch.empty(B, 4, device="cuda")
            am = native.amax_table(1, "cuda")[0]
            native.nature_fc_fwd_splitk(h3p, B, qf, b, ws, f[:B], amax_f=am, actor=(wa, ba), logits=lg,
                                        h3_exp=torch.tensor([E], dtype=torch.int32, device="cuda"))
            torch.cuda.synchronize()
            outs[form] = (f, lg, float(am.cpu().numpy().view(np.float32).max()))
        finally:
            if old is None:
                os.environ.pop("PPOX_FCW", None)
            else:
                os.environ["PPOX_FCW"] = old
    fw, lw, amw = outs["wide"]
    assert bool((fw[B] == 7.0).all())
    f = fw[:B]
    assert amw == float(f.max())
    h3 = h3v.permute(0, 3, 1, 2).reshape(B, 3136)
    ref = torch.relu(h3.double() @ W.double().t() + b.double())
    scale = ref.abs().max()
    err = lambda x: float((x.double() - ref).abs().max() / scale)
    assert err(f) <= 2 * max(err(torch.relu(torch.addmm(b, h3, W.t()))), err(outs["sg2"][0][:B])) + 1e-7
    refl = f.double() @ wa.double().t() + ba.double()
    assert float((lw.double() - refl).abs().max() / refl.abs().max()) <= 1e-5
