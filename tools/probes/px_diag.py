"""Per-tensor error of one PX-on / PX-off training pass against float64 (dev tool: the body of
tests/test_px_gpu.py::test_px_training_pass_is_fp32_class, printing every tensor's e_on, e_off instead
of stopping at the first).  Usage: python tools/probes/px_diag.py [B]   (kernel switches via the environment)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "ppo-exploration_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
import torch  # noqa: E402

import convs  # noqa: E402
from test_px_gpu import _fp64_masked, _pass, _setup  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    convs.PX_MIN_BATCH = 0
    convs.PX_DF = True
    net, ref, flat, cv = _setup(B)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(B + 1)
    dout = torch.randn(B, 4, device="cuda", generator=g)
    dv = torch.randn(B, device="cuda", generator=g)
    m_on, m_off = [], []
    if os.environ.get("DIAG_ON_FIRST") == "1":
        o_on, v_on, g_on, am = _pass(net, flat, cv, x, dout, dv, True, m_on)
        o_off, v_off, g_off, _ = _pass(net, flat, cv, x, dout, dv, False, m_off)
    else:
        o_off, v_off, g_off, _ = _pass(net, flat, cv, x, dout, dv, False, m_off)
        o_on, v_on, g_on, am = _pass(net, flat, cv, x, dout, dv, True, m_on)
    if os.environ.get("DIAG_TWICE") == "1":  # the PX-on pass again: run to run
        o2, v2, g2, _ = _pass(net, flat, cv, x, dout, dv, True)
        print("PX-on run to run:", max(float((g2[n] - g_on[n]).abs().max()) for n in g2))
    print("ReLU decisions differing on/off:", [int((a != b).sum()) if a is not None and b is not None else None
                                               for a, b in zip(m_on, m_off)])
    o64, v64, g64 = _fp64_masked(ref, x, dout, dv, m_on)
    r_off = _fp64_masked(ref, x, dout, dv, m_off)
    env = {k: v for k, v in os.environ.items() if k.startswith("PPOX_")}
    print("env", env, "px", am.px)
    for name, r in list(g64.items()) + [("out", o64), ("v", v64)]:
        a = o_on if name == "out" else v_on if name == "v" else g_on[name]
        b = o_off if name == "out" else v_off if name == "v" else g_off[name]
        scale = r.abs().max().item() + 1e-30
        e_on = (a.cpu().double() - r).abs().max().item() / scale
        rb = r_off[0] if name == "out" else r_off[1] if name == "v" else r_off[2][name]
        e_off = (b.cpu().double() - rb).abs().max().item() / scale
        print(f"{name:32s} on {e_on:.3e} off {e_off:.3e} ratio {e_on / max(e_off, 1e-12):8.2f}", flush=True)


def intermediates(B=2048):
    """f, e, amax_f of the PX-on and PX-off forward passes side by side"""
    import numpy as np
    convs.PX_MIN_BATCH = 0
    net, ref, flat, cv = _setup(B)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda")
    outs = {}
    for px in (False, True):
        cv.px = px
        out, v, _, ctx = net.forward_train(x)
        torch.cuda.synchronize()
        _, _, _, h3, f, e, _, am = ctx
        outs[px] = (f.clone(), e.clone(), out.clone(), v.clone(),
                    float(am[convs.AM_F].cpu().numpy().view(np.float32).max()), float(f.abs().max()))
    rel = lambda a, b: float((a - b).abs().max() / b.abs().max())
    print("f", rel(outs[True][0], outs[False][0]), "e", rel(outs[True][1], outs[False][1]),
          "out", rel(outs[True][2], outs[False][2]), "v", rel(outs[True][3], outs[False][3]))
    print("amax_f on/off", outs[True][4], outs[False][4], "f max", outs[True][5], outs[False][5])
    d = (outs[True][0] - outs[False][0]).abs()
    idx = torch.nonzero(d > 1e-5 * outs[False][0].abs().max())
    print("f entries off by > 1e-5 of max:", idx.shape[0], idx[:10].tolist())


def backward_intermediates(B=2048):
    """de, df and the hidden-layer weight gradient's inputs of the PX-on / PX-off passes side by side"""
    import native
    convs.PX_MIN_BATCH = 0
    convs.PX_DF = True
    net, ref, flat, cv = _setup(B)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(B + 1)
    dout = torch.randn(B, 4, device="cuda", generator=g)
    dv = torch.randn(B, device="cuda", generator=g)
    cap = {}
    wraps = {}
    for fn in ("head_backward", "head_hidden_wgrad", "px_split", "head_grads", "nature_fc_wgrad"):
        orig = getattr(native, fn)

        def w(*a, _o=orig, _n=fn, **k):
            r = _o(*a, **k)
            cap.setdefault(_n, []).append([t.clone() if isinstance(t, torch.Tensor) else t for t in a])
            return r
        wraps[fn] = orig
        setattr(native, fn, w)
    res = {}
    for px in (False, True):
        cap.clear()
        _pass(net, flat, cv, x, dout, dv, px)
        res[px] = {k: v[0] for k, v in cap.items()}
    rel = lambda a, b: float((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-30))
    for k in set(res[True]) & set(res[False]):
        for i, (a, b) in enumerate(zip(res[True][k], res[False][k])):
            if isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor) and a.shape == b.shape and a.dtype == b.dtype \
                    and a.is_floating_point():
                print(f"{k} arg {i} {tuple(a.shape)} rel {rel(a, b):.3e}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "fwd":
        intermediates(int(sys.argv[1]))
    elif len(sys.argv) > 2 and sys.argv[2] == "bwd":
        backward_intermediates(int(sys.argv[1]))
    else:
        main()
