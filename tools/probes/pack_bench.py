"""Per-optimizer-step packing cost by form (dev tool): times ppox_nature_pack_all (wmax + pack launches)
with every form of the per-rank step, then with subsets, and Adam / sumsq over the policy's flat
parameter count, on one stream with HIP events.  Usage: python tools/probes/pack_bench.py [reps=200]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "ppo-exploration_amd"))
import native  # noqa: E402


def timed(fn, reps):
    for _ in range(10):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = "cuda"
    w1, b1 = torch.randn(32, 4, 8, 8, device=dev) * 0.05, torch.randn(32, device=dev) * 0.1
    w2, w3 = torch.randn(64, 32, 4, 4, device=dev) * 0.05, torch.randn(64, 64, 3, 3, device=dev) * 0.05
    wfc, wh = torch.randn(512, 3136, device=dev) * 0.02, torch.randn(512, 512, device=dev) * 0.04
    i16 = lambda n: torch.empty(n, dtype=torch.int16, device=dev)
    q = {k: i16(native.nature_split_pack_elems(k)) for k in (1, 2, 3, 12, 13)}
    nfc, nh = native.nature_fc_pack_elems(), native.head_hidden_pack_elems()
    qfc, qh = (i16(nfc), i16(nfc)), (i16(nh), i16(nh))
    wpd2 = torch.empty(64 * 16 * 32, device=dev)
    zero = torch.empty(16 * 256, dtype=torch.int32, device=dev)
    full = dict(wpd2=None, q1=q[1], q2=q[2], q3=q[3], qd2=q[12], qd3=q[13], qfc_fwd=qfc[0], qfc_dgrad=qfc[1],
                qh_fwd=qh[0], qh_dgrad=None)
    cases = {
        "per-rank step (conv forms + fc fwd/dgrad + hidden fwd)": full,
        "conv forms only": dict(full, qfc_fwd=None, qfc_dgrad=None, qh_fwd=None),
        "fc forward form only": {k: (v if k == "qfc_fwd" else None) for k, v in full.items()},
        "fc dgrad form only": {k: (v if k == "qfc_dgrad" else None) for k, v in full.items()},
        "hidden forward form only": {k: (v if k == "qh_fwd" else None) for k, v in full.items()},
        "q1 only (conv1 forward + H1P exponent)": {k: (v if k == "q1" else None) for k, v in full.items()},
    }
    for name, f in cases.items():
        us = timed(lambda: native.nature_pack_all(w1, w2, w3, wfc, f["wpd2"], f["q1"], f["q2"], f["q3"], f["qd2"],
                                                  f["qd3"], f["qfc_fwd"], f["qfc_dgrad"], wh, f["qh_fwd"],
                                                  f["qh_dgrad"], b1=b1 if f["q1"] is not None else None, zero=zero),
                   reps)
        print(f"pack_all {name:55s} {us:7.1f} us")
    n = 8224 + 32832 + 36928 + 1606144 + 2052 + 262656 + 513
    p, g, m, v = (torch.randn(n, device=dev) * 0.01 for _ in range(4))
    v.abs_()
    parts = torch.empty(256, dtype=torch.float64, device=dev)
    print(f"sumsq  {timed(lambda: native.grad_sumsq(g, parts), reps):7.1f} us  (n = {n})")
    print(f"adam   {timed(lambda: native.adam_step(p, g, m, v, parts, 0.5, 2.5e-4, 0.9, 0.999, 1e-8, 5), reps):7.1f} us")


if __name__ == "__main__":
    main()
