"""A/B timing of the conv1 -> conv2 kernels on f32 h1 (the round-2 split forms) and on H1P (conv1's
output as f16 planes) at one batch, same box, HIP-event mean over reps (dev tool).
Usage: python tools/probes/h1p_bench.py [batch] [reps]"""
import json
import os
os.environ.setdefault("PPOX_AB", "1")  # this tool switches kernel forms / gates (native.ab_env)
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "ppo-exploration_amd"))
import torch  # noqa: E402
import native  # noqa: E402

if os.environ.get("PPOX_LIB"):
    native.load(os.environ["PPOX_LIB"])


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    torch.manual_seed(0)
    w1 = torch.randn(32, 4, 8, 8, device="cuda") * 0.05
    w2 = torch.randn(64, 32, 4, 4, device="cuda") * 0.05
    w3 = torch.randn(64, 64, 3, 3, device="cuda") * 0.05
    b1, b2 = torch.randn(32, device="cuda"), torch.randn(64, device="cuda") * 0.1
    q = {k: torch.empty(native.nature_split_pack_elems(k), dtype=torch.int16, device="cuda") for k in (1, 2, 3)}
    native.nature_pack_all(w1, w2, w3, None, None, q[1], q[2], q[3], None, None, None, None, b1=b1)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda")
    h1 = torch.empty(B, 20, 20, 32, device="cuda")
    h1p = torch.empty(B, 20, 20, 64, dtype=torch.int16, device="cuda")
    bits = torch.empty(B * 400, dtype=torch.int32, device="cuda")
    am = native.amax_table(4, "cuda")
    y = torch.empty(B, 9, 9, 64, device="cuda")
    bits2 = torch.empty(B * 162, dtype=torch.int32, device="cuda")
    g2 = torch.randn(B, 9, 9, 64, device="cuda")
    dw, db = torch.empty(64, 32, 4, 4, device="cuda"), torch.empty(64, device="cuda")
    ws = torch.empty(max(native.nature_wgrad_split_workspace_bytes(2, B),
                         native.nature_conv2_wgrad_planes_workspace_bytes(B)), dtype=torch.uint8, device="cuda")
    native.amax(g2, am[2])
    out = {"batch": B}
    out["fwd1_f32"] = timed(lambda: native.nature_conv_fwd_split(1, x, B, None, 0, 0, 28224, q[1], b1, h1,
                                                                 amax_y=am[0], relu_bits=bits), reps)
    out["fwd1_h1p"] = timed(lambda: native.nature_conv1_fwd_planes(x, B, None, 0, 0, 28224, q[1], b1, h1p,
                                                                   relu_bits=bits), reps)
    out["fwd2_f32"] = timed(lambda: native.nature_conv_fwd_split(2, h1, B, None, 0, 0, 0, q[2], b2, y, amax_x=am[0],
                                                                 amax_y=am[1], relu_bits=bits2), reps)
    out["fwd2_h1p"] = timed(lambda: native.nature_conv2_fwd_planes(h1p, q[1], B, q[2], b2, y, amax_y=am[1],
                                                                   relu_bits=bits2), reps)
    out["wgrad2_f32"] = timed(lambda: native.nature_conv_wgrad_split(2, h1, B, 0, g2, ws, dw, db, amax_x=am[0],
                                                                     amax_g=am[2]), reps)
    out["wgrad2_h1p"] = timed(lambda: native.nature_conv2_wgrad_planes(h1p, q[1], B, g2, ws, dw, db, amax_g=am[2]),
                              reps)
    print(json.dumps({k: round(v, 1) if isinstance(v, float) else v for k, v in out.items()}))


if __name__ == "__main__":
    main()
