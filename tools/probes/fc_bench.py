"""fc layer (3136 -> 512) split-f16 GEMM vs rocBLAS f32 (torch) at the training batch:
time and error vs float64.  Usage: python tools/probes/fc_bench.py [B] [lib.so]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "ppo-exploration_amd"))
import native  # noqa: E402


def t_ms(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    if len(sys.argv) > 2:
        native.load(sys.argv[2])
    d = "cuda"
    torch.manual_seed(0)
    W = torch.randn(512, 3136, device=d) * 0.02
    b = torch.randn(512, device=d) * 0.1
    h3n = torch.relu(torch.randn(B, 7, 7, 64, device=d))        # NHWC (the split kernels' order)
    h3 = h3n.permute(0, 3, 1, 2).reshape(B, 3136)               # Flatten order (rocBLAS reference)
    df = torch.randn(B, 512, device=d)
    n = native.nature_fc_pack_elems()
    qf, qd = torch.empty(n, dtype=torch.int16, device=d), torch.empty(n, dtype=torch.int16, device=d)
    native.nature_fc_pack(W, qf, qd)
    f = torch.empty(B, 512, device=d)
    g3 = torch.empty(B, 7, 7, 64, device=d)
    am = native.amax_table(2, d)  # operand amax rows, recorded once (the product's producers record them)
    native.amax(h3n, am[0])
    native.amax(df, am[1])
    flop = 2.0 * B * 3136 * 512
    res = {"B": B}
    res["split_fwd_ms"] = t_ms(lambda: native.nature_fc_fwd(h3n, B, qf, b, f, amax_h3=am[0]))
    res["rocblas_fwd_ms"] = t_ms(lambda: torch.relu(torch.addmm(b, h3, W.t())))
    wsk = torch.empty(max(native.nature_fc_fwd_splitk_workspace_bytes(B), 16), dtype=torch.uint8, device=d)
    fsk = torch.empty(B, 512, device=d)
    res["splitk_fwd_ms"] = t_ms(lambda: native.nature_fc_fwd_splitk(h3n, B, qf, b, wsk, fsk, amax_h3=am[0]))
    res["addmm_act_fwd_ms"] = t_ms(lambda: torch._addmm_activation(b, h3, W.t()))
    res["split_dgrad_ms"] = t_ms(lambda: native.nature_fc_dgrad(df, B, qd, h3n, g3, amax_df=am[1]))
    res["rocblas_dgrad_ms"] = t_ms(lambda: torch.mm(df, W))
    ws = torch.empty(native.nature_fc_wgrad_workspace_bytes(B), dtype=torch.uint8, device=d)
    dw = torch.empty(512, 3136, device=d)
    res["split_wgrad_ms"] = t_ms(lambda: native.nature_fc_wgrad(df, B, h3n, ws, dw, amax_df=am[1], amax_h3=am[0]))
    res["rocblas_wgrad_ms"] = t_ms(lambda: torch.mm(df.t(), h3))
    for k in list(res):
        if k.endswith("_ms"):
            res[k.replace("_ms", "_TFs")] = round(flop / (res[k] * 1e-3) / 1e12, 1)
            res[k] = round(res[k], 3)
    # accuracy vs float64 (first 512 rows)
    r = 512
    ref = torch.relu(h3[:r].double() @ W.double().t() + b.double())
    native.nature_fc_fwd(h3n, B, qf, b, f)
    f32 = torch.relu(torch.addmm(b, h3[:r], W.t()))
    res["fwd_err_split"] = float((f[:r].double() - ref).abs().max() / ref.abs().max())
    res["fwd_err_f32"] = float((f32.double() - ref).abs().max() / ref.abs().max())
    native.nature_fc_fwd_splitk(h3n, B, qf, b, wsk, fsk)
    res["fwd_err_splitk"] = float((fsk[:r].double() - ref).abs().max() / ref.abs().max())
    res["splitk_vs_split_maxdiff"] = float((fsk - f).abs().max() / f.abs().max())
    refd = (df[:r].double() @ W.double()).view(r, 64, 7, 7).permute(0, 2, 3, 1) * (h3n[:r] > 0)
    native.nature_fc_dgrad(df, B, qd, h3n, g3)
    res["dgrad_err_split"] = float((g3[:r].double() - refd).abs().max() / refd.abs().max())
    print(json.dumps(res))


if __name__ == "__main__":
    main()
