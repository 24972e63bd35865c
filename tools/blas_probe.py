"""rocBLAS vs hipBLASLt (torch preferred_blas_library) on the f32 GEMMs left on the
library in the training step (dev tool).  Usage: python tools/blas_probe.py [B]"""
import json
import sys

import torch


def t_ms(fn, iters=20):
    for _ in range(3):
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
    d = "cuda"
    g = torch.Generator(device=d).manual_seed(0)
    r = lambda *s: torch.randn(*s, device=d, generator=g)
    df, h3, f, de = r(B, 512), r(B, 3136), r(B, 512), r(B, 512)
    Wfc, We, b = r(512, 3136), r(512, 512), r(512)
    gW, gWe = torch.zeros(512, 3136, device=d), torch.zeros(512, 512, device=d)
    ops = {
        "fc_wgrad": lambda: gW.addmm_(df.t(), h3),
        "fc_fwd": lambda: torch.addmm(b, h3, Wfc.t()),
        "extra_fwd": lambda: torch.addmm(b, f, We.t()),
        "extra_wgrad": lambda: gWe.addmm_(de.t(), f),
        "extra_dgrad": lambda: df.addmm_(de, We),
    }
    res = {"B": B}
    for lib in ("default", "cublaslt"):
        try:
            torch.backends.cuda.preferred_blas_library(lib)
        except Exception as ex:  # noqa: BLE001
            res[lib] = str(ex)
            continue
        for k, fn in ops.items():
            res[f"{lib}:{k}"] = round(t_ms(fn), 4)
    torch.backends.cuda.preferred_blas_library("default")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
