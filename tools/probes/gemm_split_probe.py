"""Time the extra-layer weight gradient dW = de^T f (512 x 512 over B rows) as one library
GEMM vs split-K batched GEMMs + an ordered sum (dev probe)."""
import json
import sys

import torch


def timeit(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


for B in [int(x) for x in sys.argv[1:]] or [2048, 16384]:
    de = torch.randn(B, 512, device="cuda")
    f = torch.randn(B, 512, device="cuda")
    out = torch.empty(512, 512, device="cuda")
    res = {"B": B, "mm_us": timeit(lambda: torch.mm(de.t(), f, out=out))}
    ref = (de.double().t() @ f.double())
    for S in (2, 4, 8, 16, 32):
        if B % S:
            continue
        part = torch.empty(S, 512, 512, device="cuda")

        def run():
            torch.bmm(de.view(S, B // S, 512).transpose(1, 2), f.view(S, B // S, 512), out=part)
            torch.sum(part, 0, out=out)
        res[f"split{S}_us"] = timeit(run)
        run()
        res[f"split{S}_err"] = float((out.double() - ref).abs().max() / ref.abs().max())
    torch.mm(de.t(), f, out=out)
    res["mm_err"] = float((out.double() - ref).abs().max() / ref.abs().max())
    print(json.dumps(res))
