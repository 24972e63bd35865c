"""One-off GPU probe: library (MIOpen/rocBLAS) fp32 speeds for the NatureCNN
shapes and a GAE size sweep.  Informs kernel design; not part of the product."""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-exploration_amd"))


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
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
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    dev = "cuda"
    print(torch.cuda.get_device_name(), torch.cuda.get_device_properties(0).multi_processor_count, flush=True)
    # GEMM fp32
    for m, n, k in [(8192, 8192, 8192), (16384, 512, 3136), (16384, 3136, 512), (3136, 512, 16384)]:
        a = torch.randn(m, k, device=dev)
        b = torch.randn(k, n, device=dev)
        ms = timeit(lambda: a @ b)
        print(f"mm {m}x{n}x{k}: {ms:.3f} ms {2*m*n*k/ms/1e9:.1f} TF/s", flush=True)
    # NatureCNN convs with MIOpen
    for B in (4096, 16384):
        x = torch.randint(0, 256, (B, 4, 84, 84), device=dev, dtype=torch.uint8).float()
        w1 = torch.randn(32, 4, 8, 8, device=dev, requires_grad=True)
        w2 = torch.randn(64, 32, 4, 4, device=dev, requires_grad=True)
        w3 = torch.randn(64, 64, 3, 3, device=dev, requires_grad=True)

        def fwd():
            h = F.relu(F.conv2d(x, w1, stride=4))
            h = F.relu(F.conv2d(h, w2, stride=2))
            return F.relu(F.conv2d(h, w3, stride=1))
        with torch.no_grad():
            ms = timeit(fwd, iters=5)
        fl = B * 2 * (400 * 256 * 32 + 81 * 512 * 64 + 49 * 576 * 64)
        print(f"conv fwd B={B}: {ms:.2f} ms {fl/ms/1e9:.1f} TF/s", flush=True)

        def fb():
            y = fwd()
            y.sum().backward()
        ms = timeit(fb, iters=5)
        print(f"conv fwd+bwd B={B}: {ms:.2f} ms ({3*fl/ms/1e9:.1f} TF/s nominal)", flush=True)
    # GAE sweep through the C ABI
    import native
    for T, N in [(128, 4096), (128, 65536), (128, 1 << 20), (128, 1 << 22)]:
        r = torch.randn(T, N, device=dev)
        v = torch.randn(T, N, device=dev)
        d = (torch.rand(T, N, device=dev) < 0.01).to(torch.uint8)
        lv = torch.randn(N, device=dev)
        ld = d[-1].contiguous()
        a = torch.empty_like(r)
        rt = torch.empty_like(r)
        ms = timeit(lambda: native.gae(r, v, d, lv, ld, 0.99, 0.95, a, rt), iters=20)
        gb = 17 * T * N / 1e9
        print(f"gae T={T} N={N}: {ms*1e3:.1f} us  {gb/ms*1e3:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
