"""Weight-gradient split-K sweep on the ResNet-18 CIFAR wgrad shapes (8 peers, batch 128): time per split
count, with the workgroup count and the K steps (64 pixels) per workgroup, to pick the engine's split rule."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from myfyp_amd.parallel.cnn_engine import WgradArgs, _lib

lib = _lib()
P, B = 8, 128
dev = torch.device("cuda")
s = torch.cuda.current_stream().cuda_stream


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1000


# (name, cin, cout, input h, stride, kernel)
shapes = [("l1 3x3 64", 64, 64, 32, 1, 3), ("l2 3x3 128", 128, 128, 16, 1, 3), ("l3 3x3 256", 256, 256, 8, 1, 3), ("l4 3x3 512", 512, 512, 4, 1, 3),
          ("l2.c1 s2 64->128", 64, 128, 32, 2, 3), ("l3.c1 s2 128->256", 128, 256, 16, 2, 3), ("l4.c1 s2 256->512", 256, 512, 8, 2, 3),
          ("l2 proj 1x1 s2", 64, 128, 32, 2, 1), ("stem 3(8)->64", 8, 64, 32, 1, 3)]
for name, cin, cout, h, st, k in shapes:
    pad = k // 2
    ho = (h + 2 * pad - k) // st + 1
    x = torch.randn(P, B * h * h * cin, device=dev).to(torch.bfloat16)
    dy = torch.randn(P, B * ho * ho * cout, device=dev).to(torch.bfloat16)
    ncol = k * k * cin
    grad = torch.zeros(P, cout * ncol, device=dev)
    M = B * ho * ho
    bm, bn = (128 if cout > 64 else 64), (128 if ncol > 64 else 64)
    tiles = ((cout + bm - 1) // bm) * ((ncol + bn - 1) // bn)
    seen = set()
    for want in (1, 2, 3, 4, 5, 6, 8, 10, 12, 16, 20, 24, 32, 40, 48, 64):
        k_per = max(64, ((M + want - 1) // want + 63) // 64 * 64)
        splits = (M + k_per - 1) // k_per
        if splits in seen:
            continue
        seen.add(splits)
        c = WgradArgs()
        c.dy, c.dy_ps, c.x, c.x_ps = dy.data_ptr(), dy.shape[1], x.data_ptr(), x.shape[1]
        c.H, c.W, c.x_c, c.Ho, c.Wo, c.dy_c = h, h, cin, ho, ho, cout
        c.R, c.S, c.stride, c.pad = k, k, st, pad
        c.grad, c.grad_ps, c.accumulate, c.k_per_split, c.max_batch = grad.data_ptr(), grad.shape[1], int(splits > 1), k_per, B
        us = timeit(lambda: lib.conv_wgrad_launch(ctypes.byref(c), P, splits, s))
        print(f"{name:20s} tiles/peer {tiles:3d} splits {splits:3d} wgs {tiles * P * splits:5d} ksteps {k_per // 64:4d}: {us:8.1f} us", flush=True)
