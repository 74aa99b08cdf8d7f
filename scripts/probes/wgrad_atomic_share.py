"""Halo weight-gradient kernels (ResNet-18 3x3 stride-1 shapes, 8 peers x batch 128): time per split
count with the fp32 atomic reduction (accumulate=1) and with plain stores (accumulate=0: a wrong
result, timing only) — the share of the split-K atomics in each launch."""
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


for name, c_, h in [("l1", 64, 32), ("l2", 128, 16), ("l3", 256, 8), ("l4", 512, 4)]:
    x = torch.randn(P, B * h * h * c_, device=dev).to(torch.bfloat16)
    dy = torch.randn(P, B * h * h * c_, device=dev).to(torch.bfloat16)
    ncol = 9 * c_
    grad = torch.zeros(P, c_ * ncol, device=dev)
    M = B * h * h
    flops = 2.0 * P * M * c_ * ncol
    for want in (8, 16, 24, 32, 48, 64):
        k_per = max(64, ((M + want - 1) // want + 63) // 64 * 64)
        splits = (M + k_per - 1) // k_per
        row = []
        for acc in (1, 0):
            a = WgradArgs()
            a.dy, a.dy_ps, a.x, a.x_ps = dy.data_ptr(), dy.shape[1], x.data_ptr(), x.shape[1]
            a.H, a.W, a.x_c, a.Ho, a.Wo, a.dy_c = h, h, c_, h, h, c_
            a.R, a.S, a.stride, a.pad = 3, 3, 1, 1
            a.grad, a.grad_ps, a.accumulate, a.k_per_split, a.max_batch = grad.data_ptr(), grad.shape[1], acc, k_per, B
            us = timeit(lambda: lib.conv_wgrad_launch(ctypes.byref(a), P, splits, s))
            row.append(us)
        print(f"{name} C={c_:3d} splits {splits:3d} ksteps {k_per // 64:4d}: atomics {row[0]:7.1f} us ({flops / row[0] / 1e6:6.1f} TF/s)  "
              f"plain {row[1]:7.1f} us ({flops / row[1] / 1e6:6.1f} TF/s)", flush=True)
