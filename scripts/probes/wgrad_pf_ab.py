"""Halo weight-gradient kernels (ResNet-18 3x3 stride-1 shapes, 8 peers x batch 128, random
operands): prefetch depth 1 vs 2 (conv_set_wgrad_pf) at several split counts, alternating arms, and
the two arms' gradients compared (same per-split sums; the split-K atomics' order differs)."""
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


for name, c_, h, splits_list in [("l1", 64, 32, (16, 24, 32, 48, 64)), ("l2", 128, 16, (2, 4, 8, 16)), ("l3", 256, 8, (1, 2, 4, 8)), ("l4", 512, 4, (1, 2, 4))]:
    torch.manual_seed(0)
    x = torch.randn(P, B * h * h * c_, device=dev).to(torch.bfloat16)
    dy = torch.randn(P, B * h * h * c_, device=dev).to(torch.bfloat16)
    ncol = 9 * c_
    M = B * h * h
    flops = 2.0 * P * M * c_ * ncol
    for want in splits_list:
        k_per = max(64, ((M + want - 1) // want + 63) // 64 * 64)
        splits = (M + k_per - 1) // k_per
        grads, times = {}, {1: [], 2: []}
        for pf in (1, 2):
            grads[pf] = torch.zeros(P, c_ * ncol, device=dev)
        args = {}
        for pf in (1, 2):
            a = WgradArgs()
            a.dy, a.dy_ps, a.x, a.x_ps = dy.data_ptr(), dy.shape[1], x.data_ptr(), x.shape[1]
            a.H, a.W, a.x_c, a.Ho, a.Wo, a.dy_c = h, h, c_, h, h, c_
            a.R, a.S, a.stride, a.pad = 3, 3, 1, 1
            a.grad, a.grad_ps, a.accumulate, a.k_per_split, a.max_batch = grads[pf].data_ptr(), grads[pf].shape[1], int(splits > 1), k_per, B
            args[pf] = a
        for pf in (1, 2):  # correctness: one launch into a zeroed gradient
            lib.conv_set_wgrad_pf(pf)
            assert lib.conv_wgrad_launch(ctypes.byref(args[pf]), P, splits, s) == 0
        torch.cuda.synchronize()
        rel = float((grads[1] - grads[2]).abs().max() / grads[1].abs().max())
        for rep in range(3):
            for pf in ((1, 2) if rep % 2 == 0 else (2, 1)):
                lib.conv_set_wgrad_pf(pf)
                times[pf].append(timeit(lambda: lib.conv_wgrad_launch(ctypes.byref(args[pf]), P, splits, s)))
        t1, t2 = min(times[1]), min(times[2])
        print(f"{name} C={c_:3d} splits {splits:3d} ksteps {k_per // 64:4d}: PF1 {t1:7.1f} us ({flops / t1 / 1e6:6.1f} TF/s)  PF2 {t2:7.1f} us "
              f"({flops / t2 / 1e6:6.1f} TF/s)  {100 * (t1 / t2 - 1):+5.1f} %  max rel diff {rel:.2e}", flush=True)
lib.conv_set_wgrad_pf(2)
