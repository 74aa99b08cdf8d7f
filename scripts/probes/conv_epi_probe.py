"""Epilogue cost of the engine's forward-shaped convs (ResNet-18 layer-1 / layer-3 shapes, 8 peers, batch 128):
plain store vs BN statistics (forward) and vs the BN-backward epilogue (stride-1 dgrad as a forward conv: ReLU mask +
one / two BatchNorm inputs); plus the weight-gradient split-K factor on every shape."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from myfyp_amd.parallel.cnn_engine import ConvGemmArgs, WgradArgs, _lib

lib = _lib()
P, B = 8, 128
dev = torch.device("cuda")


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


s = torch.cuda.current_stream().cuda_stream
for name, c, h in (("l1 64", 64, 32), ("l3 256", 256, 8)):
    x = torch.randn(P, B * h * h * c, device=dev).to(torch.bfloat16)
    wf = (torch.randn(P, c * 9 * c, device=dev) * 0.05).to(torch.bfloat16)
    y = torch.empty_like(x)
    ys = [torch.randn_like(x) for _ in range(2)]
    mask = torch.randn_like(x)
    rows = lib.conv_gemm_stats_rows(B, h, h)
    nr = lib.conv_bnb_rows()
    stats = torch.zeros(P, rows * 2 * c, device=dev)
    ms = torch.stack([torch.zeros(P, c, device=dev), torch.ones(P, c, device=dev)], 1).reshape(P, 2 * c).contiguous()
    parts = [torch.zeros(P, nr * 2 * c, device=dev) for _ in range(2)]
    for mode, epi in ((0, "plain"), (0, "stats"), (4, "plain"), (4, "bnb1"), (4, "bnb2")):
        a = ConvGemmArgs()
        a.src, a.src_ps, a.src_h, a.src_w, a.src_c = x.data_ptr(), x.shape[1], h, h, c
        a.out_h, a.out_w, a.ncol, a.ncol_valid = h, h, c, c
        a.out, a.out_ps = y.data_ptr(), y.shape[1]
        a.R = a.S = 3
        a.stride, a.pad = 1, 1
        a.wt, a.wt_ps, a.max_batch = wf.data_ptr(), wf.shape[1], B
        if epi == "stats":
            a.stats, a.stats_ps, a.stats_rows = stats.data_ptr(), stats.shape[1], rows
        if epi.startswith("bnb"):
            a.bnb_mask, a.bnb_mask_ps, a.bnb_rows = mask.data_ptr(), mask.shape[1], nr
            a.bnb_y0, a.bnb_y0_ps, a.bnb_ms0, a.bnb_part0, a.bnb_part_ps = ys[0].data_ptr(), x.shape[1], ms.data_ptr(), parts[0].data_ptr(), parts[0].shape[1]
            if epi == "bnb2":
                a.bnb_y1, a.bnb_y1_ps, a.bnb_ms1, a.bnb_part1 = ys[1].data_ptr(), x.shape[1], ms.data_ptr(), parts[1].data_ptr()
        us = timeit(lambda: lib.conv_gemm_launch(mode, ctypes.byref(a), P, s))
        print(f"{name:8s} mode {mode} {epi:6s}: {us:8.1f} us", flush=True)

# weight gradient split-K factor (the engine: MYFYP_WGRAD_TPC = 2 -> splits below x1)
for name, cin, cout, hh, st in (("l1 64", 64, 64, 32, 1), ("l2 128", 128, 128, 16, 1), ("l3 256", 256, 256, 8, 1), ("l4 512", 512, 512, 4, 1)):
    x = torch.randn(P, B * hh * hh * cin, device=dev).to(torch.bfloat16)
    dy = torch.randn(P, B * hh * hh * cout, device=dev).to(torch.bfloat16)
    ncol = 9 * cin
    grad = torch.zeros(P, cout * ncol, device=dev)
    M = B * hh * hh
    tiles = ((cout + 127) // 128) * ((ncol + 127) // 128)
    base = max(1, (2 * 256) // max(1, tiles * P))
    for mult in (1, 2, 3):
        want = base * mult
        k_per = max(64, ((M + want - 1) // want + 63) // 64 * 64)
        splits = (M + k_per - 1) // k_per
        cw = WgradArgs()
        cw.dy, cw.dy_ps, cw.x, cw.x_ps = dy.data_ptr(), dy.shape[1], x.data_ptr(), x.shape[1]
        cw.H, cw.W, cw.x_c, cw.Ho, cw.Wo, cw.dy_c = hh, hh, cin, hh, hh, cout
        cw.R, cw.S, cw.stride, cw.pad = 3, 3, st, 1
        cw.grad, cw.grad_ps, cw.accumulate, cw.k_per_split, cw.max_batch = grad.data_ptr(), grad.shape[1], int(splits > 1), k_per, B
        us = timeit(lambda: lib.conv_wgrad_launch(ctypes.byref(cw), P, splits, s))
        print(f"{name:8s} wgrad splits {splits:2d} (x{mult}): {us:8.1f} us", flush=True)
