"""Time the conv GEMM (forward / dgrad) on ResNet-18 CIFAR shapes, 8 peers, batch 128 (TF/s per shape);
forward-shaped modes 0 / 4 through the LDS-DMA kernel (dma) and the register-staged one (reg)."""
import ctypes
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from myfyp_amd.parallel.cnn_engine import ConvGemmArgs, _lib

lib = _lib()
P, B = 8, 128
dev = torch.device("cuda")
shapes = [("l1 3x3 64", 64, 64, 32, 1), ("l2 3x3 128", 128, 128, 16, 1), ("l3 3x3 256", 256, 256, 8, 1), ("l4 3x3 512", 512, 512, 4, 1),
          ("l2.c1 s2 64->128", 64, 128, 32, 2)]
for name, cin, cout, h, st in shapes:
    ho = (h + 2 - 3) // st + 1
    x = torch.randn(P, B * h * h * cin, device=dev).to(torch.bfloat16)
    wf = (torch.randn(P, cout * 9 * cin, device=dev) * 0.05).to(torch.bfloat16)
    y = torch.empty(P, B * ho * ho * cout, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(P, B * ho * ho * cout, device=dev).to(torch.bfloat16)
    dx = torch.empty(P, B * h * h * cin, device=dev, dtype=torch.bfloat16)
    flops = 2 * P * B * ho * ho * cout * 9 * cin
    wt = torch.empty_like(wf)
    # conv_set_dma variant codes: 0 register stage; narrow (64 channels) 3 / 5 / 7 = 128x64 3 stages 2 per CU /
    # 128x64 2 stages 3 per CU / 256x64 3 stages 1 per CU; wide 9 / 17 = 256x128 3 stages / 128x128 2 stages 2 per CU
    VARIANTS = {3: "128x64/3", 5: "128x64/2", 7: "256x64/3", 9: "256x128/3", 17: "128x128/2", 0: "reg", 1: "default"}
    for mode in (0, 1, 4, 5):
        if (mode == 4 and st != 1) or (mode == 5 and st != 2):
            continue
        narrow = (cout if mode == 0 else cin) <= 64
        codes = [0] if mode == 1 else ([1] if mode == 5 else ([0, 3, 5, 7] if narrow else [0, 9, 17]))
        for dma in codes:
            lib.conv_set_dma(dma)
            a = ConvGemmArgs()
            if mode == 0:
                a.src, a.src_ps, a.src_h, a.src_w, a.src_c = x.data_ptr(), x.shape[1], h, h, cin
                a.out_h, a.out_w, a.ncol, a.ncol_valid = ho, ho, cout, cout
                a.out, a.out_ps = y.data_ptr(), y.shape[1]
            else:
                a.src, a.src_ps, a.src_h, a.src_w, a.src_c = dy.data_ptr(), dy.shape[1], ho, ho, cout
                a.out_h, a.out_w, a.ncol, a.ncol_valid = h, h, cin, cin
                a.out, a.out_ps = dx.data_ptr(), dx.shape[1]
            a.R = a.S = 3
            a.stride, a.pad = st, 1
            a.wt, a.wt_ps, a.max_batch = wf.data_ptr(), wf.shape[1], B
            s = torch.cuda.current_stream().cuda_stream
            if mode in (4, 5):  # dgrad as forward conv(s) over dY: flipped weights (timed with the conv)
                a.src, a.src_ps, a.src_h, a.src_w, a.src_c = dy.data_ptr(), dy.shape[1], ho, ho, cout
                a.out_h, a.out_w, a.ncol, a.ncol_valid = h, h, cin, cin
                a.out, a.out_ps = dx.data_ptr(), dx.shape[1]
                a.wt, a.pad = wt.data_ptr(), (1 if mode == 4 else 1)

            def launch():
                if mode == 4:
                    assert lib.conv_wt_flip_launch(wf.data_ptr(), wf.shape[1], wt.data_ptr(), wt.shape[1], cout, cin, 3, 3, P, s) == 0
                if mode == 5:
                    assert lib.conv_wt_flip_parity_launch(wf.data_ptr(), wf.shape[1], wt.data_ptr(), wt.shape[1], cout, cin, 3, 3, 1, P, s) == 0
                assert lib.conv_gemm_launch(mode, ctypes.byref(a), P, s) == 0

            for _ in range(3):
                launch()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                launch()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 20 * 1000
            useful = flops if mode == 0 or st == 1 else flops  # dgrad useful work = forward FLOPs
            print(f"{name:18s} mode {mode} {VARIANTS[dma]:10s}: {us:8.1f} us ({useful / us / 1e6:6.0f} TF/s useful)", flush=True)

# weight gradients: register stage (0) vs LDS-DMA ring with 2 (32) / 3 (64) stages, split-K as the
# engine sizes it (MYFYP_WGRAD_TPC = 2 workgroups per CU over all peers)
from myfyp_amd.parallel.cnn_engine import WgradArgs

for name, cin, cout, h, st in shapes:
    ho = (h + 2 - 3) // st + 1
    x = torch.randn(P, B * h * h * cin, device=dev).to(torch.bfloat16)
    dy = torch.randn(P, B * ho * ho * cout, device=dev).to(torch.bfloat16)
    ncol = 9 * cin
    grad = torch.zeros(P, cout * ncol, device=dev)
    M = B * ho * ho
    tiles = ((cout + 127) // 128) * ((ncol + 127) // 128)
    want = max(1, (2 * 256) // max(1, tiles * P))
    k_per = max(64, ((M + want - 1) // want + 63) // 64 * 64)
    splits = (M + k_per - 1) // k_per
    flops = 2 * P * M * cout * ncol
    for code, lab in ((0, "reg"), (32, "dma/2"), (64, "dma/3")):
        lib.conv_set_dma(code)
        c = WgradArgs()
        c.dy, c.dy_ps, c.x, c.x_ps = dy.data_ptr(), dy.shape[1], x.data_ptr(), x.shape[1]
        c.H, c.W, c.x_c, c.Ho, c.Wo, c.dy_c = h, h, cin, ho, ho, cout
        c.R, c.S, c.stride, c.pad = 3, 3, st, 1
        c.grad, c.grad_ps, c.accumulate, c.k_per_split, c.max_batch = grad.data_ptr(), grad.shape[1], int(splits > 1), k_per, B
        s = torch.cuda.current_stream().cuda_stream

        def launch():
            assert lib.conv_wgrad_launch(ctypes.byref(c), P, splits, s) == 0

        for _ in range(3):
            launch()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            launch()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1000
        print(f"{name:18s} wgrad {lab:6s} (splits {splits:2d}): {us:8.1f} us ({flops / us / 1e6:6.0f} TF/s)", flush=True)
lib.conv_set_dma(1)
