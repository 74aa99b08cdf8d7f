"""Debug the wgrad kernel on the GPU: compare with torch for tiny shapes, print error structure."""
import ctypes
import sys
import os
sys.path.insert(0, os.getcwd())
import torch, torch.nn.functional as F
from myfyp_amd.parallel.cnn_engine import WgradArgs, _lib

lib = _lib()
dev = torch.device("cuda")
def run(n, cin, cout, k, stride, pad, h, kps=64, pattern=None):
    torch.manual_seed(0)
    cpi, cpo = (cin + 7) // 8 * 8, (cout + 7) // 8 * 8
    x = torch.randn(n, cin, h, h, device=dev).bfloat16().float()
    w = torch.randn(cout, cin, k, k, device=dev)
    y = F.conv2d(x, w, stride=stride, padding=pad); ho = y.shape[2]
    dy = torch.randn_like(y).bfloat16().float()
    if pattern == "ones":
        x = torch.ones_like(x); dy = torch.ones_like(dy)
    ref = torch.nn.grad.conv2d_weight(x, w.shape, dy, stride=stride, padding=pad)
    xn = torch.zeros(n, h, h, cpi, device=dev, dtype=torch.bfloat16); xn[..., :cin] = x.permute(0, 2, 3, 1).bfloat16()
    dyn = torch.zeros(n, ho, ho, cpo, device=dev, dtype=torch.bfloat16); dyn[..., :cout] = dy.permute(0, 2, 3, 1).bfloat16()
    grad = torch.zeros(cout * cin * k * k, device=dev)
    c = WgradArgs()
    c.dy, c.x = dyn.data_ptr(), xn.data_ptr()
    c.H, c.W, c.x_c, c.Ho, c.Wo, c.dy_c = h, h, cpi, ho, ho, cpo
    c.R, c.S, c.stride, c.pad, c.cout, c.cin = k, k, stride, pad, cout, cin
    c.grad, c.k_per_split, c.max_batch = grad.data_ptr(), kps, n
    M = n * ho * ho
    rc = lib.conv_wgrad_launch(ctypes.byref(c), 1, (M + kps - 1) // kps, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    g = grad.view(cout, cin, k, k)
    err = float((g - ref).norm() / ref.norm())
    print(f"n{n} cin{cin} cout{cout} k{k} s{stride} p{pad} h{h} rc={rc} relerr={err:.4f}")
    if err > 0.05:
        print(" ref[0,:, :, :].flatten()[:12]", ref[0].flatten()[:12].tolist())
        print(" got[0,:, :, :].flatten()[:12]", g[0].flatten()[:12].tolist())
        print(" ref[:8,0,0,0]", ref[:8, 0, 0, 0].tolist())
        print(" got[:8,0,0,0]", g[:8, 0, 0, 0].tolist())
        print(" ratio sum", float(g.sum() / ref.sum()))
    return err
run(1, 8, 64, 1, 1, 0, 4, pattern="ones")
run(1, 8, 64, 1, 1, 0, 8)
run(1, 8, 16, 1, 1, 0, 8)
run(1, 64, 64, 1, 1, 0, 8)
run(1, 128, 128, 1, 1, 0, 8)
run(1, 3, 64, 3, 1, 1, 8)
run(4, 3, 64, 3, 1, 1, 32, kps=128)
