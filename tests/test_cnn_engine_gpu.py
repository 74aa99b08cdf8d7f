"""GPU numerics of the CNN engine: implicit-GEMM conv kernels vs torch fp32, and whole LeNet-5 /
ResNet-18 train steps (grouped peers) vs torch autograd + torch.optim.SGD semantics."""

import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _cp(c):
    return (c + 7) // 8 * 8


def _nhwc_pad(x_nchw, cp):
    n, c, h, w = x_nchw.shape
    out = torch.zeros(n, h, w, cp, device=x_nchw.device, dtype=torch.bfloat16)
    out[..., :c] = x_nchw.permute(0, 2, 3, 1).to(torch.bfloat16)
    return out


def _bf(t):
    return t.to(torch.bfloat16).float()


@pytest.fixture(params=[1, -1, 0, 3, 7, 9, 32, 64], ids=["dma", "dma_persist", "regstage", "dma128x64s3", "dma256x64s3", "dma256x128s3", "wgrad2", "wgrad3"])
def conv_dma(request):
    """Forward-shaped convs (mode 0, mode 4) through the LDS-DMA stage-ring kernel (1: the default
    tiles, 128x64 / 128x128 with 2 stages, register-staged wgrad; 3 / 7 / 9: the 3-stage forward
    variants, 32 / 64: the 2- / 3-stage DMA wgrad, see conv_gemm_launch) or the register-staged
    kernels (0); -1: the default tiles with 3 workgroups per launch, so each runs many M tiles and
    carries its column sums across them; restored afterwards."""
    from myfyp_amd.parallel.cnn_engine import _lib

    lib = _lib()
    old = lib.conv_set_dma(1 if request.param == -1 else request.param)
    old_wgs = lib.conv_set_dma_wgs(3 if request.param == -1 else 0)  # dma_persist: 3 workgroups run every M tile
    old_halo = lib.conv_set_fwd_halo(0 if request.param == 0 else 1)  # regstage: the register-staged kernel everywhere
    yield request.param
    lib.conv_set_dma(old)
    lib.conv_set_dma_wgs(old_wgs)
    lib.conv_set_fwd_halo(old_halo)


@pytest.mark.parametrize("cin,cout,k,stride,pad,h,n", [(3, 64, 3, 1, 1, 32, 4), (64, 128, 3, 2, 1, 16, 3), (64, 128, 1, 2, 0, 16, 2), (6, 16, 5, 1, 0, 14, 5), (256, 512, 3, 2, 1, 8, 2), (16, 24, 3, 2, 1, 7, 2), (8, 16, 1, 2, 0, 9, 3),
                                                     (64, 64, 3, 1, 1, 32, 2), (64, 64, 3, 1, 1, 16, 3), (64, 64, 3, 1, 1, 8, 5), (128, 128, 3, 1, 1, 16, 2),
                                                     (256, 128, 3, 1, 1, 8, 3), (128, 128, 3, 1, 1, 4, 5), (64, 192, 3, 1, 1, 4, 3)])
def test_conv_fwd_dgrad_wgrad_vs_torch(cin, cout, k, stride, pad, h, n, conv_dma):
    from myfyp_amd.parallel.cnn_engine import ConvGemmArgs, WgradArgs, _lib

    lib = _lib()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    x = _bf(torch.randn(n, cin, h, h, device=dev))
    w = _bf(torch.randn(cout, cin, k, k, device=dev) * (1.0 / (cin * k * k) ** 0.5))
    y_ref = F.conv2d(x, w, stride=stride, padding=pad)
    ho = y_ref.shape[2]
    cpi, cpo = _cp(cin), _cp(cout)
    xn = _nhwc_pad(x, cpi).reshape(1, -1).contiguous()
    wf = torch.zeros(cpo, k, k, cpi, device=dev, dtype=torch.bfloat16)
    wf[:cout, :, :, :cin] = w.permute(0, 2, 3, 1).to(torch.bfloat16)
    y = torch.zeros(1, n * ho * ho * cpo, device=dev, dtype=torch.bfloat16)
    srows = lib.conv_gemm_stats_rows(n, ho, ho)  # spread accumulator rows (summed below)
    stats = torch.zeros(1, srows * 2 * cpo, device=dev)
    a = ConvGemmArgs()
    a.src, a.src_ps, a.src_h, a.src_w, a.src_c = xn.data_ptr(), 0, h, h, cpi
    a.out_h, a.out_w, a.R, a.S, a.stride, a.pad = ho, ho, k, k, stride, pad
    a.wt, a.wt_ps, a.ncol, a.ncol_valid = wf.data_ptr(), 0, cpo, cout
    a.out, a.out_ps, a.relu, a.stats, a.stats_ps, a.max_batch = y.data_ptr(), 0, 0, stats.data_ptr(), 0, n
    a.stats_rows = srows
    assert lib.conv_gemm_launch(0, ctypes.byref(a), 1, torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    y_nhwc = y.view(n, ho, ho, cpo)[..., :cout].float()
    ref = y_ref.permute(0, 2, 3, 1)
    torch.testing.assert_close(y_nhwc, ref, atol=2e-2, rtol=2e-2)
    assert y.view(n, ho, ho, cpo)[..., cout:].abs().max().item() == 0 if cpo > cout else True
    st = stats.view(-1, 2, cpo).sum(0)
    torch.testing.assert_close(st[0, :cout], ref.sum((0, 1, 2)), atol=0.5, rtol=2e-2)
    _check_fused_bn_finalize_fwd(lib, a, stats, st, cout, cpo, n * ho * ho)

    # dgrad
    dy = _bf(torch.randn_like(y_ref))
    dx_ref = torch.nn.grad.conv2d_input(x.shape, w, dy, stride=stride, padding=pad)
    dyn = _nhwc_pad(dy, cpo).reshape(1, -1).contiguous()
    dx = torch.zeros(1, n * h * h * cpi, device=dev, dtype=torch.bfloat16)
    b = ConvGemmArgs()
    b.src, b.src_h, b.src_w, b.src_c = dyn.data_ptr(), ho, ho, cpo
    b.out_h, b.out_w, b.R, b.S, b.stride, b.pad = h, h, k, k, stride, pad
    b.wt, b.ncol, b.ncol_valid = wf.data_ptr(), cpi, cin  # dgrad reads the same Wf shadow (transposed LDS reads)
    b.out, b.max_batch = dx.data_ptr(), n
    assert lib.conv_gemm_launch(1, ctypes.byref(b), 1, torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    torch.testing.assert_close(dx.view(n, h, h, cpi)[..., :cin].float(), dx_ref.permute(0, 2, 3, 1), atol=3e-2, rtol=3e-2)
    if stride == 1:  # MODE 4: the same dgrad as a forward conv over dY with flipped, transposed weights
        wt = torch.zeros_like(wf)
        s_ = torch.cuda.current_stream().cuda_stream
        assert lib.conv_wt_flip_launch(wf.data_ptr(), 0, wt.data_ptr(), 0, cpo, cpi, k, k, 1, s_) == 0
        torch.cuda.synchronize()
        assert torch.equal(wt.view(cpi, k, k, cpo), wf.flip(1, 2).permute(3, 1, 2, 0))
        dx4 = torch.zeros_like(dx)
        b.wt, b.pad, b.out = wt.data_ptr(), k - 1 - pad, dx4.data_ptr()
        assert lib.conv_gemm_launch(4, ctypes.byref(b), 1, s_) == 0
        torch.cuda.synchronize()
        torch.testing.assert_close(dx4.view(n, h, h, cpi)[..., :cin].float(), dx_ref.permute(0, 2, 3, 1), atol=3e-2, rtol=3e-2)

    if stride == 2 and conv_dma != 0:  # MODE 5: parity classes as forward convs with class-flipped weights
        wt = torch.zeros_like(wf)
        s_ = torch.cuda.current_stream().cuda_stream
        assert lib.conv_wt_flip_parity_launch(wf.data_ptr(), 0, wt.data_ptr(), 0, cpo, cpi, k, k, pad, 1, s_) == 0
        torch.cuda.synchronize()
        blocks, off = [], 0
        for c in range(4):  # class c = (ph, pw): taps r0 + 2i, flipped, as [ci][tR][tS][co]
            r0, s0 = ((c >> 1) + pad) & 1, ((c & 1) + pad) & 1
            rr, ss = list(range(r0, k, 2))[::-1], list(range(s0, k, 2))[::-1]
            if rr and ss:
                blk = wf[:, rr][:, :, ss].permute(3, 1, 2, 0).reshape(-1)
                blocks.append(blk)
                off += blk.numel()
        assert torch.equal(wt.view(-1)[:off], torch.cat(blocks))
        dx5 = torch.full_like(dx, float("nan"))  # every dX pixel belongs to one class: all are written
        b.wt, b.pad, b.out = wt.data_ptr(), pad, dx5.data_ptr()
        assert lib.conv_gemm_launch(5, ctypes.byref(b), 1, s_) == 0
        torch.cuda.synchronize()
        torch.testing.assert_close(dx5.view(n, h, h, cpi)[..., :cin].float(), dx_ref.permute(0, 2, 3, 1), atol=3e-2, rtol=3e-2)

    # wgrad
    dw_ref = torch.nn.grad.conv2d_weight(x, w.shape, dy, stride=stride, padding=pad)
    M = n * ho * ho
    halo = cin % 64 == 0 and cout % 64 == 0 and k == 3 and stride == 1  # k_conv_wgrad_halo (one X patch per K step)
    for halo_on, k_per in [(1, 128), (1, (M + 63) // 64 * 64)] + ([(0, 128)] if halo else []):  # split-K (atomics) and one split (plain stores)
        old_halo = lib.conv_set_wgrad_halo(halo_on)
        splits = (M + k_per - 1) // k_per
        grad = torch.zeros(1, cpo * k * k * cpi, device=dev)  # Wf layout [cp_out][R][S][cp_in]
        c = WgradArgs()
        c.dy, c.x = dyn.data_ptr(), xn.data_ptr()
        c.H, c.W, c.x_c, c.Ho, c.Wo, c.dy_c = h, h, cpi, ho, ho, cpo
        c.R, c.S, c.stride, c.pad = k, k, stride, pad
        c.grad, c.accumulate, c.k_per_split, c.max_batch = grad.data_ptr(), int(splits > 1), k_per, n
        assert lib.conv_wgrad_launch(ctypes.byref(c), 1, splits, torch.cuda.current_stream().cuda_stream) == 0
        torch.cuda.synchronize()
        lib.conv_set_wgrad_halo(old_halo)
        gw = grad.view(cpo, k, k, cpi)
        g = gw[:cout, :, :, :cin].permute(0, 3, 1, 2)
        err = (g - dw_ref).norm() / dw_ref.norm()
        assert err < 2e-2, (k_per, float(err))
        assert gw[cout:].abs().max().item() == 0 if cpo > cout else True


@pytest.mark.parametrize("cin,cout,stride,h,n,two,mode", [(64, 64, 1, 16, 3, False, 1), (64, 128, 2, 16, 2, True, 1), (128, 128, 1, 8, 4, True, 1),
                                                          (64, 64, 1, 16, 3, False, 4), (128, 128, 1, 8, 4, True, 4), (64, 128, 1, 8, 2, True, 4),
                                                          (64, 128, 2, 16, 2, True, 5), (128, 256, 2, 9, 3, False, 5),
                                                          (64, 64, 1, 32, 2, True, 4), (64, 64, 1, 32, 3, False, 4)])
def test_dgrad_bn_backward_epilogue_vs_torch(cin, cout, stride, h, n, two, mode, conv_dma):
    """dgrad with the BN-backward epilogue: out = bf16(dX + resid) * [mask > 0] and per-channel
    (sum g, sum g*xhat) for one or two BatchNorms, against torch fp32 of the same op. mode 4: the
    stride-1 dgrad as a forward conv over dY with flipped weights (what the engine runs); mode 5: the
    stride-2 dgrad by parity class, each class a forward conv with its flipped taps."""
    from myfyp_amd.parallel.cnn_engine import ConvGemmArgs, _lib

    lib = _lib()
    dev = torch.device("cuda")
    torch.manual_seed(1)
    k, pad = 3, 1
    ho = (h + 2 * pad - k) // stride + 1
    w = _bf(torch.randn(cout, cin, k, k, device=dev) * (1.0 / (cin * k * k) ** 0.5))
    wf = w.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()
    dy = _bf(torch.randn(n, cout, ho, ho, device=dev))
    dx_ref = torch.nn.grad.conv2d_input((n, cin, h, h), w, dy, stride=stride, padding=pad)
    resid = _bf(torch.randn(n, cin, h, h, device=dev))
    mask = _bf(torch.relu(torch.randn(n, cin, h, h, device=dev)))
    ys = [_bf(torch.randn(n, cin, h, h, device=dev) * 2 + 0.5) for _ in range(2 if two else 1)]
    ms = [torch.stack([y.mean((0, 2, 3)), 1.0 / (y.var((0, 2, 3), unbiased=False) + 1e-5).sqrt()]).reshape(1, -1).contiguous() for y in ys]
    nh = lambda t: _nhwc_pad(t, cin).reshape(1, -1).contiguous()
    dyn, rn, mn = _nhwc_pad(dy, cout).reshape(1, -1).contiguous(), nh(resid), nh(mask)
    yn = [nh(y) for y in ys]
    out = torch.zeros(1, n * h * h * cin, device=dev, dtype=torch.bfloat16)
    nr = lib.conv_bnb_rows()  # spread accumulator rows of the BN-backward sums
    parts = [torch.zeros(1, nr * 2 * cin, device=dev) for _ in ys]
    b = ConvGemmArgs()
    b.src, b.src_h, b.src_w, b.src_c = dyn.data_ptr(), ho, ho, cout
    b.out_h, b.out_w, b.R, b.S, b.stride, b.pad = h, h, k, k, stride, pad
    b.wt, b.ncol, b.ncol_valid = wf.data_ptr(), cin, cin
    b.out, b.max_batch = out.data_ptr(), n
    b.resid = rn.data_ptr()
    b.bnb_rows = nr
    b.bnb_mask, b.bnb_y0, b.bnb_ms0, b.bnb_part0 = mn.data_ptr(), yn[0].data_ptr(), ms[0].data_ptr(), parts[0].data_ptr()
    if two:
        b.bnb_y1, b.bnb_ms1, b.bnb_part1 = yn[1].data_ptr(), ms[1].data_ptr(), parts[1].data_ptr()
    if mode == 4:
        wt = torch.zeros_like(wf)
        assert lib.conv_wt_flip_launch(wf.data_ptr(), 0, wt.data_ptr(), 0, cout, cin, k, k, 1, torch.cuda.current_stream().cuda_stream) == 0
        b.wt, b.pad = wt.data_ptr(), k - 1 - pad
    if mode == 5:
        if conv_dma == 0:
            pytest.skip("MODE 5 runs on the LDS-DMA kernel only")
        wt = torch.zeros_like(wf)
        assert lib.conv_wt_flip_parity_launch(wf.data_ptr(), 0, wt.data_ptr(), 0, cout, cin, k, k, pad, 1, torch.cuda.current_stream().cuda_stream) == 0
        b.wt = wt.data_ptr()
    assert lib.conv_gemm_launch(mode, ctypes.byref(b), 1, torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    g_ref = (dx_ref + resid) * (mask > 0)
    g = out.view(n, h, h, cin).float().permute(0, 3, 1, 2)
    torch.testing.assert_close(g, g_ref, atol=3e-2, rtol=3e-2)
    parts = [p_.view(nr, 2 * cin).sum(0, keepdim=True) for p_ in parts]
    for y, m, part in zip(ys, ms, parts):
        xhat = (y - m[0, :cin].view(1, -1, 1, 1)) * m[0, cin:].view(1, -1, 1, 1)
        sg_ref, sgx_ref = g_ref.sum((0, 2, 3)), (g_ref * xhat).sum((0, 2, 3))
        scale = g_ref.abs().sum((0, 2, 3)).max()
        assert (part[0, :cin] - sg_ref).abs().max() < 1e-2 * scale, float((part[0, :cin] - sg_ref).abs().max())
        # the kernel sums the bf16-rounded g it writes, exactly what the BN apply reads back
        gx = (g * xhat).sum((0, 2, 3))
        torch.testing.assert_close(part[0, cin:], gx, atol=1e-2 * float(scale), rtol=1e-3)
        assert (part[0, cin:] - sgx_ref).abs().max() < 2e-2 * scale

    # the same launch with the BN-backward finalize in its last workgroup (conv_fin_tail): apply
    # coefficients and dgamma/dbeta from the sums just checked; rows and counter re-armed
    cnt = torch.zeros(lib.conv_fin_words(), dtype=torch.int32, device=dev)
    parts_raw = [torch.zeros(1, nr * 2 * cin, device=dev) for _ in ys]
    b.bnb_part0 = parts_raw[0].data_ptr()
    if two:
        b.bnb_part1 = parts_raw[1].data_ptr()
    gammas = [torch.rand(cin, device=dev) + 0.5 for _ in ys]
    dgb = [torch.full((2, cin), 0.25, device=dev) for _ in ys]  # accumulated into (+=)
    coefs = [torch.full((3 * cin,), float("nan"), device=dev) for _ in ys]
    b.fin_cnt, b.fin_param_ps = cnt.data_ptr(), 0
    for i in range(len(ys)):
        setattr(b, f"fin_gamma{i}", gammas[i].data_ptr())
        setattr(b, f"fin_dgamma{i}", dgb[i][0].data_ptr())
        setattr(b, f"fin_dbeta{i}", dgb[i][1].data_ptr())
        setattr(b, f"fin_coef{i}", coefs[i].data_ptr())
        setattr(b, f"fin_C{i}", cin)
    assert lib.conv_gemm_launch(mode, ctypes.byref(b), 1, torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    assert int(cnt.abs().max()) == 0 and all(float(p_.abs().max()) == 0.0 for p_ in parts_raw)
    cntf = float(n * h * h)
    for m, part, gm, d, cf in zip(ms, parts, gammas, dgb, coefs):
        sg, sgx = part[0, :cin], part[0, cin:]
        tol = dict(atol=1e-3 * float(sg.abs().max() + sgx.abs().max() + 1), rtol=1e-3)
        torch.testing.assert_close(d[0], sgx + 0.25, **tol)
        torch.testing.assert_close(d[1], sg + 0.25, **tol)
        torch.testing.assert_close(cf[:cin], gm * m[0, cin:], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(cf[cin:2 * cin], sg / cntf, atol=tol["atol"] / cntf, rtol=1e-3)
        torch.testing.assert_close(cf[2 * cin:], sgx / cntf, atol=tol["atol"] / cntf, rtol=1e-3)


def _check_fused_bn_finalize_fwd(lib, a, stats, st, cout, cpo, count):
    """Re-run forward launch ``a`` with the BatchNorm finalize in its last workgroup
    (conv_fin_tail): scale/shift, mean/inv and the running statistics from the statistics ``st``
    the separate launch produced; the accumulator rows and the arrival counter end re-armed."""
    dev = stats.device
    cnt = torch.zeros(lib.conv_fin_words(), dtype=torch.int32, device=dev)
    gamma, beta = torch.rand(cpo, device=dev) + 0.5, torch.randn(cpo, device=dev)
    rmean, rvar = torch.full((cpo,), 0.5, device=dev), torch.full((cpo,), 2.0, device=dev)
    ss, msb = torch.full((2 * cpo,), float("nan"), device=dev), torch.full((2 * cpo,), float("nan"), device=dev)
    stats.zero_()
    a.fin_cnt, a.fin_gamma0, a.fin_beta, a.fin_param_ps = cnt.data_ptr(), gamma.data_ptr(), beta.data_ptr(), 0
    a.fin_rmean, a.fin_rvar, a.fin_run_ps, a.fin_ss, a.fin_ms = rmean.data_ptr(), rvar.data_ptr(), 0, ss.data_ptr(), msb.data_ptr()
    a.fin_C0, a.fin_train, a.fin_eps, a.fin_momentum = cout, 1, 1e-5, 0.1
    assert lib.conv_gemm_launch(0, ctypes.byref(a), 1, torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    a.fin_cnt = None
    assert int(cnt.abs().max()) == 0 and float(stats.abs().max()) == 0.0
    mean = st[0, :cout] / count
    var = (st[1, :cout] / count - mean * mean).clamp_min(0)
    inv = (var + 1e-5).rsqrt()
    tol = dict(rtol=2e-3, atol=2e-3)
    torch.testing.assert_close(msb[:cout], mean, **tol)
    torch.testing.assert_close(msb[cpo:cpo + cout], inv, **tol)
    torch.testing.assert_close(ss[:cout], gamma[:cout] * inv, **tol)
    torch.testing.assert_close(ss[cpo:cpo + cout], beta[:cout] - mean * gamma[:cout] * inv, **tol)
    torch.testing.assert_close(rmean[:cout], 0.45 + 0.1 * mean, **tol)
    torch.testing.assert_close(rvar[:cout], 1.8 + 0.1 * var * count / max(1, count - 1), **tol)
    if cpo > cout:  # padding channels: zero constants, running statistics untouched
        assert float(ss[cout:cpo].abs().max()) == 0.0 and float(msb[cout:cpo].abs().max()) == 0.0
        assert float((rmean[cout:] - 0.5).abs().max()) == 0.0


def _make_learners(model_fn, n_peers, n_train, n_test, batch, lr, momentum=0.0, wd=0.0):
    from myfyp_amd.learning.dataset.synthetic import synthetic_cifar10
    from myfyp_amd.learning.frameworks.torch import TorchModel
    from myfyp_amd.learning.frameworks.torch.torch_learner import TorchLearner
    from myfyp_amd.parallel.cnn_engine import CNNGroup
    from myfyp_amd.settings import Settings

    CNNGroup.reset_all()
    Settings.USE_FUSED_KERNELS = True
    data = synthetic_cifar10(n_train * n_peers, n_test * n_peers, seed=3)
    from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy

    parts = data.generate_partitions(n_peers, RandomIIDPartitionStrategy)
    learners, refs = [], []
    for i in range(n_peers):
        m = model_fn(i)
        m.optimizer_spec = lambda lr=lr, momentum=momentum, wd=wd: {"name": "sgd", "lr": lr, "momentum": momentum, "weight_decay": wd}
        ref = model_fn(i).cuda()
        lr_ = TorchLearner(TorchModel(m), parts[i], f"cnn-{i}", batch_size=batch, device="cuda")
        assert lr_._engine is not None, "CNN engine not attached"
        lr_.set_epochs(1)
        learners.append(lr_)
        refs.append(ref)
    return learners, refs, parts


def _torch_step(ref, x_u8, y, lr, momentum, wd, bf16=False):
    ref.train()
    opt = torch.optim.SGD(ref.parameters(), lr=lr, momentum=momentum, weight_decay=wd)
    opt.zero_grad()
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
        loss = F.cross_entropy(ref(x_u8).float(), y)
    loss.backward()
    opt.step()
    return float(loss.detach())


def _run_one_step(model_fn, n_peers, batch, lr, momentum=0.0, wd=0.0):
    """One grouped engine step vs torch fp32. The tolerance per parameter is set by how far torch's
    own bf16-autocast step is from fp32 (max(0.05, 2.5 x that floor); deep nets: the floor is large)."""
    import threading

    learners, refs, parts = _make_learners(model_fn, n_peers, batch, 64, batch, lr, momentum, wd)
    floors = [None] * n_peers
    for i in range(n_peers):
        r16 = model_fn(i).cuda()
        p0 = [p.detach().clone() for p in r16.parameters()]
        x, y = learners[i].device_data(True)
        _torch_step(r16, x[:batch], y[:batch], lr, momentum, wd, bf16=True)
        floors[i] = {n: (p.detach() - q).flatten() for (n, p), q in zip(r16.named_parameters(), p0)}
    g = learners[0]._engine.group
    g.perm_fn = lambda ep: torch.arange(g.nmax, dtype=torch.int32, device="cuda").unsqueeze(0).repeat(g.capacity, 1)
    before = [[p.detach().clone() for p in r.parameters()] for r in refs]
    out = [None] * n_peers
    ths = [threading.Thread(target=lambda i=i: out.__setitem__(i, learners[i].fit())) for i in range(n_peers)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    for i, (lr_, ref) in enumerate(zip(learners, refs)):
        x, y = lr_.device_data(True)
        _torch_step(ref, x[:batch], y[:batch], lr, momentum, wd)
        eng = dict(lr_.model.get_model().named_parameters())
        num = num16 = den = 0.0  # the update scale over every layer with >= 256 elements
        for (name, p_ref), p0 in zip(ref.named_parameters(), before[i]):
            d_ref = (p_ref.detach() - p0).flatten()
            d_eng = (eng[name].detach() - p0).flatten()
            if d_ref.norm() < 1e-8:
                continue
            cos = F.cosine_similarity(d_ref, d_eng, dim=0)
            rel = (d_ref - d_eng).norm() / d_ref.norm()
            rel16 = float((d_ref - floors[i][name]).norm() / d_ref.norm())
            # the engine rounds to bf16 at other points than autocast (operands per MFMA tile, fp32
            # epilogues), so its error is of the floor's size but not the same draw
            assert rel < max(0.05, 2.5 * rel16), (name, float(rel), float(cos), rel16)
            if d_ref.numel() >= 256:
                # the update's scale along torch's direction: rounding noise is unbiased, so this
                # stays near 1 even where the deep-net floor is large; a wrong step size does not
                # (a 5 % learning-rate error was caught here and by nothing else in this file,
                # profiles/r5_mutation). Per layer only a gross error (a small BN layer's ratio
                # strays ~6 % from run to run: split-K atomics); the tight bound is on the sum
                dr = torch.dot(d_ref.double(), d_ref.double())
                de, d16 = torch.dot(d_eng.double(), d_ref.double()), torch.dot(floors[i][name].double(), d_ref.double())
                ratio, ratio16 = float(de / dr), float(d16 / dr)
                assert abs(ratio - 1.0) < max(0.1, 4.0 * abs(ratio16 - 1.0)), (name, ratio, ratio16)
                num, num16, den = num + float(de), num16 + float(d16), den + float(dr)
        if den > 0:
            ratio, ratio16 = num / den, num16 / den
            assert abs(ratio - 1.0) < max(0.02, 3.0 * abs(ratio16 - 1.0)), ("all layers", ratio, ratio16)
        # BN running statistics follow torch
        for (name, b_ref) in ref.named_buffers():
            if "running" in name:
                b_eng = dict(lr_.model.get_model().named_buffers())[name]
                torch.testing.assert_close(b_eng.float(), b_ref.float(), atol=5e-2, rtol=5e-2)
    return learners, refs


@pytest.mark.parametrize("fused", ["1", "0"])
def test_lenet_train_step_matches_torch(fused, monkeypatch):
    """fused = the one-kernel LeNet step (lenet_fused.hip); 0 = the layer-by-layer conv kernels.
    Tolerance: the bf16 noise floor (torch's own bf16-autocast step vs fp32), not a fixed bound."""
    from myfyp_amd.models import LeNet5

    monkeypatch.setenv("MYFYP_LENET_FUSED", fused)
    learners, _ = _run_one_step(lambda i: LeNet5(seed=10 + i), n_peers=2, batch=32, lr=0.05, momentum=0.9)
    assert learners[0]._engine.group.lenet_fused == (fused == "1")


def _torch_fit(ref, batches, lr, momentum, wd, bf16):
    """One fit of the reference: a FRESH torch.optim.SGD (the engine also starts every fit with zero
    momentum), one step per batch in order; returns the mean training loss."""
    ref.train()
    opt = torch.optim.SGD(ref.parameters(), lr=lr, momentum=momentum, weight_decay=wd)
    losses = []
    for x, y in batches:
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
            loss = F.cross_entropy(ref(x).float(), y)
        loss.backward()
        opt.step()
        losses.append(float(loss.detach()))
    return sum(losses) / len(losses)


def test_resnet_trajectory_matches_torch_within_bf16_floor():
    """ResNet-18 over 20 local steps (4 fits of 5 steps: momentum, weight decay, BN running
    statistics carried across fits) on the grouped engine vs torch fp32 and torch bf16 autocast on
    the same batches in the same order. The engine's per-fit mean loss (the loss curve) and its final
    per-tensor parameter deltas must stay within the bf16 noise floor that torch's own autocast run
    shows against fp32 (one step only was pinned before)."""
    from myfyp_amd.models import ResNet18

    # lr 0.01: at 0.05 this 80-sample problem is chaotic (torch's own bf16 and fp32 runs part ways
    # by fit 3: 3.47 vs 4.76 on the CPU), at 0.01 they agree to ~1e-2 per fit
    steps, fits, batch, lr, mom, wd = 5, 4, 16, 0.01, 0.9, 5e-4
    learners, refs, _ = _make_learners(lambda i: ResNet18(seed=80 + i), 1, steps * batch, 16, batch, lr, mom, wd)
    lr_ = learners[0]
    g = lr_._engine.group
    g.perm_fn = lambda ep: torch.arange(g.nmax, dtype=torch.int32, device="cuda").unsqueeze(0).repeat(g.capacity, 1)
    x, y = lr_.device_data(True)
    batches = [(x[i * batch:(i + 1) * batch], y[i * batch:(i + 1) * batch]) for i in range(steps)]
    r32, r16 = refs[0], ResNet18(seed=80).cuda()
    p0 = {n: p.detach().clone() for n, p in r32.named_parameters()}
    from myfyp_amd.parallel.pending import resolve

    curve = {"engine": [], "fp32": [], "bf16": []}
    for f in range(fits):
        n_steps, loss = lr_._engine.fit(lr_, lr_._optimizer_spec(), {})
        assert n_steps == steps
        curve["engine"].append(float(resolve(loss)))  # the engine's mean training loss of this fit
        curve["fp32"].append(_torch_fit(r32, batches, lr, mom, wd, False))
        curve["bf16"].append(_torch_fit(r16, batches, lr, mom, wd, True))
    for f in range(fits):
        floor = abs(curve["bf16"][f] - curve["fp32"][f])
        assert abs(curve["engine"][f] - curve["fp32"][f]) <= max(0.05 * curve["fp32"][f] + 0.02, 3 * floor), (f, curve)
    assert curve["engine"][-1] < curve["engine"][0], curve  # it learns
    eng = dict(lr_.model.get_model().named_parameters())
    for name, p in r32.named_parameters():
        d32 = (p.detach() - p0[name]).flatten()
        if d32.norm() < 1e-8:
            continue
        d16 = (dict(r16.named_parameters())[name].detach() - p0[name]).flatten()
        de = (eng[name].detach() - p0[name]).flatten()
        rel16 = float((d16 - d32).norm() / d32.norm())
        rel = float((de - d32).norm() / d32.norm())
        assert rel < max(0.1, 2.0 * rel16), (name, rel, rel16)


class _FixedCorrection:
    """Stands in for the FedProx / SCAFFOLD callbacks: fixed optimizer extras for every fit."""

    def __init__(self, extra):
        self.extra = extra

    @staticmethod
    def get_name():
        return "fixed_correction"

    def get_info(self):
        return {}

    def set_info(self, info):
        pass

    def grad_correction(self):
        return self.extra


@pytest.mark.parametrize("mode", ["plain", "weight_decay", "fedprox", "scaffold"])
def test_lenet_fused_epoch_matches_layerwise_path(monkeypatch, mode):
    """A whole epoch with a partial last batch and momentum: fused step vs the layer-by-layer path
    (``k_opt_step``), with weight decay, a FedProx anchor/mu or SCAFFOLD c_global/c_local — the
    fused kernel reads those through its own index remaps (conv (co,ci,tap), fc1 e2t)."""
    import threading

    from myfyp_amd.models import LeNet5

    runs = []
    extras = None
    for fused in ("1", "0"):
        monkeypatch.setenv("MYFYP_LENET_FUSED", fused)
        wd = 5e-3 if mode == "weight_decay" else 0.0
        learners, _, _ = _make_learners(lambda i: LeNet5(seed=50 + i), 3, 100, 40, 32, 0.05, momentum=0.9, wd=wd)
        g = learners[0]._engine.group
        assert g.lenet_fused == (fused == "1")
        p0 = [lr_.flat_params().detach().clone() for lr_ in learners]
        if extras is None:  # same extras (device tensors, generated once) for both runs
            gen = torch.Generator(device="cuda").manual_seed(11)
            extras = []
            for q in p0:
                if mode == "fedprox":
                    extras.append({"anchor": q + 0.2 * torch.randn(q.shape, device="cuda", generator=gen), "mu": 1.0})
                elif mode == "scaffold":
                    extras.append({"c_global": 0.2 * torch.randn(q.shape, device="cuda", generator=gen),
                                   "c_local": 0.2 * torch.randn(q.shape, device="cuda", generator=gen)})
                else:
                    extras.append({})
        for lr_, ex in zip(learners, extras):
            lr_.callbacks = [_FixedCorrection(ex)] if ex else []
        ths = [threading.Thread(target=lr_.fit) for lr_ in learners]
        [t.start() for t in ths]
        [t.join() for t in ths]
        loss = g.stat.view(g.capacity, 4)[:3, :2].clone()
        ev = [lr_.evaluate() for lr_ in learners]
        runs.append(([lr_.flat_params().detach().clone() - q for lr_, q in zip(learners, p0)], loss, ev))
    (d_f, l_f, e_f), (d_l, l_l, e_l) = runs
    for a, b in zip(d_f, d_l):
        cos = F.cosine_similarity(a, b, dim=0)
        rel = (a - b).norm() / b.norm()
        assert cos > 0.98 and rel < 0.2, (mode, float(cos), float(rel))
    torch.testing.assert_close(l_f, l_l, rtol=3e-2, atol=1e-2)  # (loss sum, correct) per peer
    for a, b in zip(e_f, e_l):
        assert abs(a["test_loss"] - b["test_loss"]) < 0.05 * max(1.0, b["test_loss"]), (a, b)


@pytest.mark.parametrize("fused", ["1", "0"])
def test_lenet_eval_matches_torch(fused, monkeypatch):
    from myfyp_amd.models import LeNet5

    monkeypatch.setenv("MYFYP_LENET_FUSED", fused)
    learners, refs, parts = _make_learners(lambda i: LeNet5(seed=60 + i), 2, 32, 70, 32, 0.05)
    for lr_, ref in zip(learners, refs):
        res = lr_.evaluate()
        ref.load_state_dict(lr_.model.get_model().state_dict())
        ref.eval()
        x, y = lr_.device_data(False)
        with torch.no_grad():
            out = ref(x)
        loss = float(F.cross_entropy(out, y))
        acc = float((out.argmax(1) == y).float().mean())
        assert abs(res["test_loss"] - loss) < 0.03 * max(1.0, loss), (res, loss)
        assert abs(res["test_metric"] - acc) <= 2.0 / len(y) + 0.03


def test_resnet_train_step_matches_torch():
    from myfyp_amd.models import ResNet18

    _run_one_step(lambda i: ResNet18(seed=20 + i), n_peers=2, batch=16, lr=0.05, momentum=0.9, wd=5e-4)


def test_cnn_eval_matches_torch():
    from myfyp_amd.models import ResNet18

    learners, refs, parts = _make_learners(lambda i: ResNet18(seed=30 + i), 2, 32, 48, 16, 0.05)
    for lr_, ref in zip(learners, refs):
        res = lr_.evaluate()
        ref.load_state_dict(lr_.model.get_model().state_dict())
        ref.eval()
        x, y = lr_.device_data(False)
        with torch.no_grad():
            out = ref(x)
        loss = float(F.cross_entropy(out, y))
        acc = float((out.argmax(1) == y).float().mean())
        assert abs(res["test_loss"] - loss) < 0.05 * max(1.0, loss), (res, loss)
        assert abs(res["test_metric"] - acc) <= 2.0 / len(y) + 0.05


def test_cnn_graph_replay_matches_eager():
    """Fits replayed from the captured HIP graph reproduce the eager launch sequence and keep
    lowering the training loss."""
    import threading

    from myfyp_amd.models import LeNet5

    runs = []
    for eager in (True, False):
        learners, _, _ = _make_learners(lambda i: LeNet5(seed=40 + i), 2, 512, 256, 64, 0.05, momentum=0.9)
        g = learners[0]._engine.group
        g.eager = eager
        losses = []
        for _ in range(4):
            ths = [threading.Thread(target=lr_.fit) for lr_ in learners]
            [t.start() for t in ths]
            [t.join() for t in ths]
            losses.append(float(g.stat.view(g.capacity, 4)[0, 0]))
        runs.append((losses, learners[0].flat_params().detach().clone(), len(g._graphs)))
    (l_e, p_e, n_e), (l_g, p_g, n_g) = runs
    assert n_e == 0 and n_g >= 1
    assert l_g[-1] < l_g[0] and l_e[-1] < l_e[0]
    np.testing.assert_allclose(l_e, l_g, rtol=1e-2)
    # wgrad split-K accumulates with fp32 atomics: summation order (not the math) may differ
    torch.testing.assert_close(p_e, p_g, atol=2e-3, rtol=2e-2)


@pytest.mark.parametrize("late", [False, True])
def test_cnn_epoch_graph_captured_after_first_run(monkeypatch, late):
    """The first fit of an epoch shape runs eagerly and is captured right after it (so round 1
    replays a ready graph); MYFYP_CNN_CAPTURE_LATE=1 captures on the second fit instead. Both
    placements train (finite losses)."""
    import threading

    from myfyp_amd.models import LeNet5

    monkeypatch.setenv("MYFYP_CNN_CAPTURE_LATE", "1" if late else "0")
    learners, _, _ = _make_learners(lambda i: LeNet5(seed=40 + i), 2, 512, 256, 64, 0.05, momentum=0.9)
    g = learners[0]._engine.group
    counts, losses = [], []
    for _ in range(2):
        ths = [threading.Thread(target=lr_.fit) for lr_ in learners]
        [t.start() for t in ths]
        [t.join() for t in ths]
        counts.append(len(g._graphs))
        losses.append(float(g.stat.view(g.capacity, 4)[0, 0]))
    assert counts == ([0, 1] if late else [1, 1]), counts
    assert np.isfinite(losses).all(), losses


def _within_floor(floor, opt_in):
    """Opt-in path vs default, per peer, against the default path's OWN run-to-run distance
    measured in the same test (two default runs). ``scripts/probes/cnn_ab_noise.py`` on MI355X
    (``profiles/r5_cnn_ab_noise/cnn_ab.log``): two default runs of one ResNet-18 epoch (batch 16,
    SGD momentum) differ by cos 0.979-0.986 / rel 0.17-0.21 (fp32 atomic order in the BN
    statistics and split-K sums flips bf16 roundings; the BatchNorms amplify them), and every
    opt-in path lands at the same distance from the default (cos 0.976-0.984 / rel 0.18-0.22).
    So the bound is that floor plus a small margin (rel x1.2 + 0.03, cos - 0.015) — no constant
    fallback (round 4 allowed rel up to 0.25 whatever the floor)."""
    for (c_n, r_n), (c_f, r_f) in zip(floor, opt_in):
        assert c_f > c_n - 0.015 and r_f < 1.2 * r_n + 0.03, ((c_f, r_f), (c_n, r_n))


def test_resnet_bn1_prologue_fusion_matches_materialised_path(monkeypatch):
    """BN1-apply + ReLU folded into conv2's forward / wgrad prologues, with the ReLU mask recomputed
    from y1 in the BN backward, against the path that materialises a1 (k_bn_act). The prologue
    rounds relu(y*sc + sh) to bf16 exactly like k_bn_act. The runs still differ in the order of
    the BN-statistics and split-K fp32 atomics; at batch 16 with bf16 activations that order alone
    moves one step's update by ~20 % (measured: two unfused runs give cos 0.977, rel 0.21 —
    scripts/probes/cnn_fuse_noise.py). So the fused run is compared against the unfused
    run-to-run noise floor, and the first step's loss (forward only) must agree tightly."""
    import threading

    from myfyp_amd.models import ResNet18

    runs = []
    for fuse in ("0", "0", "1"):
        monkeypatch.setenv("MYFYP_CNN_FUSE_BN", fuse)
        learners, _, _ = _make_learners(lambda i: ResNet18(seed=70 + i), 2, 16, 16, 16, 0.05, momentum=0.9, wd=5e-4)
        g = learners[0]._engine.group
        assert g.fuse_bn1 == (fuse == "1")
        p0 = [lr_.flat_params().detach().clone() for lr_ in learners]
        ths = [threading.Thread(target=lr_.fit) for lr_ in learners]
        [t.start() for t in ths]
        [t.join() for t in ths]
        loss = float(g.stat.view(g.capacity, 4)[0, 0])
        runs.append(([lr_.flat_params().detach().clone() - q for lr_, q in zip(learners, p0)], loss))
    (d_u1, l_u1), (d_u2, l_u2), (d_f, l_f) = runs

    def dist(xs, ys):
        return [(float(F.cosine_similarity(a, b, dim=0)), float((a - b).norm() / b.norm())) for a, b in zip(xs, ys)]

    _within_floor(dist(d_u2, d_u1), dist(d_f, d_u1))
    assert abs(l_f - l_u1) < 1e-2 * max(1.0, abs(l_u1)), (l_f, l_u1, l_u2)


def test_resnet_bn_finalize_in_conv_tail_matches_separate_launches(monkeypatch):
    """BatchNorm finalize run by the producing conv's last workgroup (MYFYP_CNN_FUSE_FIN=1,
    conv.hip conv_fin_tail: forward statistics -> scale/shift + running statistics, BN-backward sums
    -> apply coefficients + dgamma/dbeta) against the separate k_bn_finalize / k_bn_bwd_finalize
    launches. Same math; only the order in which the fp32 accumulator rows are summed differs. One
    step of two peers: the forward loss and the running statistics agree closely,
    and the update within the run-to-run floor / the measured bf16 chaos level (see the tests
    above). A lost arrival or an unsummed row would be far outside these bounds."""
    import threading

    from myfyp_amd.models import ResNet18

    runs = []
    for flag in ("0", "0", "1"):
        monkeypatch.setenv("MYFYP_CNN_FUSE_FIN", flag)
        learners, _, _ = _make_learners(lambda i: ResNet18(seed=110 + i), 2, 16, 16, 16, 0.05, momentum=0.9, wd=5e-4)
        g = learners[0]._engine.group
        assert g.fuse_fin == (flag == "1")
        p0 = [lr_.flat_params().detach().clone() for lr_ in learners]
        ths = [threading.Thread(target=lr_.fit) for lr_ in learners]
        [t.start() for t in ths]
        [t.join() for t in ths]
        loss = float(g.stat.view(g.capacity, 4)[0, 0])
        torch.cuda.synchronize()
        run_stats = [g.params[slot, g.n_params:].detach().float().clone() for slot in range(len(learners))]
        runs.append(([lr_.flat_params().detach().clone() - q for lr_, q in zip(learners, p0)], loss, run_stats))
    (d_u1, l_u1, s_u1), (d_u2, l_u2, s_u2), (d_f, l_f, s_f) = runs
    # the epoch loss (a sum over the batch) moves by bf16 rounding flips behind the first BN whose
    # statistics were summed in another order (measured 1.5e-4 relative); wrong statistics move it
    # by percents
    assert abs(l_f - l_u1) < 1e-3 * max(1.0, abs(l_u1)), (l_f, l_u1, l_u2)
    # running statistics: a bf16 rounding flip after the first BN (statistics summed in another
    # order) reaches the deeper layers' statistics (measured: 12 of 9654 values 1e-4..1.5e-4 off);
    # a lost arrival or an unsummed accumulator row moves whole channels by far more
    floor = max(float((a - b).abs().max()) for a, b in zip(s_u2, s_u1))
    for a, b in zip(s_f, s_u1):
        assert float((a - b).abs().max()) <= max(4 * floor, 5e-4), (float((a - b).abs().max()), floor)

    def dist(xs, ys):
        return [(float(F.cosine_similarity(a, b, dim=0)), float((a - b).norm() / b.norm())) for a, b in zip(xs, ys)]

    _within_floor(dist(d_u2, d_u1), dist(d_f, d_u1))


def test_resnet_stride2_dgrad_as_parity_forward_matches_default(monkeypatch):
    """MYFYP_CNN_S2_FWD=1 (stride-2 dgrads as four parity-class forward convs, conv.hip MODE 5) against
    the default MODE 2 path, over one local epoch of two peers. MODE 5 sums the taps in another
    order, so its bf16 dX differs in the last bit; at batch 16 such a difference grows through the
    BatchNorms to about 20 % of one epoch's update (measured: two MODE-2 paths that differ only in
    fp32 atomic order gave cos 0.977, rel 0.21 — scripts/probes/cnn_fuse_noise.py). The default
    path's own repeat runs are nearly bit-identical now (rel 3e-4), so the bound is that measured
    bf16 chaos level, not the run-to-run floor."""
    import threading

    from myfyp_amd.models import ResNet18

    runs = []
    for flag in ("0", "0", "1"):
        monkeypatch.setenv("MYFYP_CNN_S2_FWD", flag)
        learners, _, _ = _make_learners(lambda i: ResNet18(seed=90 + i), 2, 16, 16, 16, 0.05, momentum=0.9, wd=5e-4)
        g = learners[0]._engine.group
        assert g.s2_fwd == (flag == "1")
        p0 = [lr_.flat_params().detach().clone() for lr_ in learners]
        ths = [threading.Thread(target=lr_.fit) for lr_ in learners]
        [t.start() for t in ths]
        [t.join() for t in ths]
        runs.append([lr_.flat_params().detach().clone() - q for lr_, q in zip(learners, p0)])
    d_u1, d_u2, d_f = runs

    def dist(xs, ys):
        return [(float(F.cosine_similarity(a, b, dim=0)), float((a - b).norm() / b.norm())) for a, b in zip(xs, ys)]

    _within_floor(dist(d_u2, d_u1), dist(d_f, d_u1))


@pytest.mark.parametrize("mode", [0, 4])
@pytest.mark.parametrize("cout,h", [(128, 12), (64, 32)])
def test_conv_grouped_peers_with_uneven_batches(mode, conv_dma, cout, h):
    """Three peers in one launch (grid.z) with per-peer valid batches 5 / 1 / 3 (``nbatch``), forward
    with BN statistics (mode 0) and the stride-1 dgrad as a forward conv (mode 4): every peer's rows
    match torch and rows past a peer's batch are left untouched (the persistent DMA kernel sizes its
    M tiles per peer)."""
    from myfyp_amd.parallel.cnn_engine import ConvGemmArgs, _lib

    lib = _lib()
    dev = torch.device("cuda")
    torch.manual_seed(5)
    P, nmax, cin, k = 3, 5, 64, 3  # (64, 32): the halo forward (k_conv_fwd_halo) on layer-1 shapes
    nbs = [5, 1, 3]
    cpi, cpo = _cp(cin), _cp(cout)
    xs = [_bf(torch.randn(nmax, cin, h, h, device=dev)) for _ in range(P)]
    ws = [_bf(torch.randn(cout, cin, k, k, device=dev) * (1.0 / (cin * k * k) ** 0.5)) for _ in range(P)]
    if mode == 0:
        src = torch.stack([_nhwc_pad(x, cpi).reshape(-1) for x in xs]).contiguous()
        wf = torch.stack([w.permute(0, 2, 3, 1).to(torch.bfloat16).reshape(-1) for w in ws]).contiguous()
        ncol, c_src, refs = cpo, cpi, [F.conv2d(x, w, padding=1) for x, w in zip(xs, ws)]
    else:  # dY of the conv cin -> cout; dX = conv_transpose, weights flipped per peer
        dys = [_bf(torch.randn(nmax, cout, h, h, device=dev)) for _ in range(P)]
        src = torch.stack([_nhwc_pad(d, cpo).reshape(-1) for d in dys]).contiguous()
        wf0 = torch.stack([w.permute(0, 2, 3, 1).to(torch.bfloat16).reshape(-1) for w in ws]).contiguous()
        wf = torch.zeros_like(wf0)
        assert lib.conv_wt_flip_launch(wf0.data_ptr(), wf0.shape[1], wf.data_ptr(), wf.shape[1], cpo, cpi, k, k, P, torch.cuda.current_stream().cuda_stream) == 0
        ncol, c_src = cpi, cpo
        refs = [torch.nn.grad.conv2d_input((nmax, cin, h, h), w, d, padding=1) for w, d in zip(ws, dys)]
    out = torch.full((P, nmax * h * h * ncol), 7.0, device=dev, dtype=torch.bfloat16)
    nb = torch.tensor(nbs, dtype=torch.int32, device=dev)
    rows = lib.conv_gemm_stats_rows(nmax, h, h)
    stats = torch.zeros(P, rows * 2 * ncol, device=dev)
    a = ConvGemmArgs()
    a.src, a.src_ps, a.src_h, a.src_w, a.src_c = src.data_ptr(), src.shape[1], h, h, c_src
    a.out_h, a.out_w, a.R, a.S, a.stride, a.pad = h, h, k, k, 1, 1
    a.wt, a.wt_ps, a.ncol, a.ncol_valid = wf.data_ptr(), wf.shape[1], ncol, (cout if mode == 0 else cin)
    a.out, a.out_ps, a.nbatch, a.max_batch = out.data_ptr(), out.shape[1], nb.data_ptr(), nmax
    if mode == 0:
        a.stats, a.stats_ps, a.stats_rows = stats.data_ptr(), stats.shape[1], rows
    assert lib.conv_gemm_launch(mode, ctypes.byref(a), P, torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    for p in range(P):
        o = out[p].view(nmax, h, h, ncol)
        n = nbs[p]
        c = cout if mode == 0 else cin
        torch.testing.assert_close(o[:n, ..., :c].float(), refs[p][:n].permute(0, 2, 3, 1), atol=3e-2, rtol=3e-2)
        assert bool((o[n:] == 7.0).all()), f"peer {p}: rows past its batch were written"
        if mode == 0:
            st = stats[p].view(rows, 2, ncol).sum(0)
            torch.testing.assert_close(st[0, :cout], refs[p][:n].sum((0, 2, 3)), atol=0.5, rtol=2e-2)


@pytest.mark.parametrize("h,n", [(32, 2), (32, 3)])
def test_bn_prologue_in_patch_kernels_matches_materialised(h, n):
    """BN1-apply + ReLU folded into the patch-staged kernels (ResNet-18 layer-1 conv2): the forward
    (k_conv_fwd_halo with pro_ss) and the weight gradient (k_conv_wgrad_halo with pro_ss) read the
    BatchNorm input y and transform each staged pixel once; the stride-1 dgrad's BN-backward epilogue
    takes its ReLU mask from y (bnb_mask_ss). Against the same kernels on the materialised
    activation a = k_bn_act(y): outputs and weight gradients bit-identical (same bf16 operands, same
    MFMA order), BatchNorm column sums equal up to their fp32 atomic order."""
    from myfyp_amd.parallel.cnn_engine import ConvGemmArgs, WgradArgs, _lib

    lib = _lib()
    dev = torch.device("cuda")
    s_ = torch.cuda.current_stream().cuda_stream
    torch.manual_seed(5)
    C, k, pad = 64, 3, 1
    rows = n * h * h
    y = (torch.randn(1, rows * C, device=dev) * 2 + 0.3).to(torch.bfloat16)
    ss = torch.cat([torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.5]).view(1, -1).contiguous()
    a_mat = torch.zeros_like(y)
    nb = torch.full((1,), n, dtype=torch.int32, device=dev)
    assert lib.cnn_bn_act(y.data_ptr(), 0, ss.data_ptr(), None, 0, None, 0, None, 1, nb.data_ptr(), rows, h * h, C, a_mat.data_ptr(), 0, 1, s_) == 0
    w = (torch.randn(C, k, k, C, device=dev) * (1.0 / (C * 9) ** 0.5)).to(torch.bfloat16)  # Wf [co][r][s][ci]
    srows = lib.conv_gemm_stats_rows(n, h, h)

    def fwd(src, pro):
        out = torch.zeros_like(y)
        st = torch.zeros(1, srows * 2 * C, device=dev)
        a = ConvGemmArgs()
        a.src, a.src_h, a.src_w, a.src_c = src.data_ptr(), h, h, C
        a.out_h, a.out_w, a.R, a.S, a.stride, a.pad = h, h, k, k, 1, pad
        a.wt, a.ncol, a.ncol_valid = w.data_ptr(), C, C
        a.out, a.stats, a.stats_rows, a.max_batch = out.data_ptr(), st.data_ptr(), srows, n
        if pro:
            a.pro_ss = ss.data_ptr()
        assert lib.conv_gemm_launch(0, ctypes.byref(a), 1, s_) == 0
        torch.cuda.synchronize()
        return out, st.view(srows, 2, C).sum(0)

    (o_f, st_f), (o_m, st_m) = fwd(y, True), fwd(a_mat, False)
    assert torch.equal(o_f, o_m)
    torch.testing.assert_close(st_f, st_m, rtol=1e-5, atol=1e-3)

    dy = torch.randn(1, rows * C, device=dev).to(torch.bfloat16)

    def wgrad(x, pro):
        grad = torch.zeros(1, C * 9 * C, device=dev)
        c = WgradArgs()
        c.dy, c.x = dy.data_ptr(), x.data_ptr()
        c.H, c.W, c.x_c, c.Ho, c.Wo, c.dy_c = h, h, C, h, h, C
        c.R, c.S, c.stride, c.pad = k, k, 1, pad
        c.grad, c.accumulate, c.k_per_split, c.max_batch = grad.data_ptr(), 0, (rows + 63) // 64 * 64, n
        if pro:
            c.pro_ss = ss.data_ptr()
        assert lib.conv_wgrad_launch(ctypes.byref(c), 1, 1, s_) == 0
        torch.cuda.synchronize()
        return grad

    assert torch.equal(wgrad(y, True), wgrad(a_mat, False))

    # stride-1 dgrad (MODE 4, flipped weights) with the BN-backward epilogue of this BN: mask from a
    # (materialised) vs mask from y
    wt = torch.zeros_like(w)
    assert lib.conv_wt_flip_launch(w.data_ptr(), 0, wt.data_ptr(), 0, C, C, k, k, 1, s_) == 0
    ms = torch.cat([torch.randn(C, device=dev), torch.rand(C, device=dev) + 0.5]).view(1, -1).contiguous()
    nr = lib.conv_bnb_rows()

    def dgrad(mask_mat):
        out = torch.zeros_like(y)
        part = torch.zeros(1, nr * 2 * C, device=dev)
        b = ConvGemmArgs()
        b.src, b.src_h, b.src_w, b.src_c = dy.data_ptr(), h, h, C
        b.out_h, b.out_w, b.R, b.S, b.stride, b.pad = h, h, k, k, 1, k - 1 - pad
        b.wt, b.ncol, b.ncol_valid = wt.data_ptr(), C, C
        b.out, b.max_batch, b.bnb_rows = out.data_ptr(), n, nr
        b.bnb_y0, b.bnb_ms0, b.bnb_part0 = y.data_ptr(), ms.data_ptr(), part.data_ptr()
        if mask_mat:
            b.bnb_mask = a_mat.data_ptr()
        else:
            b.bnb_mask_ss = ss.data_ptr()
        assert lib.conv_gemm_launch(4, ctypes.byref(b), 1, s_) == 0
        torch.cuda.synchronize()
        return out, part.view(nr, 2 * C).sum(0)

    (g_m, p_m), (g_y, p_y) = dgrad(True), dgrad(False)
    assert torch.equal(g_m, g_y)
    torch.testing.assert_close(p_y, p_m, rtol=1e-5, atol=1e-3)


def test_resnet_fused_fit_interrupted_mid_epoch():
    """``interrupt_fit`` on a fused CNN fit already on the device (reference: a Lightning fit stopped
    mid-epoch, lightning_learner.py:110-114): the device is held busy so the epoch has not started
    when peer 0 is interrupted; peer 0's parameters and BN running statistics stay exactly as they
    were while peer 1 of the same gang trains on; the next fit (a new fit id) trains peer 0 again."""
    import threading

    from myfyp_amd.models import ResNet18

    learners, _, _ = _make_learners(lambda i: ResNet18(seed=40 + i), 2, 64 * 6, 64, 64, 0.05, momentum=0.9)

    def fit_all():
        ths = [threading.Thread(target=lr_.fit) for lr_ in learners]
        [t.start() for t in ths]
        [t.join() for t in ths]

    def state(i):
        m = learners[i].model.get_model()
        return [t.detach().clone() for t in list(m.parameters()) + [b for n, b in m.named_buffers() if "running" in n]]

    fit_all()  # first fit: eager run + graph capture
    torch.cuda.synchronize()
    s0, s1 = state(0), state(1)
    torch.cuda._sleep(200_000_000)  # the epoch queued behind this cannot start before the interrupt
    fit_all()
    learners[0].interrupt_fit()
    torch.cuda.synchronize()
    a0, a1 = state(0), state(1)
    assert all(torch.equal(x, y) for x, y in zip(s0, a0)), "interrupted peer changed"
    assert any(not torch.equal(x, y) for x, y in zip(s1, a1)), "the other peer did not train"
    fit_all()  # a later fit is not affected by the stale stop word
    torch.cuda.synchronize()
    assert any(not torch.equal(x, y) for x, y in zip(a0, state(0))), "peer 0 did not train after the interrupted fit"


@pytest.mark.parametrize("c,h,n,splits", [(64, 32, 2, 1), (64, 32, 3, 5), (128, 16, 3, 2), (256, 8, 5, 3), (512, 4, 16, 1), (64, 8, 3, 2)])
def test_wgrad_halo_prefetch_depths_agree(c, h, n, splits):
    """k_conv_wgrad_halo with two register stages in flight (PF 2, the default) against one (PF 1,
    pinned to torch by test_conv_fwd_dgrad_wgrad_vs_torch's earlier rounds): K loops of 1, 2 and odd
    step counts; equal up to the split-K atomics' order."""
    from myfyp_amd.parallel.cnn_engine import WgradArgs, _lib

    lib = _lib()
    dev = torch.device("cuda")
    torch.manual_seed(c + h)
    x = torch.randn(1, n * h * h * c, device=dev).to(torch.bfloat16)
    dy = torch.randn(1, n * h * h * c, device=dev).to(torch.bfloat16)
    M = n * h * h
    k_per = max(64, ((M + splits - 1) // splits + 63) // 64 * 64)
    sp = (M + k_per - 1) // k_per
    grads = {}
    old = lib.conv_set_wgrad_pf(1)
    try:
        for pf in (1, 2):
            lib.conv_set_wgrad_pf(pf)
            g = torch.zeros(1, c * 9 * c, device=dev)
            a = WgradArgs()
            a.dy, a.dy_ps, a.x, a.x_ps = dy.data_ptr(), dy.shape[1], x.data_ptr(), x.shape[1]
            a.H, a.W, a.x_c, a.Ho, a.Wo, a.dy_c = h, h, c, h, h, c
            a.R, a.S, a.stride, a.pad = 3, 3, 1, 1
            a.grad, a.grad_ps, a.accumulate, a.k_per_split, a.max_batch = g.data_ptr(), g.shape[1], int(sp > 1), k_per, n
            assert lib.conv_wgrad_launch(ctypes.byref(a), 1, sp, torch.cuda.current_stream().cuda_stream) == 0
            torch.cuda.synchronize()
            grads[pf] = g
    finally:
        lib.conv_set_wgrad_pf(old)
    if sp == 1:
        assert torch.equal(grads[1], grads[2])
    else:
        torch.testing.assert_close(grads[2], grads[1], rtol=1e-5, atol=1e-4 * float(grads[1].abs().max()))
    assert float(grads[1].abs().max()) > 0
