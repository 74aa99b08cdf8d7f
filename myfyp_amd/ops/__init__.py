"""Fused device ops (HIP, gfx950) with PyTorch reference implementations for CPU hosts.

Every op takes/returns torch tensors. Device tensors go to the hand-written kernels in
``csrc/kernels`` (through :mod:`myfyp_amd.ops._native`); CPU tensors use the reference math below,
which is also the numerics oracle in ``tests/test_kernels_gpu.py``.

Ops
---
* ``weighted_average``  — FedAvg reduction over K models (multi-tensor, one launch per layer list)
* ``stacked_weighted_sum`` / ``broadcast_rows`` — reductions over a ``[P, N]`` stacked flat buffer
  (co-located peers) feeding / consuming the RCCL all-reduce
* ``coordinate_median`` — FedMedian (register sorting network, K ≤ 16)
* ``adam_step`` / ``sgd_step`` — fused optimizers over a flat buffer, optionally with the FedProx
  proximal term and the SCAFFOLD control-variate correction fused in (K5, K8, K13)
* ``scale_add_noise`` — attack injection (sign flip / Gaussian noise, K14)
"""

from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import torch

from myfyp_amd.ops import _native

__all__ = [
    "weighted_average",
    "stacked_weighted_sum",
    "broadcast_rows",
    "coordinate_median",
    "adam_step",
    "sgd_step",
    "scale_add_noise",
    "native_available",
]


def native_available() -> bool:
    return _native.available()


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _lib():
    return _native.load(required=True)


def fast_lib():
    """Native library with GIL-holding bindings for launch-only entry points (see _native.load_fast)."""
    return _native.load_fast()


def check(rc: int, what: str) -> None:
    _native.check(rc, what)


# ---------------------------------------------------------------------------------------------
# aggregation
# ---------------------------------------------------------------------------------------------
def weighted_average(param_lists: Sequence[Sequence[torch.Tensor]], norm_weights: Sequence[float]) -> List[torch.Tensor]:
    """``out[l] = Σ_k w_k · params[k][l]`` (weights already normalised)."""
    k = len(param_lists)
    out: List[torch.Tensor] = []
    dev = param_lists[0][0].device
    if dev.type != "cuda":
        for layer in range(len(param_lists[0])):
            acc = torch.zeros_like(param_lists[0][layer], dtype=torch.float64)
            for p, w in zip(param_lists, norm_weights):
                acc += p[layer].double() * w
            out.append(acc.to(param_lists[0][layer].dtype))
        return out
    lib = _lib()
    w = torch.tensor(list(norm_weights), dtype=torch.float32, device=dev)
    for layer in range(len(param_lists[0])):
        srcs = [p[layer].contiguous().float() for p in param_lists]
        dst = torch.empty_like(srcs[0])
        ptrs = torch.tensor([s.data_ptr() for s in srcs], dtype=torch.int64, device=dev)
        _native.check(lib.myfyp_weighted_sum(dst.data_ptr(), ptrs.data_ptr(), w.data_ptr(), k, dst.numel(), _stream()), "weighted_sum")
        out.append(dst.to(param_lists[0][layer].dtype))
    return out


def stacked_weighted_sum(stacked: torch.Tensor, weights: torch.Tensor, out: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
    """``out[n] = scale · Σ_p weights[p] · stacked[p, n]`` for a ``[P, N]`` fp32 buffer."""
    if stacked.device.type != "cuda":
        out.copy_((weights.view(-1, 1).to(stacked.dtype) * stacked).sum(0) * scale)
        return out
    lib = _lib()
    p, n = stacked.shape
    _native.check(
        lib.myfyp_stacked_weighted_sum(out.data_ptr(), stacked.data_ptr(), p, n, stacked.stride(0), weights.data_ptr(), float(scale), _stream()),
        "stacked_weighted_sum",
    )
    return out


def broadcast_rows(src: torch.Tensor, stacked: torch.Tensor, mask: Optional[torch.Tensor] = None, shadow: Optional[torch.Tensor] = None) -> None:
    """``stacked[p, :] = src`` for every row p with ``mask[p] != 0`` (and the bf16 shadow copy)."""
    if stacked.device.type != "cuda":
        rows = range(stacked.shape[0]) if mask is None else [i for i in range(stacked.shape[0]) if float(mask[i]) != 0]
        for r in rows:
            stacked[r].copy_(src)
            if shadow is not None:
                shadow[r].copy_(src.to(shadow.dtype))
        return
    lib = _lib()
    p, n = stacked.shape
    _native.check(lib.myfyp_broadcast_rows(stacked.data_ptr(), src.data_ptr(), p, n, stacked.stride(0), _ptr(mask), _stream()), "broadcast_rows")
    if shadow is not None:
        shadow.copy_(stacked.to(shadow.dtype))


def coordinate_median(param_lists: Sequence[Sequence[torch.Tensor]]) -> List[torch.Tensor]:
    k = len(param_lists)
    out: List[torch.Tensor] = []
    dev = param_lists[0][0].device
    if dev.type != "cuda" or k > 16:
        for layer in range(len(param_lists[0])):
            st = torch.stack([p[layer].float() for p in param_lists])
            s, _ = torch.sort(st, dim=0)
            med = s[(k - 1) // 2] if k % 2 else 0.5 * (s[k // 2 - 1] + s[k // 2])
            out.append(med.to(param_lists[0][layer].dtype))
        return out
    for layer in range(len(param_lists[0])):
        srcs = [p[layer].contiguous().float().reshape(-1) for p in param_lists]
        dst = torch.empty_like(srcs[0])
        median_into(srcs, [dst])
        out.append(dst.view_as(param_lists[0][layer]).to(param_lists[0][layer].dtype))
    return out


def _host_ptrs(ts: Sequence[torch.Tensor]) -> ctypes.c_void_p:
    """Host table of device row pointers (the native entry points pass it as a kernel argument)."""
    arr = (ctypes.c_uint64 * max(1, len(ts)))(*[t.data_ptr() for t in ts])
    return ctypes.cast(arr, ctypes.c_void_p), arr  # keep arr alive across the call


def median_into(rows: Sequence[torch.Tensor], outs: Sequence[torch.Tensor]) -> None:
    """``outs[p] = coordinate-wise median(rows)`` for 1-D fp32 rows; on the GPU one launch
    (``k_coordinate_median<K>``) for K <= 16 rows and <= 16 outputs, which may alias the rows."""
    k = len(rows)
    if rows[0].device.type == "cuda" and k <= 16 and len(outs) <= 16 and all(t.is_contiguous() and t.dtype == torch.float32 for t in [*rows, *outs]):
        src, keep_s = _host_ptrs(rows)
        dst, keep_d = _host_ptrs(outs)
        _native.check(_lib().myfyp_coordinate_median_multi(dst, len(outs), src, k, rows[0].numel(), _stream()), "coordinate_median_multi")
        return
    s, _ = torch.sort(torch.stack([r.float() for r in rows]), dim=0)
    med = s[(k - 1) // 2] if k % 2 else 0.5 * (s[k // 2 - 1] + s[k // 2])
    for o in outs:
        o.copy_(med)


def scaffold_reduce(buf: torch.Tensor, dys: Sequence[torch.Tensor], dcs: Sequence[torch.Tensor], weights: Sequence[float]) -> None:
    """``buf = [Σ w_k Δy_k | Σ w_k | Σ Δc_k | K]`` (2n + 2 floats) from the local contributors."""
    n = (buf.numel() - 2) // 2
    k = len(dys)
    if buf.device.type == "cuda" and k <= 16:
        y, keep_y = _host_ptrs(dys)
        c, keep_c = _host_ptrs(dcs)
        w = (ctypes.c_float * max(1, k))(*weights)
        _native.check(_lib().myfyp_scaffold_reduce(buf.data_ptr(), y, c, ctypes.cast(w, ctypes.c_void_p), k, n, _stream()), "scaffold_reduce")
        return
    buf.zero_()
    for dy, dc, wt in zip(dys, dcs, weights):
        buf[:n].add_(dy, alpha=wt)
        buf[n + 1 : 2 * n + 1].add_(dc)
    buf[n] = float(sum(weights))
    buf[2 * n + 1] = float(k)


def scaffold_apply(outs: Sequence[torch.Tensor], x_start: torch.Tensor, buf: torch.Tensor, c: torch.Tensor, c_init: bool, global_lr: float) -> None:
    """``outs[p] = x_start + η_g · buf[:n] / buf[n]``; ``c = (0 if c_init else c) + buf[n+1:2n+1] / buf[2n+1]``."""
    n = x_start.numel()
    if buf.device.type == "cuda" and len(outs) <= 16:
        o, keep = _host_ptrs(outs)
        _native.check(_lib().myfyp_scaffold_apply(o, len(outs), x_start.data_ptr(), buf.data_ptr(), c.data_ptr(), int(c_init), float(global_lr), n, _stream()),
                      "scaffold_apply")
        return
    x_new = torch.addcmul(x_start, buf[:n], global_lr / buf[n : n + 1].clamp_min(1e-12))
    dc = buf[n + 1 : 2 * n + 1] / buf[2 * n + 1 : 2 * n + 2].clamp_min(1.0)
    if c_init:
        c.copy_(dc)
    else:
        c.add_(dc)
    for t in outs:
        t.copy_(x_new)


# ---------------------------------------------------------------------------------------------
# optimizers (flat fp32 buffers)
# ---------------------------------------------------------------------------------------------
def _corrected_grad(param, grad, anchor, mu):
    """FedProx's proximal gradient term (SCAFFOLD is applied in the update space: _scaffold_step)."""
    g = grad
    if anchor is not None and mu != 0.0:
        g = g + mu * (param - anchor)
    return g


def _scaffold_step(param, c_global, c_local, lr: float) -> None:
    """SCAFFOLD correction in the update space: ``w -= lr·(c − c_i)`` after the optimizer step
    (``opt_update`` in ``csrc/kernels/common.h`` explains why not in Adam's gradient)."""
    if c_global is not None and c_local is not None:
        param.sub_(c_global - c_local, alpha=lr)


def adam_step(
    param: torch.Tensor,
    grad: torch.Tensor,
    exp_avg: torch.Tensor,
    exp_avg_sq: torch.Tensor,
    step: int,
    lr: float = 1e-3,
    beta1: float = 0.9,
    beta2: float = 0.999,
    eps: float = 1e-8,
    weight_decay: float = 0.0,
    shadow: Optional[torch.Tensor] = None,
    anchor: Optional[torch.Tensor] = None,
    c_global: Optional[torch.Tensor] = None,
    c_local: Optional[torch.Tensor] = None,
    mu: float = 0.0,
) -> None:
    """One Adam step (torch.optim.Adam semantics, L2 ``weight_decay``), in place, step ≥ 1."""
    if param.device.type != "cuda":
        g = _corrected_grad(param, grad, anchor, mu)
        if weight_decay:
            g = g + weight_decay * param
        exp_avg.mul_(beta1).add_(g, alpha=1 - beta1)
        exp_avg_sq.mul_(beta2).addcmul_(g, g, value=1 - beta2)
        bc1 = 1 - beta1**step
        bc2 = 1 - beta2**step
        denom = (exp_avg_sq / bc2).sqrt_().add_(eps)
        param.addcdiv_(exp_avg, denom, value=-lr / bc1)
        _scaffold_step(param, c_global, c_local, lr)
        if shadow is not None:
            shadow.copy_(param.to(shadow.dtype))
        return
    lib = _lib()
    _native.check(
        lib.myfyp_adam_step(
            param.data_ptr(), grad.data_ptr(), exp_avg.data_ptr(), exp_avg_sq.data_ptr(), _ptr(shadow), param.numel(),
            lr, beta1, beta2, eps, weight_decay, int(step), _ptr(anchor), _ptr(c_global), _ptr(c_local), float(mu), _stream(),
        ),
        "adam_step",
    )


def sgd_step(
    param: torch.Tensor,
    grad: torch.Tensor,
    momentum_buf: Optional[torch.Tensor],
    lr: float,
    momentum: float = 0.0,
    weight_decay: float = 0.0,
    nesterov: bool = False,
    anchor: Optional[torch.Tensor] = None,
    c_global: Optional[torch.Tensor] = None,
    c_local: Optional[torch.Tensor] = None,
    mu: float = 0.0,
) -> None:
    """One SGD(+momentum, +nesterov) step (torch.optim.SGD semantics; buffer starts at 0)."""
    if param.device.type != "cuda":
        g = _corrected_grad(param, grad, anchor, mu)
        if weight_decay:
            g = g + weight_decay * param
        if momentum != 0.0 and momentum_buf is not None:
            momentum_buf.mul_(momentum).add_(g)
            g = g + momentum * momentum_buf if nesterov else momentum_buf
        param.add_(g, alpha=-lr)
        _scaffold_step(param, c_global, c_local, lr)
        return
    lib = _lib()
    _native.check(
        lib.myfyp_sgd_step(
            param.data_ptr(), grad.data_ptr(), _ptr(momentum_buf), param.numel(), lr, momentum, weight_decay, int(nesterov),
            _ptr(anchor), _ptr(c_global), _ptr(c_local), float(mu), _stream(),
        ),
        "sgd_step",
    )


def scale_add_noise(t: torch.Tensor, scale: float, sigma: float, seed: int = 0) -> None:
    """``t = scale·t + σ·N(0,1)`` in place (sign flip: scale=-1, σ=0)."""
    if t.device.type != "cuda" or t.dtype != torch.float32 or not t.is_contiguous():
        g = torch.Generator(device="cpu").manual_seed(seed)
        noise = torch.randn(t.shape, generator=g, dtype=torch.float32).to(t.device, t.dtype) if sigma else 0.0
        t.mul_(scale).add_(noise * sigma if sigma else 0.0)
        return
    lib = _lib()
    _native.check(lib.myfyp_scale_add_noise(t.data_ptr(), t.numel(), float(scale), float(sigma), int(seed), _stream()), "scale_add_noise")
