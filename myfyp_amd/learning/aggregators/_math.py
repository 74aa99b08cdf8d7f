"""Array-library-neutral reductions used by aggregators.

Parameters arrive either as numpy arrays (wire format, host) or as torch tensors (device-resident
models on the MI355X). For device tensors the reductions run on the GPU — through the fused HIP
kernels in :mod:`myfyp_amd.ops` when the extension is loaded — and never round-trip through host
memory.
"""

from __future__ import annotations

from typing import List, Sequence

import numpy as np


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


def weighted_mean(param_lists: Sequence[Sequence], weights: Sequence[float]) -> List:
    """``Σ_i w_i·p_i / Σ w_i`` per layer."""
    total = float(sum(weights))
    if total == 0:
        raise ValueError("Sum of weights is zero")
    first = param_lists[0][0]
    if _is_torch(first):
        from myfyp_amd import ops

        return ops.weighted_average([list(p) for p in param_lists], [float(w) / total for w in weights])
    out = []
    for layer_idx in range(len(param_lists[0])):
        acc = np.zeros_like(param_lists[0][layer_idx], dtype=np.float64)
        for p, w in zip(param_lists, weights):
            acc += np.asarray(p[layer_idx], dtype=np.float64) * w
        out.append((acc / total).astype(np.asarray(param_lists[0][layer_idx]).dtype))
    return out


def coordinate_median(param_lists: Sequence[Sequence]) -> List:
    """Per-coordinate median across models (even count → mean of the two middle values)."""
    first = param_lists[0][0]
    if _is_torch(first):
        from myfyp_amd import ops

        return ops.coordinate_median([list(p) for p in param_lists])
    out = []
    for layer_idx in range(len(param_lists[0])):
        stacked = np.stack([np.asarray(p[layer_idx]) for p in param_lists])
        out.append(np.median(stacked, axis=0).astype(stacked.dtype))
    return out


def trimmed_mean(param_lists: Sequence[Sequence], beta: float) -> List:
    """Per-coordinate mean after dropping the ``beta`` fraction of largest and smallest values."""
    n = len(param_lists)
    k = int(np.floor(beta * n))
    if 2 * k >= n:
        raise ValueError("beta too large for the number of models")
    first = param_lists[0][0]
    out = []
    for layer_idx in range(len(param_lists[0])):
        if _is_torch(first):
            import torch

            stacked = torch.stack([p[layer_idx] for p in param_lists]).float()
            s, _ = torch.sort(stacked, dim=0)
            out.append(s[k : n - k].mean(dim=0).to(first.dtype))
        else:
            stacked = np.sort(np.stack([np.asarray(p[layer_idx]) for p in param_lists]), axis=0)
            out.append(stacked[k : n - k].mean(axis=0).astype(stacked.dtype))
    return out


def flatten(params: Sequence) -> "np.ndarray":
    if _is_torch(params[0]):
        import torch

        return torch.cat([p.reshape(-1).float() for p in params])
    return np.concatenate([np.asarray(p, dtype=np.float64).reshape(-1) for p in params])


def to_numpy_list(params: Sequence) -> List[np.ndarray]:
    return [p.detach().cpu().numpy() if _is_torch(p) else np.asarray(p) for p in params]
