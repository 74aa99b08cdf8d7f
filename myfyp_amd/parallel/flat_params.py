"""Flat parameter buffers (SURVEY §2.10 native component #4).

All trainable parameters of a module are re-pointed into ONE contiguous fp32 buffer (and their
gradients into one grad buffer). Consequences on MI355X:

* the optimizer is one fused HIP launch over the whole model (K5) instead of one per tensor;
* aggregation / RCCL all-reduce / broadcast operate on one pointer (bucketed by byte size);
* co-located peers can share one ``[P, numel]`` allocation (``PeerGroup``), so a grouped kernel
  or a single weighted reduction covers all of them.

The module keeps working as a normal ``nn.Module`` (``state_dict`` returns views into the buffer).
"""

from __future__ import annotations

from typing import List, Optional, Tuple

import torch


class FlatParams:
    """Owns (or adopts) the flat buffers of a module's trainable parameters."""

    def __init__(self, module: torch.nn.Module, storage: Optional[torch.Tensor] = None, grad_storage: Optional[torch.Tensor] = None) -> None:
        self.params: List[torch.nn.Parameter] = [p for p in module.parameters() if p.requires_grad]
        self.shapes: List[Tuple[int, ...]] = [tuple(p.shape) for p in self.params]
        self.offsets: List[int] = []
        n = 0
        for p in self.params:
            self.offsets.append(n)
            n += p.numel()
        self.numel = n
        device = self.params[0].device if self.params else torch.device("cpu")
        if storage is None:
            storage = torch.empty(n, dtype=torch.float32, device=device)
        if grad_storage is None:
            grad_storage = torch.zeros(n, dtype=torch.float32, device=device)
        if storage.numel() != n or grad_storage.numel() != n:
            raise ValueError(f"flat storage has {storage.numel()} elements, module needs {n}")
        self.flat = storage
        self.grad = grad_storage
        with torch.no_grad():
            for p, off in zip(self.params, self.offsets):
                view = self.flat[off : off + p.numel()].view_as(p)
                view.copy_(p.data.to(view.dtype))
                p.data = view
                p.grad = self.grad[off : off + p.numel()].view_as(p)

    def views(self) -> List[torch.Tensor]:
        return [self.flat[o : o + p.numel()].view(s) for p, o, s in zip(self.params, self.offsets, self.shapes)]

    def zero_grad(self) -> None:
        self.grad.zero_()
        # autograd may have replaced .grad (e.g. set_to_none elsewhere): re-point
        for p, off in zip(self.params, self.offsets):
            if p.grad is None or p.grad.data_ptr() != self.grad[off:].data_ptr():
                p.grad = self.grad[off : off + p.numel()].view_as(p)

    def rebind(self) -> None:
        """Re-point parameters at the buffer (after ``load_state_dict`` replaced ``.data``)."""
        with torch.no_grad():
            for p, off in zip(self.params, self.offsets):
                view = self.flat[off : off + p.numel()].view_as(p)
                if p.data.data_ptr() != view.data_ptr():
                    view.copy_(p.data)
                    p.data = view
