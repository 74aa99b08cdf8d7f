"""``SCAFFOLDCallback`` at its reference path (``pytorch/callbacks/scaffold_callback.py:32-150``).

Unlike the reference (whose correction is a no-op: it edits detached ``state_dict`` tensors,
SURVEY §2.11 #7), the correction ``g + c − c_i`` is applied inside the fused optimizer kernel.
"""

from myfyp_amd.learning.frameworks.torch.callbacks import SCAFFOLDCallback

__all__ = ["SCAFFOLDCallback"]
