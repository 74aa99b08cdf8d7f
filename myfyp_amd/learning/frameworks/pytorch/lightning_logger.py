"""``FederatedLogger`` (parity: ``pytorch/lightning_logger.py:26-65``).

In the reference, Lightning calls ``log_metrics(metrics, step)`` and the logger forwards every
value as a *local* (per-step) metric of the node. The same object works for any training loop:
call ``log_metrics`` with a dict and a step. ``TorchLearner`` logs ``train_loss`` itself (once per
epoch, reduced on the device, instead of a host sync per step).
"""

from __future__ import annotations

from typing import Any, Dict, Optional

from myfyp_amd.management.logger import logger


class FederatedLogger:
    def __init__(self, addr: str) -> None:
        self.self_name = addr

    @property
    def name(self) -> str:
        return "p2pfl"

    @property
    def version(self) -> Optional[int]:
        return None

    def log_hyperparams(self, params: Dict[str, Any]) -> None:
        """Hyper-parameters are not stored (reference: no-op)."""

    def log_metrics(self, metrics: Dict[str, float], step: int) -> None:
        for k, v in metrics.items():
            logger.log_metric(self.self_name, k, float(v), step=step)

    def save(self) -> None:
        """Nothing buffered (reference: no-op)."""

    def finalize(self, status: str) -> None:
        """Nothing to flush (reference: no-op)."""


__all__ = ["FederatedLogger"]
