"""Keras metric forwarding (parity: ``tensorflow/callbacks/keras_logger.py:27-62``): every batch's
logs become local metrics of the node. Usable as a Keras callback when Keras is installed (it only
needs the ``on_train_batch_end`` hook); here it is a plain object with the same method."""

from __future__ import annotations

from typing import Dict, Optional

from myfyp_amd.management.logger import logger


class FederatedLogger:
    def __init__(self, node_name: str) -> None:
        self.node_name = node_name
        self.step = 0

    def on_train_batch_end(self, batch: int, logs: Optional[Dict[str, float]] = None) -> None:
        for k, v in (logs or {}).items():
            logger.log_metric(self.node_name, k, float(v), step=self.step)
        self.step += 1
