"""Resource monitor thread (parity: ``p2pfl/management/node_monitor.py:31-86``).

Reports CPU %, RAM %, network MB/s like the reference and, new for MI355X, the GPU's allocated /
reserved HBM (from the PyTorch-ROCm caching allocator, no extra tools needed). Fixes the
reference's blocking ``.run()`` start: callers use ``.start()``.
"""

from __future__ import annotations

import datetime
import threading
import time
from typing import Callable, Dict

from myfyp_amd.settings import Settings


class NodeMonitor(threading.Thread):
    """Periodically calls ``report(node, metric, value, time)``."""

    def __init__(self, node_addr: str, metric_report_callback: Callable[[str, str, float, datetime.datetime], None]) -> None:
        super().__init__(daemon=True, name=f"node-monitor-{node_addr}")
        self.node_addr = node_addr
        self.report_callback = metric_report_callback
        self.period = Settings.RESOURCE_MONITOR_PERIOD
        self._stop_event = threading.Event()
        self._last_net = None

    def stop(self) -> None:
        self._stop_event.set()

    def run(self) -> None:
        while not self._stop_event.is_set():
            now = datetime.datetime.now()
            for k, v in self.sample().items():
                self.report_callback(self.node_addr, k, v, now)
            self._stop_event.wait(self.period)

    def sample(self) -> Dict[str, float]:
        out: Dict[str, float] = {}
        try:
            import psutil

            out["cpu"] = psutil.cpu_percent()
            out["ram"] = psutil.virtual_memory().percent
            net = psutil.net_io_counters()
            t = time.time()
            if self._last_net is not None:
                dt = max(1e-6, t - self._last_net[2])
                out["net_in"] = (net.bytes_recv - self._last_net[0]) / dt / 1e6
                out["net_out"] = (net.bytes_sent - self._last_net[1]) / dt / 1e6
            self._last_net = (net.bytes_recv, net.bytes_sent, t)
        except Exception:
            pass
        try:
            import torch

            if torch.cuda.is_available():
                out["gpu_mem_allocated_gb"] = torch.cuda.memory_allocated() / 2**30
                out["gpu_mem_reserved_gb"] = torch.cuda.memory_reserved() / 2**30
        except Exception:
            pass
        return out
