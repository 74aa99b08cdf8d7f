"""Resource monitor thread (parity: ``p2pfl/management/node_monitor.py:31-86``).

Reports CPU %, RAM % and network MB/s, like the reference. New for MI355X:
- device telemetry through AMD SMI or sysfs (``device_telemetry.py``): power, GFX and HBM
  activity, HBM used and total, temperature;
- the caching allocator's allocated / reserved HBM;
- weight-plane traffic from the federation's ``CommStats``: MB moved and MB/s per collective kind,
  and the last latency in µs. The side-stream FedAvg pipeline is timed with HIP events.

It also fixes the reference's blocking ``.run()`` start: callers use
``.start()``.
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
        self._last_comm: Dict[str, tuple] = {}
        self._telemetry = None

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
                if self._telemetry is None:
                    from myfyp_amd.management.device_telemetry import DeviceTelemetry

                    self._telemetry = DeviceTelemetry(torch.cuda.current_device())
                out.update(self._telemetry.sample())
        except Exception:
            pass
        out.update(self.comm_sample())
        return out

    def comm_sample(self) -> Dict[str, float]:
        """Per collective kind: cumulative MB, MB/s since the previous sample, last latency (µs)."""
        from myfyp_amd.parallel.federation import Federation

        fed = Federation._instance
        if fed is None or getattr(fed, "comm", None) is None:
            return {}
        out: Dict[str, float] = {}
        t = time.time()
        snap = fed.comm.snapshot()
        for kind, st in snap.items():
            mb = st["bytes"] / 1e6
            out[f"comm_{kind}_mb"] = mb
            prev = self._last_comm.get(kind)
            if prev is not None and t > prev[1]:
                out[f"comm_{kind}_mb_s"] = (mb - prev[0]) / (t - prev[1])
            self._last_comm[kind] = (mb, t)
            if st["us_last"] is not None:
                out[f"comm_{kind}_us"] = st["us_last"]
        return out
