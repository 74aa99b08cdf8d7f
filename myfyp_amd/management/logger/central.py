"""Live cross-rank metric relay (parity: the reference's central Ray logger actor,
``p2pfl/management/logger/decorators/ray_logger.py:32-250``, which receives every node's metrics
while the experiment runs).

Here the job is one process per GPU and the peers of a rank share that process's logger. Every
metric stored on a rank > 0 is also queued and shipped to rank 0 over the control bus
(``Federation.bus``, a mailbox on the job's TCPStore) every ``Settings.CENTRAL_LOG_PERIOD``
seconds. Rank 0 inserts the records as they arrive, so ``logger.get_global_logs()`` /
``get_local_logs()`` and the web services there show the whole job live. Metrics stay where they
were produced too, and ``Federation.gather_logs`` at shutdown still merges everything everywhere.
Both stores dedupe: evaluation metrics keep one value per round, and local series skip
(step, value) pairs they already hold.
"""

from __future__ import annotations

import threading
from typing import Any, List, Optional, Tuple

from myfyp_amd.settings import Settings

Record = Tuple[str, str, int, str, float, Optional[int]]  # addr, exp, round, metric, value, step

RELAY_ADDR = "__central_logger__"
RELAY_KIND = "logs"


class CentralLogRelay:
    """Installed by ``Federation.finalize`` when the job has more than one rank."""

    def __init__(self, fed, logger) -> None:
        self.fed, self.logger = fed, logger
        self.rank = fed.rank
        self._out: List[Record] = []
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self.sent = 0
        self.received = 0
        self._thread: Optional[threading.Thread] = None
        if self.rank != 0:
            logger.add_metric_listener(self._on_metric)
            self._thread = threading.Thread(target=self._flush_loop, name=f"central-log-{self.rank}", daemon=True)
            self._thread.start()

    # ---------------------------------------------------------------- ranks > 0
    def _on_metric(self, addr: str, exp: str, rnd: int, metric: str, value: Any, step: Optional[int]) -> None:
        try:
            v = float(value)
        except (TypeError, ValueError):
            return
        with self._lock:
            self._out.append((addr, exp, int(rnd), metric, v, None if step is None else int(step)))

    def flush(self) -> None:
        with self._lock:
            batch, self._out = self._out, []
        bus = self.fed.bus
        if batch and bus is not None and 0 in self.fed.members:
            bus.send(0, RELAY_ADDR, RELAY_KIND, {"rank": self.rank, "records": [list(r) for r in batch]})
            self.sent += len(batch)

    def _flush_loop(self) -> None:
        while not self._stop.wait(float(Settings.CENTRAL_LOG_PERIOD)):
            try:
                self.flush()
            except Exception:  # the bus may be closing at shutdown
                pass

    # ---------------------------------------------------------------- rank 0
    def ingest(self, msg: dict) -> None:
        records = msg.get("records") or []
        self.logger.ingest_records([tuple(r) for r in records])
        self.received += len(records)

    def stop(self) -> None:
        self._stop.set()
        if self.rank != 0:
            self.logger.remove_metric_listener(self._on_metric)
            try:
                self.flush()
            except Exception:
                pass
