"""Heartbeat sender + failure detector (parity: ``protocols/heartbeater.py:33-113``)."""

from __future__ import annotations

import threading
import time
from typing import Optional

from myfyp_amd.communication.commands.message.heartbeat_command import heartbeater_cmd_name
from myfyp_amd.communication.protocols.client import Client
from myfyp_amd.communication.protocols.neighbors import Neighbors
from myfyp_amd.management.logger import logger
from myfyp_amd.settings import Settings


class Heartbeater(threading.Thread):
    """Broadcasts ``beat`` every ``HEARTBEAT_PERIOD``; evicts peers silent for ``HEARTBEAT_TIMEOUT``."""

    def __init__(self, self_addr: str, neighbors: Neighbors, client: Client) -> None:
        super().__init__(daemon=True, name=f"heartbeater-thread-{self_addr}")
        self._self_addr = self_addr
        self._neighbors = neighbors
        self._client = client
        self._terminate = threading.Event()

    def stop(self) -> None:
        self._terminate.set()

    def beat(self, nei: str, time: float) -> None:
        """Refresh (or add as non-direct) a neighbour on a received heartbeat."""
        if nei == self._self_addr:
            return
        self._neighbors.refresh_or_add(nei, time)

    def run(self, period: Optional[float] = None, timeout: Optional[float] = None) -> None:
        period = Settings.HEARTBEAT_PERIOD if period is None else period
        timeout = Settings.HEARTBEAT_TIMEOUT if timeout is None else timeout
        toggle = False
        while not self._terminate.is_set():
            t = time.time()
            if toggle:  # first period skipped (peers need one period to beat), then every period
                for nei, (_, _, last) in self._neighbors.get_all().items():
                    if t - last > timeout:
                        logger.info(self._self_addr, f"Heartbeat timeout for {nei} ({t - last:.2f}). Removing...")
                        self._neighbors.remove(nei)
            toggle = True
            self._client.broadcast(self._client.build_message(heartbeater_cmd_name, args=[str(time.time())]))
            self._terminate.wait(max(0.0, period - (time.time() - t)))
