"""Thread-safe neighbour table (parity: ``protocols/neighbors.py:27-167``).

Entry: ``addr -> (channel|None, stub|None, last_beat_ts)``; "direct" means the stub is set.
Fixes: ``get_all`` copies under the lock.
"""

from __future__ import annotations

import threading
import time
from typing import Any, Dict, Tuple

from myfyp_amd.management.logger import logger
from myfyp_amd.utils.lockcheck import make_lock

NeighborEntry = Tuple[Any, Any, float]


class Neighbors:
    """Base neighbour table; transports implement ``connect``/``disconnect``/``refresh_or_add``."""

    def __init__(self, self_addr: str) -> None:
        self.self_addr = self_addr
        self.neis: Dict[str, NeighborEntry] = {}
        self.neis_lock = make_lock("Neighbors.neis", reentrant=True)

    def connect(self, addr: str, non_direct: bool = False, handshake_msg: bool = True) -> NeighborEntry:
        raise NotImplementedError

    def disconnect(self, addr: str, disconnect_msg: bool = True) -> None:
        raise NotImplementedError

    def temporary_stub(self, addr: str):
        """A stub for a one-off send to a non-neighbour (``create_connection=True``)."""
        return None

    def refresh_or_add(self, addr: str, time: float) -> None:
        with self.neis_lock:
            if addr in self.neis:
                ch, stub, _ = self.neis[addr]
                self.neis[addr] = (ch, stub, time)
                return
        self.add(addr, non_direct=True)

    def add(self, addr: str, *args, **kwargs) -> bool:
        """Add (or upgrade to direct) a neighbour. The transport handshake runs OUTSIDE the table
        lock so two peers connecting to each other concurrently cannot deadlock."""
        if addr == self.self_addr:
            logger.info(self.self_addr, "❌ Cannot add itself")
            return False
        non_direct = kwargs.get("non_direct", False)
        with self.neis_lock:
            existing = self.neis.get(addr)
            if existing is not None and (non_direct or existing[1] is not None):
                logger.debug(self.self_addr, f"❌ Cannot add duplicates. {addr} already exists.")
                return False
        try:
            entry = self.connect(addr, *args, **kwargs)
        except Exception as e:
            logger.error(self.self_addr, f"❌ Cannot add {addr}: {e}")
            return False
        with self.neis_lock:
            existing = self.neis.get(addr)
            if existing is not None and existing[1] is not None and entry[1] is None:
                return False  # a concurrent direct connect won
            self.neis[addr] = entry
        return True

    def remove(self, addr: str, *args, **kwargs) -> None:
        with self.neis_lock:
            if addr in self.neis:
                try:
                    self.disconnect(addr, *args, **kwargs)
                finally:
                    self.neis.pop(addr, None)

    def get(self, addr: str) -> NeighborEntry:
        with self.neis_lock:
            return self.neis[addr]

    def get_all(self, only_direct: bool = False) -> Dict[str, NeighborEntry]:
        with self.neis_lock:
            neis = dict(self.neis)
        if only_direct:
            return {k: v for k, v in neis.items() if v[1] is not None}
        return neis

    def exists(self, addr: str) -> bool:
        with self.neis_lock:
            return addr in self.neis

    def clear_neighbors(self) -> None:
        for addr in list(self.get_all()):
            self.remove(addr)

    @staticmethod
    def now() -> float:
        return time.time()
