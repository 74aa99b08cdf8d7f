"""Process-wide address registry of the in-memory transport (parity: ``memory/server_singleton.py``).

The reference keeps a plain dict in a singleton whose ``stop()`` wipes every entry
(``memory_server.py:90-94``). Here the table is lock-protected and a node removes
only its own entry. Cross-rank mailboxes (``parallel/federation.py``) deliver into it too.
"""

from __future__ import annotations

import threading
from typing import Any, Dict, Optional


class ServerRegistry:
    """``addr → protocol`` table."""

    _servers: Dict[str, Any] = {}
    _lock = threading.Lock()

    @classmethod
    def register(cls, addr: str, proto: Any) -> None:
        with cls._lock:
            if addr in cls._servers and cls._servers[addr] is not proto:
                raise ValueError(f"Address {addr} already in use")
            cls._servers[addr] = proto

    @classmethod
    def unregister(cls, addr: str) -> None:
        with cls._lock:
            cls._servers.pop(addr, None)

    @classmethod
    def get(cls, addr: str) -> Optional[Any]:
        with cls._lock:
            return cls._servers.get(addr)

    @classmethod
    def reset(cls) -> None:
        with cls._lock:
            cls._servers.clear()


# reference name
ServerSingleton = ServerRegistry
