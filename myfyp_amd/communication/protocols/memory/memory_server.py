"""In-memory server (parity: ``memory/memory_server.py:30-222``).

Receiving needs no thread or socket: registering the protocol under its address is the whole
"server". Dispatch (dedup → TTL relay → command) is the protocol's transport-independent
``handle_message``/``handle_weights``.
"""

from __future__ import annotations

from myfyp_amd.communication.protocols.memory.server_singleton import ServerRegistry
from myfyp_amd.management.logger import logger


class InMemoryServer:
    def __init__(self, protocol) -> None:
        self.protocol = protocol

    @property
    def addr(self) -> str:
        return self.protocol.addr

    def start(self) -> None:
        ServerRegistry.register(self.addr, self.protocol)
        logger.info(self.addr, f"InMemoryServer started at {self.addr}")

    def stop(self) -> None:
        ServerRegistry.unregister(self.addr)
        logger.info(self.addr, f"InMemoryServer stopped at {self.addr}")

    def is_running(self) -> bool:
        return ServerRegistry.get(self.addr) is self.protocol
