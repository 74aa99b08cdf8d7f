"""Address parsing (parity: ``protocols/grpc/address.py:26-114``): IPv4/IPv6 ``host[:port]``
(no port → free ephemeral port) and ``unix:///abs/path`` Unix-domain sockets."""

from __future__ import annotations

import os
import socket
from ipaddress import ip_address
from typing import Optional


class AddressParser:
    """Parse a node address into host / port / family."""

    def __init__(self, address: str) -> None:
        self.host: Optional[str] = None
        self.port: Optional[int] = None
        self.is_v6: Optional[bool] = None
        self.unix_domain = False
        self._parse(address)

    def _parse(self, address: str) -> None:
        if address.startswith("unix://") and os.path.isabs(address[len("unix://") :]):
            self.unix_domain = True
            self.host = address
            return
        try:
            raw_host, sep, raw_port = address.rpartition(":")
            if sep and raw_host and not (raw_host.count(":") and not raw_host.startswith("[")):
                port = int(raw_port)
                if not 1 <= port <= 65535:
                    raise ValueError("Port number is invalid.")
                self.port = port
            else:
                raw_host = address
                with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
                    s.bind(("", 0))
                    self.port = s.getsockname()[1]
            self.host = raw_host.strip("[]")
            self.is_v6 = ip_address(self.host).version == 6
        except ValueError:
            self.host = self.port = self.is_v6 = None

    def get_parsed_address(self) -> str:
        if self.unix_domain:
            if self.host is None:
                raise ValueError("Unix domain address is invalid.")
            return self.host
        if self.host is None:
            raise ValueError("The address is invalid.")
        return f"[{self.host}]:{self.port}" if self.is_v6 else f"{self.host}:{self.port}"
