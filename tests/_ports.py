"""A free TCP port on 127.0.0.1 for torchrun rendezvous (xdist workers run torchrun tests in
parallel: a pid-derived port can collide, a kernel-assigned one cannot while it is unbound)."""

import socket


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]
