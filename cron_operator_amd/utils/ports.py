"""Loopback ports to hand to a process that binds them later.

Binding port 0 and closing the socket returns a port from the kernel's ephemeral range, and
that range is exactly where every concurrent ``bind(0)`` server and every outgoing connection
draws from -- between the check and the child's own ``bind`` the port is often taken (a
rendezvous or probe port lost that race under parallel tests).  Ports here are drawn at random
*below* the ephemeral range and checked free, so the only competitors are other callers of
this function.
"""
from __future__ import annotations

import random
import socket


def _ephemeral_low() -> int:
    try:
        with open("/proc/sys/net/ipv4/ip_local_port_range") as fh:
            return int(fh.read().split()[0])
    except (OSError, ValueError, IndexError):
        return 32768


def free_port(host: str = "127.0.0.1", low: int = 15000, tries: int = 200) -> int:
    """A port on ``host`` that is free right now, outside the ephemeral range when possible."""
    high = _ephemeral_low()
    if high - low >= 1000:
        for _ in range(tries):
            port = random.randrange(low, high)
            with socket.socket() as s:
                try:
                    s.bind((host, port))
                except OSError:
                    continue
                return port
    with socket.socket() as s:  # a tiny or unknown non-ephemeral range: let the kernel choose
        s.bind((host, 0))
        return s.getsockname()[1]
