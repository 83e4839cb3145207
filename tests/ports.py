"""Rendezvous ports for multi-process tests.

A port taken from the kernel's ephemeral range (bind to 0, then close) can be handed out again to
the client side of another connection before the store listens on it (EADDRINUSE seen on the GPU
box between two relay-test variants).  Ports are drawn instead below the ephemeral range
(/proc/sys/net/ipv4/ip_local_port_range starts at 32768), checked bindable, never reused in-process.
"""

from __future__ import annotations

import os
import random
import socket

_used: set[int] = set()
_rng = random.Random(os.getpid() ^ int.from_bytes(os.urandom(4), "little"))


def free_port(lo: int = 20000, hi: int = 32000) -> int:
    for _ in range(200):
        p = _rng.randrange(lo, hi)
        if p in _used:
            continue
        with socket.socket() as s:
            try:
                s.bind(("127.0.0.1", p))
            except OSError:
                continue
        _used.add(p)
        return p
    raise RuntimeError("no free rendezvous port in [%d, %d)" % (lo, hi))
