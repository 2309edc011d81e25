"""Device workspaces (Solver handles and their buffers) kept between the functional
calls of the reference API — fit / backward_pass with arbitrary closures (the tiles
handle) and linearize_dynamics on the device — so that an MPC loop calling them
allocates no device workspace per call (include/ilqr.h: "hot calls never allocate").

A call checks its workspace OUT of the cache and back in when done, so two threads
calling with the same shape at once never share one (the second builds its own; the
surplus is closed on check-in). At most MAX_CACHED workspaces stay cached, the least
recently used evicted and closed at once."""
from __future__ import annotations

import contextlib
import threading

MAX_CACHED = 8
_CACHE: dict = {}
_LOCK = threading.Lock()


@contextlib.contextmanager
def workspace(key, factory):
    """`with workspace(key, factory) as s`: the cached workspace `key` (factory() on a
    miss), exclusively this caller's until the block ends."""
    with _LOCK:
        s = _CACHE.pop(key, None)
    if s is None:
        s = factory()
    try:
        yield s
    finally:
        evicted = []
        with _LOCK:
            if key in _CACHE:
                evicted.append(s)
            else:
                _CACHE[key] = s
                while len(_CACHE) > MAX_CACHED:
                    evicted.append(_CACHE.pop(next(iter(_CACHE))))
        for e in evicted:
            e.close()


def clear():
    """Close every cached workspace."""
    with _LOCK:
        ss = list(_CACHE.values())
        _CACHE.clear()
    for s in ss:
        s.close()


def size() -> int:
    return len(_CACHE)
