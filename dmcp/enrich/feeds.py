"""Work feeds of the local enrichment engine (torch-free: the GPU worker
process and its model-free rehearsal engine import them before any model).
"""
from __future__ import annotations

import threading
from collections import deque
from typing import Any, Deque, Iterable, List, Tuple

from .types import EnrichmentInput


class IterFeed:
    """A feed over a (possibly lazy) iterable of ``(key, EnrichmentInput)``:
    items are pulled only when the engine has room for them, so a producer
    that reads sources on demand never runs ahead of the GPU."""

    def __init__(self, items: Iterable[Tuple[Any, EnrichmentInput]]) -> None:
        self._it = iter(items)
        self.done = False

    def take(self, n: int, wait: bool = False) -> List[Tuple[Any, EnrichmentInput]]:
        out = []
        while len(out) < n and not self.done:
            try:
                out.append(next(self._it))
            except StopIteration:
                self.done = True
        return out


class QueueFeed:
    """A thread-safe feed another thread fills (the GPU worker's pipe reader):
    ``put`` items, ``close`` when no more will come.  ``take(wait=True)``
    blocks until an item arrives or the feed is closed."""

    def __init__(self) -> None:
        self._q: Deque[Tuple[Any, EnrichmentInput]] = deque()
        self._cv = threading.Condition()
        self._closed = False

    def put(self, items: Iterable[Tuple[Any, EnrichmentInput]]) -> None:
        with self._cv:
            self._q.extend(items)
            self._cv.notify_all()

    def close(self) -> None:
        with self._cv:
            self._closed = True
            self._cv.notify_all()

    @property
    def done(self) -> bool:
        with self._cv:
            return self._closed and not self._q

    def take(self, n: int, wait: bool = False) -> List[Tuple[Any, EnrichmentInput]]:
        with self._cv:
            if wait:
                while not self._q and not self._closed:
                    self._cv.wait(0.5)
            out = []
            while self._q and len(out) < n:
                out.append(self._q.popleft())
            return out




class MultiFeed:
    """Several sessions' classes as ONE feed for one engine (the GPU worker
    serving several projects at once): items ``((sid, key), input, readme)``,
    taken round-robin over the sessions that have some, so every project
    progresses.  ``done`` only after :meth:`shutdown`."""

    def __init__(self) -> None:
        self._cv = threading.Condition()
        self._q: "dict[int, Deque[Tuple[Any, EnrichmentInput]]]" = {}
        self._readme: "dict[int, Any]" = {}
        self._order: Deque[int] = deque()
        self._ended: set = set()   # sessions whose ``end`` arrived: dropped once drained
        self._shutdown = False

    def begin(self, sid: int, readme) -> None:
        with self._cv:
            self._q[sid] = deque()
            self._readme[sid] = readme
            self._order.append(sid)

    def put(self, sid: int, items: Iterable[Tuple[Any, EnrichmentInput]]) -> None:
        with self._cv:
            q = self._q.get(sid)
            if q is None:
                return
            q.extend(items)
            self._cv.notify_all()

    def end(self, sid: int) -> None:
        """No more items of ``sid`` (queued ones are still taken)."""
        with self._cv:
            q = self._q.get(sid)
            if q is None:
                return
            if q:
                self._ended.add(sid)  # its queued items are still taken; dropped when drained
            else:
                self._drop(sid)

    def _drop(self, sid: int) -> None:
        self._q.pop(sid, None)
        self._readme.pop(sid, None)
        self._ended.discard(sid)
        try:
            self._order.remove(sid)
        except ValueError:
            pass

    def shutdown(self) -> None:
        with self._cv:
            self._shutdown = True
            self._cv.notify_all()

    @property
    def done(self) -> bool:
        with self._cv:
            return self._shutdown and not any(self._q.values())

    def take(self, n: int, wait: bool = False) -> List[tuple]:
        with self._cv:
            if wait:
                while not any(self._q.values()) and not self._shutdown:
                    self._cv.wait(0.5)
            out: List[tuple] = []
            while len(out) < n:
                progressed = False
                for sid in list(self._order):
                    q = self._q.get(sid)
                    if q:
                        key, inp = q.popleft()
                        out.append(((sid, key), inp, self._readme[sid]))
                        progressed = True
                        if not q and sid in self._ended:
                            self._drop(sid)
                        if len(out) >= n:
                            break
                if not progressed:
                    break
            return out

    def sessions(self) -> int:
        """Sessions still held (begun and not yet ended-and-drained)."""
        with self._cv:
            return len(self._q)
