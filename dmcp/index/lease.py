"""Cross-process project lease: one analyze / sync / rebuild / resume per project.

The reference guards a project with its status state machine only
(``ProjectStateMachine.java:34-70``: ANALYZING -> ANALYZING is illegal) and a
check-then-act status read, which two processes can interleave; a crashed
analysis left the project wedged in ANALYZING for ever.  Here
every long operation first takes a lease on the project row
(:meth:`ProjectRepository.try_acquire_lease`: one conditional UPDATE), a
daemon thread heartbeats it every ``ttl / 3`` seconds while the operation
runs, and the operation releases it at the end.  A second process asking for
the same project gets ``PROJECT_BUSY``; a holder that died stops
heartbeating, its lease runs out after ``ttl`` seconds, and only then may
another process recover the project's ANALYZING / SYNCING status.

A holder whose heartbeat cannot renew (a long write transaction holding the
SQLite write lock, a database outage) knows when its last renewal runs out
(``valid_until``): past it :meth:`ProjectLease.check` fails with
``LEASE_LOST`` even though no other owner was seen yet, so the operation
stops writing instead of racing whoever takes the project over -- and it
never marks the project ERROR (that status is no longer its to write).
"""
from __future__ import annotations

import logging
import os
import socket
import threading
import time
import uuid
from typing import Callable, Optional

from ..utils.errors import DomainError

LOG = logging.getLogger(__name__)


def new_owner_id() -> str:
    """host:pid:random -- unique per operation, readable in the projects row."""
    return f"{socket.gethostname()}:{os.getpid()}:{uuid.uuid4().hex[:8]}"


class ProjectLease:
    """``with ProjectLease(repo, project_id, ttl_s):`` -- raises
    ``DomainError(PROJECT_BUSY)`` when another live operation holds it."""

    def __init__(self, projects, project_id: str, ttl_s: float = 60.0, name: Optional[str] = None,
                 clock: Callable[[], float] = time.time) -> None:
        self.projects = projects
        self.project_id = project_id
        self.ttl_s = max(1.0, float(ttl_s))
        self.name = name or project_id
        self.owner = new_owner_id()
        self.clock = clock
        self.lost = False
        self.valid_until = 0.0  # the lease is ours until then (last successful acquire / renewal)
        self.took_over_expired = False
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.held = False

    def acquire(self) -> "ProjectLease":
        now = self.clock()
        prev_owner, prev_until = self.projects.lease_of(self.project_id)
        if not self.projects.try_acquire_lease(self.project_id, self.owner, self.ttl_s, now):
            raise DomainError(f"Project {self.name} is already being processed", "PROJECT_BUSY")
        self.valid_until = now + self.ttl_s
        # a previous holder that never released: crashed (its lease ran out)
        self.took_over_expired = prev_owner is not None and prev_owner != self.owner
        if self.took_over_expired:
            LOG.warning("Project %s: lease of %s expired at %s; taking over", self.name, prev_owner, prev_until)
        self.held = True
        self._thread = threading.Thread(target=self._heartbeat, name=f"lease-{self.project_id[:8]}", daemon=True)
        self._thread.start()
        return self

    def _heartbeat(self) -> None:
        period = self.ttl_s / 3.0
        wait = period
        while not self._stop.wait(wait):
            try:
                until = self.clock() + self.ttl_s
                if not self.projects.renew_lease(self.project_id, self.owner, until):
                    self.lost = True
                    LOG.error("Project %s: lease lost to another process", self.name)
                    return
                self.valid_until = until
                wait = period
            except Exception as e:  # a busy database: retry soon -- the lease runs out at valid_until
                LOG.warning("Project %s: lease heartbeat failed: %s", self.name, e)
                wait = min(period, 0.5)

    def expired(self) -> bool:
        """True once the last renewal ran out (another process may own it now)."""
        return self.held and self.clock() > self.valid_until

    def check(self) -> None:
        """Raises ``LEASE_LOST`` when the heartbeat found the lease taken, or
        could not renew it before it ran out."""
        if self.lost:
            raise DomainError(f"Project {self.name}: lease lost to another process", "LEASE_LOST")
        if self.expired():
            raise DomainError(f"Project {self.name}: lease expired (not renewed since "
                              f"{self.valid_until - self.ttl_s:.0f})", "LEASE_LOST")

    def is_lost(self, error: Optional[BaseException] = None) -> bool:
        """Whether an operation that failed with ``error`` no longer owns the
        project (its status then belongs to the new owner)."""
        if isinstance(error, DomainError) and error.error_code == "LEASE_LOST":
            return True
        return self.lost or self.expired()

    def release(self) -> None:
        if not self.held:
            return
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5.0)
        self.held = False
        try:
            self.projects.release_lease(self.project_id, self.owner)
        except Exception as e:  # it expires on its own
            LOG.warning("Project %s: lease release failed: %s", self.name, e)

    def __enter__(self) -> "ProjectLease":
        return self.acquire()

    def __exit__(self, *exc) -> bool:
        self.release()
        return False
