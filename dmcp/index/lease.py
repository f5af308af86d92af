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
        self.took_over_expired = False
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.held = False

    def acquire(self) -> "ProjectLease":
        now = self.clock()
        prev_owner, prev_until = self.projects.lease_of(self.project_id)
        if not self.projects.try_acquire_lease(self.project_id, self.owner, self.ttl_s, now):
            raise DomainError(f"Project {self.name} is already being processed", "PROJECT_BUSY")
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
        while not self._stop.wait(period):
            try:
                if not self.projects.renew_lease(self.project_id, self.owner, self.clock() + self.ttl_s):
                    self.lost = True
                    LOG.error("Project %s: lease lost to another process", self.name)
                    return
            except Exception as e:  # a busy database: try again next period
                LOG.warning("Project %s: lease heartbeat failed: %s", self.name, e)

    def check(self) -> None:
        """Raises ``LEASE_LOST`` when the heartbeat found the lease taken."""
        if self.lost:
            raise DomainError(f"Project {self.name}: lease lost to another process", "LEASE_LOST")

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
