"""Spring-style 6-field cron scheduler for periodic sync.

Parity: ``ProjectSyncScheduler.java:22-60`` -- ``@Scheduled(cron =
"${sync.cron:0 0 2 * * *}")`` calling ``syncAllProjects`` when
``sync.enabled=true``.  Fields: second minute hour day-of-month month
day-of-week; supports ``*``, lists, ranges, steps, month/day names and ``?``.
"""
from __future__ import annotations

import logging
import threading
from datetime import datetime, timedelta
from typing import Callable, List, Optional, Set

LOG = logging.getLogger(__name__)

_MONTHS = {m: i + 1 for i, m in enumerate(
    ["JAN", "FEB", "MAR", "APR", "MAY", "JUN", "JUL", "AUG", "SEP", "OCT", "NOV", "DEC"])}
_DAYS = {d: i for i, d in enumerate(["SUN", "MON", "TUE", "WED", "THU", "FRI", "SAT"])}


def _field(spec: str, lo: int, hi: int, names=None) -> Set[int]:
    out: Set[int] = set()
    for part in spec.split(","):
        part = part.strip().upper()
        step = 1
        if "/" in part:
            part, s = part.split("/", 1)
            step = int(s)
        if part in ("*", "?", ""):
            a, b = lo, hi
        elif "-" in part:
            x, y = part.split("-", 1)
            a, b = _val(x, names), _val(y, names)
        else:
            a = _val(part, names)
            b = hi if step > 1 else a
        if a < lo or b > hi or a > b:
            raise ValueError(f"cron field out of range: {spec}")
        out.update(range(a, b + 1, step))
    return out


def _val(tok: str, names) -> int:
    if names and tok in names:
        return names[tok]
    return int(tok)


class CronExpression:
    def __init__(self, expr: str) -> None:
        parts = expr.split()
        if len(parts) == 5:  # tolerate classic 5-field cron (seconds = 0)
            parts = ["0"] + parts
        if len(parts) != 6:
            raise ValueError(f"cron expression must have 6 fields: {expr!r}")
        self.expr = expr
        self.seconds = _field(parts[0], 0, 59)
        self.minutes = _field(parts[1], 0, 59)
        self.hours = _field(parts[2], 0, 23)
        self.dom_any = parts[3] in ("*", "?")
        self.days = _field(parts[3], 1, 31)
        self.months = _field(parts[4], 1, 12, _MONTHS)
        self.dow_any = parts[5] in ("*", "?")
        # 0 and 7 are both Sunday; ranges such as 1-7 / 5-7 stay valid (Spring accepts them)
        self.dows = {d % 7 for d in _field(parts[5], 0, 7, _DAYS)}

    def _day_ok(self, t: datetime) -> bool:
        dow = (t.weekday() + 1) % 7  # Sunday = 0
        dom_ok = t.day in self.days
        dow_ok = dow in self.dows
        if self.dom_any and self.dow_any:
            return True
        if self.dom_any:
            return dow_ok
        if self.dow_any:
            return dom_ok
        return dom_ok or dow_ok

    def next_after(self, t: datetime) -> datetime:
        t = t.replace(microsecond=0) + timedelta(seconds=1)
        for _ in range(366 * 24 * 60 * 2):
            if t.month not in self.months:
                t = (t.replace(day=1, hour=0, minute=0, second=0) + timedelta(days=32)).replace(day=1)
                continue
            if not self._day_ok(t):
                t = t.replace(hour=0, minute=0, second=0) + timedelta(days=1)
                continue
            if t.hour not in self.hours:
                t = t.replace(minute=0, second=0) + timedelta(hours=1)
                continue
            if t.minute not in self.minutes:
                t = t.replace(second=0) + timedelta(minutes=1)
                continue
            if t.second not in self.seconds:
                t = t + timedelta(seconds=1)
                continue
            return t
        raise ValueError(f"cron expression never fires: {self.expr}")


class CronScheduler:
    def __init__(self, expr: str, job: Callable[[], None], clock: Callable[[], datetime] = datetime.now) -> None:
        self.cron = CronExpression(expr)
        self.job = job
        self.clock = clock
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.runs: List[datetime] = []

    def start(self) -> None:
        self._thread = threading.Thread(target=self._loop, name="sync-scheduler", daemon=True)
        self._thread.start()
        LOG.info("Sync scheduler started (%s)", self.cron.expr)

    def _loop(self) -> None:
        while not self._stop.is_set():
            now = self.clock()
            nxt = self.cron.next_after(now)
            if self._stop.wait(max(0.0, (nxt - now).total_seconds())):
                return
            self.runs.append(nxt)
            try:
                self.job()
            except Exception:  # a failing run must not kill the scheduler
                LOG.exception("Scheduled job failed")

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
