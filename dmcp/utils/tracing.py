"""Lightweight tracing / metrics.

The reference has no tracer: it logs phase counters at INFO and one wall-clock
line per GraalJS run.  Here every pipeline phase and every MCP/REST call is a
:class:`span`; durations feed process-wide counters/histograms (exposed by
``GET /metrics`` in Prometheus text format and the ``stats`` MCP-less CLI) and,
when ``DMCP_TRACE_FILE`` is set, are appended as JSON lines.
"""
from __future__ import annotations

import bisect
import json
import logging
import os
import threading
import time
from contextlib import contextmanager
from typing import Dict, Iterator, List, Optional

LOG = logging.getLogger("dmcp.trace")

_BUCKETS_MS = [0.1, 0.25, 0.5, 1, 2.5, 5, 10, 25, 50, 100, 250, 500, 1000, 2500, 5000, 10000, 30000, 60000]


class Metrics:
    def __init__(self) -> None:
        self._lock = threading.Lock()
        self.counters: Dict[str, float] = {}
        self.hist: Dict[str, List[int]] = {}
        self.hist_sum: Dict[str, float] = {}
        self.samples: Dict[str, List[float]] = {}

    def inc(self, name: str, value: float = 1.0) -> None:
        with self._lock:
            self.counters[name] = self.counters.get(name, 0.0) + value

    def observe_ms(self, name: str, ms: float) -> None:
        with self._lock:
            h = self.hist.get(name)
            if h is None:
                h = self.hist[name] = [0] * (len(_BUCKETS_MS) + 1)
                self.hist_sum[name] = 0.0
                self.samples[name] = []
            h[bisect.bisect_left(_BUCKETS_MS, ms)] += 1
            self.hist_sum[name] += ms
            s = self.samples[name]
            if len(s) < 10000:
                s.append(ms)

    def percentile(self, name: str, q: float) -> Optional[float]:
        with self._lock:
            s = sorted(self.samples.get(name, ()))
        if not s:
            return None
        k = min(len(s) - 1, max(0, int(round(q * (len(s) - 1)))))
        return s[k]

    def prometheus(self) -> str:
        lines = []
        with self._lock:
            for k, v in sorted(self.counters.items()):
                n = _metric_name(k)
                lines.append(f"# TYPE {n} counter")
                lines.append(f"{n} {v}")
            for k, h in sorted(self.hist.items()):
                n = _metric_name(k) + "_ms"
                lines.append(f"# TYPE {n} histogram")
                acc = 0
                for b, c in zip(_BUCKETS_MS, h):
                    acc += c
                    lines.append(f'{n}_bucket{{le="{b}"}} {acc}')
                acc += h[-1]
                lines.append(f'{n}_bucket{{le="+Inf"}} {acc}')
                lines.append(f"{n}_sum {self.hist_sum[k]}")
                lines.append(f"{n}_count {acc}")
        return "\n".join(lines) + "\n"

    def snapshot(self) -> dict:
        with self._lock:
            names = list(self.hist)
            counters = dict(self.counters)
        out = {"counters": counters, "latencyMs": {}}
        for n in names:
            out["latencyMs"][n] = {"p50": self.percentile(n, 0.5), "p99": self.percentile(n, 0.99),
                                   "count": sum(self.hist[n])}
        return out

    def reset(self) -> None:
        with self._lock:
            self.counters.clear()
            self.hist.clear()
            self.hist_sum.clear()
            self.samples.clear()


def _metric_name(k: str) -> str:
    return "dmcp_" + "".join(c if c.isalnum() else "_" for c in k)


METRICS = Metrics()
_trace_lock = threading.Lock()


@contextmanager
def span(name: str, sink: Optional[Dict[str, float]] = None, **attrs) -> Iterator[dict]:
    """Times a block; records ms into METRICS, ``sink[name]`` and the trace file."""
    t0 = time.perf_counter()
    info: dict = dict(attrs)
    err = None
    try:
        yield info
    except BaseException as e:
        err = e
        raise
    finally:
        ms = (time.perf_counter() - t0) * 1e3
        METRICS.observe_ms(name, ms)
        if err is not None:
            METRICS.inc(name + ".errors")
        if sink is not None:
            sink[name] = sink.get(name, 0.0) + ms
        path = os.environ.get("DMCP_TRACE_FILE")
        if path:
            rec = {"ts": time.time(), "span": name, "ms": round(ms, 3), **info}
            if err is not None:
                rec["error"] = repr(err)
            with _trace_lock:
                with open(path, "a", encoding="utf-8") as f:
                    f.write(json.dumps(rec, default=str) + "\n")
        LOG.debug("span %s %.2f ms %s", name, ms, info)
