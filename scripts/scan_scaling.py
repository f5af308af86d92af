#!/usr/bin/env python3
"""Native scan thread scaling + analyze phase breakdown on the current host.

    python scripts/scan_scaling.py [--classes 2000]
"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dmcp.parsers.base import native, to_parsed_project  # noqa: E402
from dmcp.utils import synth  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--classes", type=int, default=2000)
    a = ap.parse_args()
    work = tempfile.mkdtemp(prefix="dmcp-scan-")
    repo = os.path.join(work, "shop")
    synth.java_spring_repo(repo, a.classes, commit=False)
    n = native()
    out = {"cpus": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "scan_ms": {}}
    for threads in (1, 2, 4, 8, 16, 32):
        best = 1e9
        for _ in range(5):
            t0 = time.perf_counter()
            raw = n.scan_project(repo, "java", threads, "")
            best = min(best, time.perf_counter() - t0)
        out["scan_ms"][threads] = round(best * 1e3, 2)
    t0 = time.perf_counter()
    doc = json.loads(raw)
    t1 = time.perf_counter()
    pp = to_parsed_project(doc)
    t2 = time.perf_counter()
    out.update(json_decode_ms=round((t1 - t0) * 1e3, 2), convert_ms=round((t2 - t1) * 1e3, 2),
               json_bytes=len(raw))
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
