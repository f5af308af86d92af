"""Native scan thread scaling on a 2,000-class synthetic repository: the
in-memory ``scan_sources`` path with 1..32 workers, plus the Python-side
decode (json.loads + ParsedProject) the indexer runs after it."""
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dmcp.index.git import GitClient  # noqa: E402
from dmcp.models.domain import RepositoryUrl  # noqa: E402
from dmcp.parsers.base import native, to_parsed_project  # noqa: E402
from dmcp.utils import synth  # noqa: E402

with tempfile.TemporaryDirectory() as t:
    synth.java_spring_repo(f"{t}/src", int(sys.argv[1]) if len(sys.argv) > 1 else 2000)
    tree = GitClient(f"{t}/c").snapshot(RepositoryUrl.of(f"{t}/src"), "main")
    items = list(tree.files.items())
    n = native()
    print(f"files={len(items)} bytes={sum(len(b) for _, b in items)} cpus={os.cpu_count()}", flush=True)
    for th in (1, 2, 4, 8, 16, 32):
        best, inner = 1e9, 0
        for _ in range(5):
            t0 = time.perf_counter()
            raw = n.scan_sources(items, "java", th, "")
            dt = time.perf_counter() - t0
            if dt < best:
                best, inner = dt, json.loads(raw)["stats"]["elapsedUs"]
        print(f"threads={th} scan_sources_ms={best * 1e3:.1f} native_scan_ms={inner / 1e3:.1f}", flush=True)
    t0 = time.perf_counter()
    doc = json.loads(raw)
    t1 = time.perf_counter()
    pp = to_parsed_project(doc)
    t2 = time.perf_counter()
    pp.build_graph()
    t3 = time.perf_counter()
    print(f"json_ms={(t1 - t0) * 1e3:.1f} convert_ms={(t2 - t1) * 1e3:.1f} graph_ms={(t3 - t2) * 1e3:.1f} "
          f"doc_kb={len(raw) // 1024}", flush=True)
