#!/usr/bin/env python3
"""cProfile of the indexing hot path (bench.py's step) -> top functions by own time."""
import cProfile
import io
import os
import pstats
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("PROFILE_WITH_TORCH"):  # bench.py imports torch (distributed init) before indexing
    import torch  # noqa: F401,E402

from dmcp.app import App  # noqa: E402
from dmcp.config import Config  # noqa: E402
from dmcp.utils import synth  # noqa: E402

work = tempfile.mkdtemp(prefix="dmcp-prof-")
repo = os.path.join(work, "shop")
synth.java_spring_repo(repo, int(sys.argv[1]) if len(sys.argv) > 1 else 2000)
app = App(Config(db_path=os.path.join(work, "db"), git_clone_base_path=os.path.join(work, "c"),
                 enrich_backend="null", require_enrichment_for_analyze=False, parser_threads=16))
app.indexer.analyze_project(repo)
pr = cProfile.Profile()
stats = []
pr.enable()
for _ in range(5):
    stats.append(app.indexer.analyze_project(repo).stats)
pr.disable()
for s in stats:
    print({k: round(v, 1) for k, v in s.items()})
buf = io.StringIO()
pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(40)
print(buf.getvalue())
