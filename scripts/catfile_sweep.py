"""Blob-read concurrency sweep: ``read_blobs`` over a 2,000-class synthetic
repository with loose objects and after ``git gc`` (packed), 1..8 processes."""
import subprocess
import sys
import tempfile
import time

sys.path.insert(0, ".")
from dmcp.index.git import GitClient  # noqa: E402
from dmcp.index.source import list_tree, read_blobs  # noqa: E402
from dmcp.utils import synth  # noqa: E402


def sweep(tag, g, d, shas):
    for procs in (1, 2, 4, 8):
        best = 1e9
        for _ in range(3):
            t0 = time.perf_counter()
            r = read_blobs(g, d, shas, 0, procs)
            best = min(best, time.perf_counter() - t0)
        print(f"{tag} procs={procs} best_ms={best * 1e3:.1f} n={len(r)}", flush=True)


with tempfile.TemporaryDirectory() as t:
    synth.java_spring_repo(f"{t}/src", 2000)
    g = GitClient(f"{t}/c")
    d = f"{t}/b"
    subprocess.run(["git", "clone", "-q", "--bare", "--shared", f"{t}/src", d], check=True)
    shas = [x[1] for x in list_tree(g, d, "HEAD")]
    sweep("loose", g, d, shas)
    subprocess.run(["git", "-C", f"{t}/src", "gc", "-q"], check=True)
    sweep("packed", g, d, shas)
