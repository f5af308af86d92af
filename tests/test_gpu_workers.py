"""The GPU worker pool (dmcp/enrich/workers.py) with real GPU workers.

A one-GPU box cannot host one worker per GPU, so four worker processes share
cuda:0: the same code path as four GPUs (one child per device entry,
HIP_VISIBLE_DEVICES per child, hipGraph-captured decode, the grammar engine,
MultiFeed sessions), with the dealing, fault isolation and the device witness
checked on real MI355X workers instead of the CPU rehearsal of
tests/test_workers.py."""
import os
import signal
import time

import pytest

from conftest import make_app
from dmcp.enrich.types import EnrichmentInput
from dmcp.enrich.workers import GpuWorkerPool, ProcessLLMBackend
from dmcp.utils import synth

pytestmark = pytest.mark.gpu

N = 4
MODEL = {"preset": "tiny", "max_batch": 16, "max_rows": 32, "max_seq": 1024, "seed": 1}


def _inputs(n):
    return [EnrichmentInput("public class G%d { void a() {} void b() {} }" % i, f"co.g.G{i}", "java", "SERVICE",
                            ["a", "b", "c"][: 1 + i % 3]) for i in range(n)]


@pytest.fixture(scope="module")
def pool():
    p = GpuWorkerPool(["cuda:0"] * N, MODEL, start_timeout_s=600)
    yield p
    p.close()


def test_workers_report_the_device_and_the_kernel_library(pool):
    assert len(pool.workers) == N and len({w.info["pid"] for w in pool.workers}) == N
    for w in pool.workers:
        wit = w.info["witness"]
        assert "error" not in wit, wit
        assert wit["arch"].startswith("gfx950") and wit["cus"] >= 256 and wit["hbm_gib"] > 200, wit
        assert wit["hipops"].endswith("_hipops.so") and wit["hipops_abi"] > 0, wit
        assert w.info["gpu"] == "0"


def test_small_project_is_dealt_over_every_gpu_worker(tmp_path, pool):
    """A 33-class project (each GPU's share of 257 classes over 8) through a
    whole analyze_project: every class enriched, every worker used."""
    repo = tmp_path / "small"
    synth.java_spring_repo(str(repo), 32, base_package="co.acme.small", seed=3)
    be = ProcessLLMBackend(pool)
    before = dict(pool.per_worker_items)
    app = make_app(tmp_path, backend=be)
    t0 = time.time()
    r = app.indexer.analyze_project(str(repo))
    assert r.success and r.classes_analyzed == 33
    assert r.stats["enriched"] == 33 and r.stats["enrichFailed"] == 0
    assert app.repos.classes.find_unenriched_by_project_id(r.project_id) == []
    got = [pool.per_worker_items.get(i, 0) - before.get(i, 0) for i in range(N)]
    assert sum(got) == 33 and min(got) >= 33 // N, got
    st = be.stats()
    assert st["workers"] == N and st["decode_steps"] > 0 and st.get("graph_replays", 0) > 0, st
    # the device witness: kernel nodes of the replayed decode graphs (tiny: 2 layers, > 10 kernels a step)
    assert st.get("graph_kernels", 0) > 10 * st["graph_replays"], st
    app.db.close()  # the module-scoped pool outlives this app
    assert time.time() - t0 < 300


def test_killed_gpu_worker_is_isolated_and_replaced(pool):
    be = ProcessLLMBackend(pool)
    victim = pool.workers[2]
    old_pid = victim.proc.pid
    results, killed = {}, False
    for i, r in be.enrich_stream(_inputs(48), None):
        results[i] = r
        if not killed and victim.inflight:
            os.kill(old_pid, signal.SIGKILL)  # mid-stream, while its GPU process holds classes
            killed = True
    assert killed
    assert sorted(results) == list(range(48))
    failed = [r for r in results.values() if not r.success]
    assert failed and len(failed) <= MODEL["max_batch"] * 2, len(failed)  # only what the victim held
    assert all("worker died" in r.error_message for r in failed)
    # the next stream runs on a fresh GPU child in place of the dead one
    res = be.enrich_batch(_inputs(8), None)
    assert all(r.success for r in res), [r.error_message for r in res if not r.success]
    assert pool.workers[2].proc.pid != old_pid and pool.workers[2].alive
    assert "error" not in pool.workers[2].info["witness"]
