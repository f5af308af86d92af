"""One worker process per GPU (dmcp/enrich/workers.py), rehearsed on the CPU:
two real child processes run the tiny model on the fp32 reference ops.

Covers the service path of the local enrichment backend: work spread over
every worker from one queue, results in input order through
``enrich_batch``, a killed worker isolated (its classes fail, the others
finish; a fresh child replaces it at the next stream), and a whole
``analyze_project`` streaming every class through the pool."""
import json
import os
import signal
import time

import pytest

from conftest import make_app
from dmcp.enrich.types import EnrichmentInput
from dmcp.enrich.workers import GpuWorkerPool, ProcessLLMBackend, recv_frame, send_frame
from dmcp.utils import synth

MODEL = {"preset": "tiny", "max_batch": 4, "max_rows": 16, "max_seq": 768, "seed": 1}


def _inputs(n):
    return [EnrichmentInput("public class S%d { void a() {} void b() {} }" % i, f"co.x.S{i}", "java", "SERVICE",
                            ["a", "b", "c"][: 1 + i % 3]) for i in range(n)]


@pytest.fixture(scope="module")
def pool():
    # one OpenMP thread per worker: the tiny model needs no more, and spin-
    # waiting OpenMP teams crawl when the test run shares the cores (xdist)
    p = GpuWorkerPool(["cpu", "cpu"], MODEL, engine={"use_graphs": False}, start_timeout_s=300,
                      env_extra={"OMP_NUM_THREADS": "1"})
    yield p
    p.close()


def test_frames_roundtrip():
    import io
    buf = io.BytesIO()
    send_frame(buf, {"op": "x", "v": [1, "é"]})
    send_frame(buf, {"op": "y"})
    buf.seek(0)
    assert recv_frame(buf) == {"op": "x", "v": [1, "é"]} and recv_frame(buf) == {"op": "y"}
    assert recv_frame(buf) is None


def test_work_is_spread_and_results_keep_input_order(pool):
    be = ProcessLLMBackend(pool)
    before = dict(pool.per_worker_items)
    inputs = _inputs(14)
    res = be.enrich_batch(inputs, "A shop README. " * 8)
    assert [r.full_class_name for r in res] == [i.full_class_name for i in inputs]
    assert all(r.success for r in res), [r.error_message for r in res if not r.success]
    for r, inp in zip(res, inputs):
        assert [m.method_name for m in r.methods] == inp.method_names
    got = {k: pool.per_worker_items.get(k, 0) - before.get(k, 0) for k in (0, 1)}
    assert got[0] > 0 and got[1] > 0 and got[0] + got[1] == 14
    st = be.stats()
    assert st["workers"] == 2 and st["prefills"] == 14 and st["decode_steps"] > 0
    assert len({w.info["pid"] for w in pool.workers}) == 2 and all(w.info["pid"] != os.getpid() for w in pool.workers)


def test_abandoned_stream_leaves_the_workers_serving(pool):
    """A caller that stops consuming a stream (an exception while applying a
    reply) must not leave a worker waiting for more of that session: the
    next stream completes on the same processes."""
    be = ProcessLLMBackend(pool)
    pids = [w.proc.pid for w in pool.workers]
    gen = be.enrich_stream(_inputs(12), None)
    next(gen)
    gen.close()  # GeneratorExit inside the pool's stream
    t0 = time.time()
    res = be.enrich_batch(_inputs(6), None)
    assert all(r.success for r in res), [r.error_message for r in res if not r.success]
    assert [w.proc.pid for w in pool.workers] == pids and pool.deaths == 0
    assert time.time() - t0 < 120


def test_late_eof_of_a_replaced_worker_is_ignored(pool):
    """Events carry the worker object: the EOF of a child that was already
    replaced (killed for a hang, its reader thread ending later) must not
    mark the fresh worker at the same index dead."""
    class Ghost:  # a worker object no longer in the pool, at index 0
        index = 0
    cur = pool.workers[0]
    pool._on_frame(Ghost(), None)
    res = ProcessLLMBackend(pool).enrich_batch(_inputs(4), None)
    assert all(r.success for r in res), [r.error_message for r in res if not r.success]
    assert pool.workers[0] is cur and cur.alive


def test_killed_worker_is_isolated_and_replaced(pool):
    be = ProcessLLMBackend(pool)
    inputs = _inputs(16)
    victim = pool.workers[1]
    old_pid = victim.proc.pid
    results = {}
    killed = False
    for i, r in be.enrich_stream(inputs, None):
        results[i] = r
        if not killed and victim.inflight:
            os.kill(old_pid, signal.SIGKILL)  # mid-stream, while it holds classes
            killed = True
    assert killed, "the victim never held classes when a reply arrived"
    assert sorted(results) == list(range(16))
    failed = [r for r in results.values() if not r.success]
    assert failed and all("worker died" in r.error_message for r in failed)
    assert sum(r.success for r in results.values()) >= 16 - pool.capacity
    assert pool.deaths >= 1
    # the next stream runs on a FRESH child in place of the dead one
    res = be.enrich_batch(_inputs(4), None)
    assert all(r.success for r in res)
    assert pool.workers[1].proc.pid != old_pid and pool.workers[1].alive


def test_analyze_project_streams_every_class_through_the_pool(tmp_path, pool):
    repo = tmp_path / "shop"
    synth.java_spring_repo(str(repo), 16)
    be = ProcessLLMBackend(pool)
    before = dict(pool.per_worker_items)
    app = make_app(tmp_path, backend=be)
    t0 = time.time()
    r = app.indexer.analyze_project(str(repo))
    assert r.success and r.classes_analyzed == 17
    assert r.stats["enriched"] == 17 and r.stats["enrichFailed"] == 0
    assert app.repos.classes.find_unenriched_by_project_id(r.project_id) == []
    got = {k: pool.per_worker_items.get(k, 0) - before.get(k, 0) for k in (0, 1)}
    assert got[0] > 0 and got[1] > 0
    # every method row got its description from the model's (grammar-forced) reply
    m = app.repos.methods.find_by_class_name("co.acme.shop.order.OrderService")
    assert m and all(x.description for x in m)  # every method: a reply that does not fit is split, not cut
    g = app.cache.get_graph(r.project_id)
    assert g.node_info("co.acme.shop.order.OrderService").description
    app.db.close()  # not app.close(): the module-scoped pool outlives this app
    assert time.time() - t0 < 600


def test_failed_init_reports_no_worker(tmp_path):
    with pytest.raises(RuntimeError):
        GpuWorkerPool(["cpu"], {"preset": "no-such-preset"}, start_timeout_s=120)


def test_bench_enrich_local_path_on_cpu_workers(tmp_path, pool):
    """bench.py's extra.enrichLocal (the GPU service path) run end to end on
    the CPU rehearsal pool: a real analyze_project streamed through it."""
    import bench
    from dmcp.parallel.dist import DistContext
    args = bench.parse_args(["--enrich-local-classes", "16"])
    rec = bench._enrich_local(pool, args, DistContext(), str(tmp_path), 0)
    assert rec["classesEnriched"] == rec["classesAnalyzed"] == 17 and rec["classesPerSec"] > 0
    assert rec["decodeStepMs"] > 0 and rec["hostMsPerStep"] > 0 and rec["prefillBatches"] >= 1


# ---------------------------------------------------------------- dealing
# model-free "echo" workers: each step of step_s answers every class a worker
# holds (a latency-bound continuous batch), so wall times measure the dealing

def _echo_pool(n, step_s=0.05, steps=1, **kw):
    return GpuWorkerPool(["cpu"] * n, {"preset": "echo", "step_s": step_s, "steps": steps, "max_batch": 512},
                         start_timeout_s=120, env_extra={"OMP_NUM_THREADS": "1"}, **kw)


def test_small_project_is_spread_over_every_gpu():
    """257 classes on 8 workers: 32 +- 1 each (was: all 257 on worker 0,
    whose in-flight capacity is 768)."""
    pool = _echo_pool(8)
    try:
        assert pool.capacity == 768
        res = ProcessLLMBackend(pool).enrich_batch(_inputs(257), "readme")
        assert all(r.success for r in res) and len(res) == 257
        counts = [pool.per_worker_items.get(i, 0) for i in range(8)]
        assert sum(counts) == 257 and max(counts) - min(counts) <= 1 and min(counts) >= 32, counts
        # a generator input without a length hint is still dealt (by capacity)
        gen = (inp for inp in _inputs(20))
        assert all(r.success for _, r in ProcessLLMBackend(pool).enrich_stream(gen, None))
    finally:
        pool.close()


def test_concurrent_streams_share_the_pool(tmp_path):
    """Two projects analysed at once split the workers (project affinity)
    and overlap: both finish in < 1.3x the time of one alone."""
    import threading
    repos = []
    for k in range(2):
        r = tmp_path / f"svc{k}"
        synth.java_spring_repo(str(r), 40, base_package=f"co.acme.s{k}", seed=k + 5)
        repos.append(str(r))
    pool = _echo_pool(8, step_s=0.1, steps=12)  # every class takes 12 steps of a continuous batch
    try:
        be = ProcessLLMBackend(pool)
        app = make_app(tmp_path, backend=be)
        app.indexer.analyze_project(repos[0])  # warm: sqlite, native scanner, the children's first session
        t0 = time.time()
        r = app.indexer.analyze_project(repos[0])
        one = time.time() - t0
        assert r.stats["enriched"] == r.classes_analyzed
        before = dict(pool.per_worker_items)
        out = {}

        def run(k):
            out[k] = app.indexer.analyze_project(repos[k])
        t0 = time.time()
        ts = [threading.Thread(target=run, args=(k,)) for k in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(120)
        both = time.time() - t0
        assert all(out[k].success and out[k].stats["enrichFailed"] == 0 for k in range(2))
        assert both < 1.3 * one, (both, one)
        used = [i for i in range(8) if pool.per_worker_items.get(i, 0) > before.get(i, 0)]
        assert len(used) == 8  # every worker served one of the two projects
        assert not pool.streams and all(w.owner is None for w in pool.workers)
        app.db.close()
    finally:
        pool.close()


def test_idle_worker_is_not_killed_as_hung():
    """A worker idle for longer than hang_timeout_s is not killed when the
    next stream's first reply takes a while (its clock starts when it gets
    work, not at its last frame)."""
    pool = _echo_pool(1, step_s=1.2, hang_timeout_s=2.0)
    try:
        be = ProcessLLMBackend(pool)
        assert all(r.success for r in be.enrich_batch(_inputs(3), None))
        time.sleep(2.5)
        res = be.enrich_batch(_inputs(3), None)
        assert all(r.success for r in res), [r.error_message for r in res]
        assert pool.deaths == 0 and pool.workers[0].alive
    finally:
        pool.close()


def test_bulk_with_local_backend_starts_one_pool(tmp_path, monkeypatch):
    """analyze-batch --workers 4 with the local backend: the repositories run
    on threads of one App and share ONE worker pool."""
    from dmcp.config import Config
    from dmcp.enrich import workers as W
    from dmcp.parallel.bulk import BulkItem, bulk_analyze
    made = []
    real = W.GpuWorkerPool.__init__

    def counting(self, *a, **kw):
        made.append(1)
        real(self, *a, **kw)
    monkeypatch.setattr(W.GpuWorkerPool, "__init__", counting)
    items = []
    for k in range(4):
        r = tmp_path / f"r{k}"
        synth.java_spring_repo(str(r), 8, base_package=f"co.b.r{k}", seed=k)
        items.append(BulkItem(str(r)))
    cfg = Config(db_path=str(tmp_path / "b.db"), git_clone_base_path=str(tmp_path / "clones"),
                 enrich_backend="local", local_llm_devices="cpu,cpu", local_llm_preset="echo",
                 local_llm_allow_random_weights=True, recover_stuck_on_start=False)
    res = bulk_analyze(cfg, items, workers=4)
    assert all(r.success for r in res), [r.message for r in res]
    assert len(made) == 1


def test_serve_mcp_never_spawns_gpu_workers(tmp_path):
    """The read-only MCP server (application-mcp.yml) with ENRICH_BACKEND=local
    serves its tools without starting the enrichment workers."""
    import subprocess
    import sys
    import psutil
    env = dict(os.environ, ENRICH_BACKEND="local", LOCAL_LLM_DEVICES="cpu", LOCAL_LLM_PRESET="echo",
               LOCAL_LLM_ALLOW_RANDOM_WEIGHTS="true", DMCP_DB_PATH=str(tmp_path / "m.db"))
    proc = subprocess.Popen([sys.executable, "-m", "dmcp", "serve-mcp"], stdin=subprocess.PIPE,
                            stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, env=env,
                            cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    try:
        def rpc(i, method, params=None):
            proc.stdin.write((json.dumps({"jsonrpc": "2.0", "id": i, "method": method,
                                          "params": params or {}}) + "\n").encode())
            proc.stdin.flush()
            return json.loads(proc.stdout.readline())
        assert rpc(1, "initialize", {"protocolVersion": "2024-11-05", "capabilities": {},
                                     "clientInfo": {"name": "t", "version": "1"}})["result"]
        r = rpc(2, "tools/call", {"name": "list_projects", "arguments": {}})
        assert not r["result"]["isError"]
        assert psutil.Process(proc.pid).children(recursive=True) == []
    finally:
        proc.stdin.close()
        proc.wait(30)
