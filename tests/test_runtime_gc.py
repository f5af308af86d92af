"""GC policy of the indexer (dmcp/utils/runtime.py): automatic passes are
held off inside an analysis and the collector's state is restored after it,
on success and on failure, with sections on several threads nesting by count."""
import gc
import threading

import pytest

from conftest import make_app
from dmcp.enrich.backend import FakeBackend, NullBackend
from dmcp.utils import synth
from dmcp.utils.errors import DomainError
from dmcp.utils.runtime import GcPause


@pytest.fixture(autouse=True)
def _gc_on():
    was = gc.isenabled()
    gc.enable()
    yield
    (gc.enable if was else gc.disable)()


def test_pause_disables_and_restores():
    p = GcPause().start()
    assert not gc.isenabled()
    p.resume()
    assert gc.isenabled()
    p.resume()  # idempotent
    assert gc.isenabled()
    with GcPause():
        assert not gc.isenabled()
    assert gc.isenabled()


def test_pause_keeps_a_disabled_collector_disabled():
    gc.disable()
    with GcPause():
        assert not gc.isenabled()
    assert not gc.isenabled()


def test_nested_sections_restore_on_the_last_exit():
    a, b = GcPause().start(), GcPause().start()
    a.resume()
    assert not gc.isenabled()  # b still open
    b.resume(collect=True)
    assert gc.isenabled()


def test_sections_on_several_threads():
    go, done = threading.Barrier(5), []

    def worker():
        p = GcPause().start()
        go.wait()
        assert not gc.isenabled()
        go.wait()
        p.resume()
        done.append(1)
    ts = [threading.Thread(target=worker) for _ in range(4)]
    for t in ts:
        t.start()
    go.wait()
    go.wait()
    for t in ts:
        t.join()
    assert len(done) == 4 and gc.isenabled()


def test_analysis_restores_the_collector(tmp_path):
    synth.java_spring_repo(str(tmp_path / "shop"), 8)
    app = make_app(tmp_path, backend=NullBackend(), require_enrichment_for_analyze=False)
    seen = []
    real = app.indexer._phase1_static

    def spy(*a, **k):
        seen.append(gc.isenabled())  # inside the section
        return real(*a, **k)
    app.indexer._phase1_static = spy
    assert app.indexer.analyze_project(str(tmp_path / "shop")).success
    assert seen == [False] and gc.isenabled()
    with pytest.raises(DomainError):
        app.indexer.analyze_project(str(tmp_path / "missing"))
    assert gc.isenabled()
    app.close()


def test_enrichment_runs_with_the_collector_on(tmp_path):
    synth.java_spring_repo(str(tmp_path / "shop"), 4)
    fake = FakeBackend()
    app = make_app(tmp_path, backend=fake)
    seen = []
    real = app.indexer._enrich_identifiers

    def spy(*a, **k):
        seen.append(gc.isenabled())
        return real(*a, **k)
    app.indexer._enrich_identifiers = spy
    assert app.indexer.analyze_project(str(tmp_path / "shop")).success
    assert seen == [True] and gc.isenabled()
    app.close()
