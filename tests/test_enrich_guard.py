"""Random-weight enrichment guard (round-6 verdict item 3).

The reference refuses to analyze without a usable LLM
(``CodeContextService.java:149-156``, READ_ONLY_MODE).  The local MI355X
backend without a checkpoint would instead write random-init noise into
``source_classes`` / ``source_methods``, which Phase 3 and resume never redo
(the rows are non-null).  Here: ``ENRICH_BACKEND=local`` without
``LOCAL_LLM_MODEL_PATH`` refuses unless ``LOCAL_LLM_ALLOW_RANDOM_WEIGHTS``;
every enriched class records its ``enrichment_source`` and a real backend
redoes the rows a synthetic one (random weights, echo, fake) wrote
(``CodeContextService.java:361-434``: Phase 3 picks up every class without
a usable description)."""
import json

import pytest

from conftest import make_app
from dmcp.config import Config
from dmcp.enrich.backend import (FakeBackend, LazyBackend, RefusedBackend, SYNTHETIC_PREFIX, create_backend,
                                 is_synthetic, local_source_tag)
from dmcp.utils import synth
from dmcp.utils.errors import DomainError


class _RealFake(FakeBackend):
    """The offline fake posing as a real backend (an API model)."""
    source_tag = "anthropic:test-model"


@pytest.fixture
def repo(tmp_path):
    synth.java_spring_repo(str(tmp_path / "shop"), 8)
    return tmp_path / "shop"


def _sources(app, project_id):
    return app.repos.classes.enrichment_sources(project_id)


def test_local_without_checkpoint_is_refused():
    be = create_backend(Config(enrich_backend="local"))
    assert isinstance(be, RefusedBackend) and not be.enabled
    assert "LOCAL_LLM_MODEL_PATH" in be.disabled_reason and "LOCAL_LLM_ALLOW_RANDOM_WEIGHTS" in be.disabled_reason
    # echo (model-free) is synthetic too
    assert isinstance(create_backend(Config(enrich_backend="local", local_llm_preset="echo")), RefusedBackend)


def test_opt_in_flag_and_checkpoint_tags(tmp_path):
    be = create_backend(Config(enrich_backend="local", local_llm_allow_random_weights=True))
    assert isinstance(be, LazyBackend) and be.enabled and not be.built
    assert be.source_tag == "synthetic:random-init:dmcp-coder-1b" and is_synthetic(be.source_tag)
    assert not be.built  # the tag is known without spawning GPU workers
    ck = tmp_path / "ckpt"
    ck.mkdir()
    be2 = create_backend(Config(enrich_backend="local", local_llm_model_path=str(ck)))
    assert isinstance(be2, LazyBackend) and be2.enabled
    assert be2.source_tag == f"local:{ck}" and not is_synthetic(be2.source_tag)
    assert local_source_tag(Config(local_llm_preset="echo")) == SYNTHETIC_PREFIX + "echo"
    cfg = Config.from_env({"ENRICH_BACKEND": "local", "LOCAL_LLM_ALLOW_RANDOM_WEIGHTS": "true"})
    assert cfg.local_llm_allow_random_weights is True
    assert Config.from_env({}).local_llm_allow_random_weights is False
    assert create_backend(Config(enrich_backend="fake")).source_tag == "synthetic:fake"
    assert create_backend(Config(enrich_backend="auto", anthropic_api_key="k")).source_tag.startswith("anthropic:")


def test_refused_backend_blocks_analysis_with_its_reason(tmp_path, repo):
    app = make_app(tmp_path, backend=create_backend(Config(enrich_backend="local")))
    with pytest.raises(DomainError) as e:
        app.indexer.analyze_project(str(repo))
    assert e.value.error_code == "READ_ONLY_MODE" and "LOCAL_LLM_MODEL_PATH" in str(e.value)
    assert app.repos.projects.find_all() == []
    app.close()
    # REQUIRE_ENRICHMENT_FOR_ANALYZE=false: a static index, no noise rows
    app = make_app(tmp_path, backend=create_backend(Config(enrich_backend="local")),
                   require_enrichment_for_analyze=False)
    r = app.indexer.analyze_project(str(repo))
    assert r.success and r.stats.get("enriched", 0) == 0
    assert set(_sources(app, r.project_id).values()) == {None}
    assert len(app.repos.classes.find_unenriched_by_project_id(r.project_id)) == r.classes_analyzed
    with pytest.raises(DomainError) as e:
        app.indexer.resume_enrichment(r.project_id)
    assert e.value.error_code == "READ_ONLY_MODE" and "LOCAL_LLM_MODEL_PATH" in str(e.value)
    app.close()


def test_real_backend_redoes_synthetic_rows(tmp_path, repo):
    synthetic = FakeBackend()
    app = make_app(tmp_path, backend=synthetic)
    r = app.indexer.analyze_project(str(repo))
    assert r.success and len(synthetic.calls) == r.classes_analyzed
    assert set(_sources(app, r.project_id).values()) == {"synthetic:fake"}
    # a synthetic backend's Phase 3 / resume only redoes missing rows
    assert app.indexer.resume_enrichment(r.project_id)["recovered"] == 0
    assert app.repos.classes.find_unenriched_by_project_id(r.project_id) == []
    assert len(app.repos.classes.find_unenriched_by_project_id(r.project_id, include_synthetic=True)) == \
        r.classes_analyzed
    app.close()

    def real(inp):
        return json.dumps({"description": f"real {inp.full_class_name}", "methods": [
            {"methodName": m, "description": f"real {m}", "businessLogic": ["step"]} for m in inp.method_names]})
    rb = _RealFake(responder=real)
    app2 = make_app(tmp_path, backend=rb)  # the service restarted with a checkpoint / API key
    out = app2.indexer.resume_enrichment(r.project_id)
    assert out["recovered"] == r.classes_analyzed and len(rb.calls) == r.classes_analyzed
    assert set(_sources(app2, r.project_id).values()) == {"anthropic:test-model"}
    for sc in app2.repos.classes.find_by_project_id(r.project_id):
        assert sc.description == f"real {sc.full_class_name}"
        for m in app2.repos.methods.find_by_class_id(sc.id):  # no fake "Performs x" survives
            assert m.description is None or m.description == f"real {m.method_name}"
    g = app2.cache.get_graph(r.project_id)
    assert all(g.node_info(sc.full_class_name).description.startswith("real ")
               for sc in app2.repos.classes.find_by_project_id(r.project_id))
    # nothing left to redo
    assert app2.indexer.resume_enrichment(r.project_id)["recovered"] == 0
    app2.close()


def test_phase3_of_a_real_backend_redoes_rows_kept_by_sync(tmp_path, repo):
    """Rows a sync keeps (unchanged classes) keep their synthetic marker; the
    next analysis' Phase 3 -- or resume -- under a real backend redoes them."""
    app = make_app(tmp_path, backend=FakeBackend())
    r = app.indexer.analyze_project(str(repo))
    app.close()
    rb = _RealFake()
    app2 = make_app(tmp_path, backend=rb)
    s = app2.indexer.sync_project(app2.repos.projects.find_by_id(r.project_id))
    assert s.success and len(rb.calls) == 0  # nothing changed: sync enriches nothing
    assert set(_sources(app2, r.project_id).values()) == {"synthetic:fake"}
    assert app2.indexer.resume_enrichment(r.project_id)["recovered"] == r.classes_analyzed
    assert set(_sources(app2, r.project_id).values()) == {"anthropic:test-model"}
    app2.close()


def test_enrichment_source_column_migrates_an_old_database(tmp_path):
    """Migration 10 adds the column to a database at migration 9 (rows keep
    NULL: never treated as synthetic)."""
    import sqlite3
    from dmcp.store import db as dbm
    path = str(tmp_path / "old.db")
    conn = sqlite3.connect(path)
    conn.execute("CREATE TABLE IF NOT EXISTS schema_version (version INTEGER PRIMARY KEY, description TEXT)")
    conn.close()
    old = [m for m in dbm.MIGRATIONS if m[0] < 10]
    saved = dbm.MIGRATIONS
    try:
        dbm.MIGRATIONS = old
        d = dbm.Database(path, background_checkpoint=False)
        d.close()
    finally:
        dbm.MIGRATIONS = saved
    d = dbm.Database(path, background_checkpoint=False)
    cols = [r[1] for r in d.query("PRAGMA table_info(source_classes)")]
    assert "enrichment_source" in cols
    d.close()
