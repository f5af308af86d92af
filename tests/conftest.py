import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu on the GPU box")
    config.addinivalue_line("markers", "slow: long-running test")
    if os.environ.get("PYTEST_XDIST_WORKER"):
        # parallel workers share the CPUs: one intra-op pool per worker of the
        # machine's size oversubscribes it (spinning OpenMP threads made the
        # CPU-reference engine tests ~100x slower under -n 6)
        import torch
        n = int(os.environ.get("PYTEST_XDIST_WORKER_COUNT", "1"))
        torch.set_num_threads(max(1, (os.cpu_count() or 2) // max(1, n)))


@pytest.fixture(scope="session", autouse=True)
def _native_built():
    # build the in-tree native modules once (no-op when up to date)
    from dmcp import buildtools
    buildtools.build_srcscan()
    yield


@pytest.fixture
def tmp_db(tmp_path):
    from dmcp.store.db import Database
    db = Database(str(tmp_path / "t.db"))
    yield db
    db.close()


def make_app(root, backend=None, **overrides):
    """An App over a fresh SQLite file with the offline fake enrichment backend."""
    from dmcp.app import App
    from dmcp.config import Config
    from dmcp.enrich.backend import FakeBackend
    cfg = Config(db_path=str(root / "db.sqlite"), git_clone_base_path=str(root / "clones"),
                 recover_stuck_on_start=True).merged(overrides)
    return App(cfg, backend=backend if backend is not None else FakeBackend())


@pytest.fixture(scope="module")
def java_app(tmp_path_factory):
    """A 16-class Spring repo ("shop") analyzed once with the fake backend."""
    from dmcp.utils import synth
    root = tmp_path_factory.mktemp("javaapp")
    fqcns = synth.java_spring_repo(str(root / "shop"), 16)
    app = make_app(root)
    res = app.indexer.analyze_project(str(root / "shop"))
    assert res.success, res.message
    app.fqcns = fqcns
    app.project_id = res.project_id
    yield app
    app.close()


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no ROCm GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture
def pg_server(tmp_path):
    """A PostgreSQL wire-protocol server (tests/pgfake.py) on a fresh SQLite
    file, SCRAM-SHA-256 authentication."""
    from tests.pgfake import FakePgServer
    with FakePgServer(str(tmp_path / "pg.sqlite"), auth="scram") as srv:
        yield srv
