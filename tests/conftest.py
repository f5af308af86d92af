import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu on the GPU box")
    config.addinivalue_line("markers", "slow: long-running test")


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
