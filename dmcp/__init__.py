"""dmcp -- domain-aware code-graph MCP server (MI355X-host rebuild of waabox/domain-mcp-server).

Layers: ``models`` (domain), ``graph`` (in-memory project graph +
cache), ``store`` (SQLite schema + repositories), ``parsers`` (native C++
front-ends via ``dmcp._srcscan``), ``index`` (analyze / rebuild / sync
pipeline, git, cron), ``enrich`` (LLM enrichment backends, incl. the optional
MI355X local model), ``query`` (context ops + graph DSL), ``api`` (MCP stdio +
REST), ``ops`` (HIP kernels for gfx950), ``parallel`` (fan-out / multi-GPU
work distribution), ``utils``.
"""
__version__ = "1.0.1"


def _load_native_override() -> None:
    """``DMCP_SRCSCAN_SO``: load that build of the native module as
    ``dmcp._srcscan`` (the ASan/UBSan build, scripts/asan_tests.sh)."""
    import os
    import sys
    path = os.environ.get("DMCP_SRCSCAN_SO")
    if not path or "dmcp._srcscan" in sys.modules:
        return
    import importlib.util
    spec = importlib.util.spec_from_file_location("dmcp._srcscan", path)
    if spec is None or spec.loader is None:
        raise ImportError(f"DMCP_SRCSCAN_SO={path}: not a loadable module")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sys.modules["dmcp._srcscan"] = mod
    globals()["_srcscan"] = mod


_load_native_override()
