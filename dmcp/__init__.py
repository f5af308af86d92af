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
