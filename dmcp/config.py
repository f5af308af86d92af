"""Typed runtime configuration.

Parity: ``src/main/resources/application.yml:1-74`` and ``application-mcp.yml``.
Every reference key is honoured -- including the ones the reference declares
but never reads (``claude.model``, ``claude.max-tokens``, ``git.ssh-key-path``,
``git.timeout-seconds``, ``mcp.server.*``) -- with the reference
defaults.  Sources, lowest to highest precedence: defaults, an optional
TOML/YAML file (``DMCP_CONFIG``), environment variables.
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, field
from typing import Any, Dict, Optional

DEFAULT_CLAUDE_MODEL = "claude-sonnet-4-5-20250929"


@dataclass
class Config:
    # storage (application.yml:11-29).  DATABASE_URL may be sqlite:///path, a
    # path, or PostgreSQL (postgresql://u:p@h:5432/db?currentSchema=s or the
    # reference's jdbc:postgresql://h:5432/db form + DATABASE_USERNAME /
    # DATABASE_PASSWORD): then database_url is set and db_path is unused
    db_path: str = field(default_factory=lambda: os.path.join(
        os.path.expanduser("~"), ".dmcp", "dmcp.db"))
    database_url: Optional[str] = None
    database_username: Optional[str] = None
    database_password: Optional[str] = None
    # HTTP (application.yml:1-5)
    server_port: int = 8080
    server_host: str = "127.0.0.1"
    app_url: str = "http://localhost:8080"
    # enrichment (application.yml:38-41, ClaudeApiClient.java:40,123-125,151)
    anthropic_api_key: Optional[str] = None
    anthropic_base_url: str = "https://api.anthropic.com"
    claude_model: str = DEFAULT_CLAUDE_MODEL
    claude_max_tokens: int = 16384
    claude_timeout_seconds: float = 240.0
    claude_max_retries: int = 2
    enrich_max_concurrent: int = 5          # CodeContextService.java:77
    enrich_batch_size: int = 20             # CodeContextService.java:75
    enrich_backend: str = "auto"            # auto | anthropic | null | fake | local
    enrich_max_source_chars: int = 200_000  # prompt budget for huge files
    require_enrichment_for_analyze: bool = True  # READ_ONLY_MODE parity
    # local MI355X enrichment backend (extension, see dmcp/enrich/local.py)
    local_llm_preset: str = "dmcp-coder-1b"
    # a Llama-format checkpoint directory (config.json + *.safetensors +
    # tokenizer.json) used instead of the random-initialised preset
    local_llm_model_path: str = ""
    # without a checkpoint the local backend refuses to enrich (its random
    # weights would write noise descriptions that Phase 3 and resume never
    # redo); bench / smoke / tests opt in to the random-initialised presets
    local_llm_allow_random_weights: bool = False
    # fp8 (e4m3) KV cache: half the decode-attention bytes; every tuned and
    # benchmarked number is fp8 (56.8 vs 43.9 classes/s bf16, profiles/enrich_*_r3_prompt.jsonl)
    local_llm_kv_dtype: str = "fp8"
    # batched-prefill GEMMs: "auto" = MXFP8 (csrc/pgemm.hip) on a gfx950 GPU,
    # bf16 elsewhere; "bf16" / "fp8" force one
    local_llm_prefill_dtype: str = "auto"
    local_llm_decode_dtype: str = "bf16"
    # reply budget in tokens (the reference's claude.max-tokens analog): a
    # class whose reply does not fit is generated in several parts and merged
    local_llm_max_new_tokens: int = 4096
    # decode each method of a class as its own sequence from the class head's
    # KV (a class's latency: head + longest method, not all methods in a row)
    local_llm_fork_methods: bool = True
    # ... only for classes whose own prompt is at most this many tokens (0 =
    # every class; profiles/enrich_fork_context_ab_r5.txt)
    local_llm_fork_max_context: int = 0
    # byte caps of the reply's free strings (class description, method
    # description, business-logic step) and the step count; 0 = derived from
    # the reply budget (dmcp/enrich/local.py ReplyShape.from_budget: 256 / 128
    # / 64 bytes and 4 steps at 4,096 tokens)
    local_llm_desc_max_bytes: int = 0
    local_llm_method_max_bytes: int = 0
    local_llm_step_max_bytes: int = 0
    local_llm_max_steps: int = 0
    local_llm_devices: str = "all"
    # "process": one worker process per GPU, started before this process
    # touches HIP (the service default); "inline": engines in this process
    local_llm_workers: str = "process"
    local_llm_max_batch: int = 768      # KV slots (concurrent sequences) per GPU (profiles/enrich_batch_sweep_r5.txt)
    # enrichment hands the backend every pending class as one stream (a local
    # engine keeps its continuous batch full); false = the reference's
    # barriers of enrich_batch_size classes
    enrich_stream: bool = True
    # git (application.yml:44-47)
    git_clone_base_path: str = "/tmp/domain-mcp-repos"
    git_ssh_key_path: Optional[str] = None
    git_timeout_seconds: int = 300
    # read sources straight from git objects (bare clone + cat-file) instead of
    # a working-tree checkout; larger trees fall back to a checkout
    git_in_memory: bool = True
    git_in_memory_max_mb: int = 1024
    # sync (application.yml:49-52)
    sync_enabled: bool = False
    sync_cron: str = "0 0 2 * * *"
    # MCP (application.yml:54-59; serverInfo is hard-coded 1.0.1 in the reference)
    mcp_server_name: str = "domain-mcp-server"
    mcp_server_version: str = "1.0.1"
    mcp_server_description: str = ("Domain MCP Server - Analyzes git repositories and extracts "
                                   "business information")
    # pipeline tunables (CodeContextService.java:73, 176-177)
    max_readme_length: int = 10_000
    description_length: int = 500
    parser_threads: int = 0
    # SQLite: WAL checkpoints on a background thread (dmcp/store/db.py::_Checkpointer)
    db_background_checkpoint: bool = True
    recover_stuck_on_start: bool = True
    # cross-process project lease (dmcp/index/lease.py) and graph-cache freshness
    project_lease_seconds: float = 60.0
    graph_refresh_seconds: float = 1.0
    # source scan isolation: "auto" (a child process for remote repositories),
    # "process" (always), "inline" (never); a hung or crashed scan becomes
    # ANALYSIS_FAILED after scan_timeout_seconds (GoSourceParser.java:62)
    scan_isolation: str = "auto"
    scan_timeout_seconds: float = 120.0
    log_level: str = "INFO"

    @classmethod
    def from_env(cls, env: Optional[Dict[str, str]] = None, file: Optional[str] = None) -> "Config":
        env = dict(os.environ if env is None else env)
        cfg = cls()
        path = file or env.get("DMCP_CONFIG")
        if path:
            cfg = cfg.merged(load_config_file(path))
        mapping = {
            "DMCP_DB_PATH": "db_path",
            "SERVER_PORT": "server_port",
            "SERVER_HOST": "server_host",
            "APP_URL": "app_url",
            "ANTHROPIC_API_KEY": "anthropic_api_key",
            "ANTHROPIC_BASE_URL": "anthropic_base_url",
            "CLAUDE_MODEL": "claude_model",
            "CLAUDE_MAX_TOKENS": "claude_max_tokens",
            "CLAUDE_TIMEOUT_SECONDS": "claude_timeout_seconds",
            "CLAUDE_MAX_RETRIES": "claude_max_retries",
            "ENRICH_MAX_CONCURRENT": "enrich_max_concurrent",
            "ENRICH_BATCH_SIZE": "enrich_batch_size",
            "ENRICH_BACKEND": "enrich_backend",
            "REQUIRE_ENRICHMENT_FOR_ANALYZE": "require_enrichment_for_analyze",
            "LOCAL_LLM_PRESET": "local_llm_preset",
            "LOCAL_LLM_MODEL_PATH": "local_llm_model_path",
            "LOCAL_LLM_ALLOW_RANDOM_WEIGHTS": "local_llm_allow_random_weights",
            "LOCAL_LLM_KV_DTYPE": "local_llm_kv_dtype",
            "LOCAL_LLM_PREFILL_DTYPE": "local_llm_prefill_dtype",
            "LOCAL_LLM_DECODE_DTYPE": "local_llm_decode_dtype",
            "LOCAL_LLM_MAX_NEW_TOKENS": "local_llm_max_new_tokens",
            "LOCAL_LLM_FORK_METHODS": "local_llm_fork_methods",
            "LOCAL_LLM_FORK_MAX_CONTEXT": "local_llm_fork_max_context",
            "LOCAL_LLM_DESC_MAX_BYTES": "local_llm_desc_max_bytes",
            "LOCAL_LLM_METHOD_MAX_BYTES": "local_llm_method_max_bytes",
            "LOCAL_LLM_STEP_MAX_BYTES": "local_llm_step_max_bytes",
            "LOCAL_LLM_MAX_STEPS": "local_llm_max_steps",
            "LOCAL_LLM_DEVICES": "local_llm_devices",
            "LOCAL_LLM_WORKERS": "local_llm_workers",
            "LOCAL_LLM_MAX_BATCH": "local_llm_max_batch",
            "ENRICH_STREAM": "enrich_stream",
            "GIT_CLONE_BASE_PATH": "git_clone_base_path",
            "GIT_SSH_KEY_PATH": "git_ssh_key_path",
            "GIT_TIMEOUT_SECONDS": "git_timeout_seconds",
            "GIT_IN_MEMORY": "git_in_memory",
            "GIT_IN_MEMORY_MAX_MB": "git_in_memory_max_mb",
            "SYNC_ENABLED": "sync_enabled",
            "SYNC_CRON": "sync_cron",
            "MCP_SERVER_NAME": "mcp_server_name",
            "MCP_SERVER_VERSION": "mcp_server_version",
            "PARSER_THREADS": "parser_threads",
            "DB_BACKGROUND_CHECKPOINT": "db_background_checkpoint",
            "RECOVER_STUCK_ON_START": "recover_stuck_on_start",
            "PROJECT_LEASE_SECONDS": "project_lease_seconds",
            "GRAPH_REFRESH_SECONDS": "graph_refresh_seconds",
            "SCAN_ISOLATION": "scan_isolation",
            "SCAN_TIMEOUT_SECONDS": "scan_timeout_seconds",
            "LOG_LEVEL": "log_level",
        }
        updates: Dict[str, Any] = {}
        for key, attr in mapping.items():
            if key in env and env[key] != "":
                updates[attr] = env[key]
        db_url = env.get("DATABASE_URL")
        if db_url and "DMCP_DB_PATH" not in env:
            if is_postgres_url(db_url):
                updates["database_url"] = db_url
            else:
                updates["db_path"] = sqlite_path_from_url(db_url)
        for key, attr in (("DATABASE_USERNAME", "database_username"), ("DATABASE_PASSWORD", "database_password")):
            if env.get(key):
                updates[attr] = env[key]
        return cfg.merged(updates)

    def merged(self, values: Dict[str, Any]) -> "Config":
        types = {f.name: f.type for f in dataclasses.fields(self)}
        kw = {}
        for k, v in values.items():
            k = k.replace("-", "_").replace(".", "_")
            if k not in types:
                continue
            kw[k] = _coerce(v, getattr(self, k), types[k])
        return dataclasses.replace(self, **kw)

    def has_api_key(self) -> bool:
        return bool(self.anthropic_api_key and self.anthropic_api_key.strip())

    def resolved_enrich_backend(self) -> str:
        b = (self.enrich_backend or "auto").lower()
        if b == "auto":
            return "anthropic" if self.has_api_key() else "none"
        return b


def is_postgres_url(url: Optional[str]) -> bool:
    return bool(url) and url.startswith(("postgresql://", "postgres://", "jdbc:postgresql://"))


def sqlite_path_from_url(url: str) -> str:
    if url.startswith("sqlite:///"):
        # SQLAlchemy convention: sqlite:///relative.db, sqlite:////absolute.db
        return url[len("sqlite:///"):]
    if url.startswith("sqlite://"):
        return url[len("sqlite://"):]
    if is_postgres_url(url):
        raise ValueError("a PostgreSQL URL names no SQLite file; set it as DATABASE_URL (Config.database_url)")
    if url.startswith("jdbc:"):
        raise ValueError(f"unsupported JDBC URL {url!r}: only jdbc:postgresql:// is")
    return url


def _coerce(value: Any, current: Any, typ: Any) -> Any:
    t = str(typ)
    if value is None:
        return None
    if "bool" in t or isinstance(current, bool):
        if isinstance(value, bool):
            return value
        return str(value).strip().lower() in ("1", "true", "yes", "on")
    if "int" in t and "Optional" not in t or isinstance(current, int) and not isinstance(current, bool):
        return int(value)
    if "float" in t or isinstance(current, float):
        return float(value)
    return str(value) if not isinstance(value, str) else value


def load_config_file(path: str) -> Dict[str, Any]:
    """Reads a TOML or YAML config file and flattens nested sections
    (``claude.max-tokens`` -> ``claude_max_tokens``)."""
    with open(path, "rb") as f:
        data = f.read()
    if path.endswith((".yml", ".yaml")):
        import yaml
        tree = yaml.safe_load(data.decode("utf-8")) or {}
    else:
        try:
            import tomllib  # type: ignore
        except ImportError:  # py3.10
            import tomli as tomllib  # type: ignore
        tree = tomllib.loads(data.decode("utf-8"))
    flat: Dict[str, Any] = {}

    def walk(prefix: str, node: Any) -> None:
        if isinstance(node, dict):
            for k, v in node.items():
                key = f"{prefix}_{k}" if prefix else str(k)
                walk(key.replace("-", "_").replace(".", "_"), v)
        else:
            flat[prefix] = node

    walk("", tree)
    aliases = {"claude_api_key": "anthropic_api_key", "git_clone_base_path": "git_clone_base_path",
               "server_port": "server_port", "mcp_server_name": "mcp_server_name",
               "mcp_server_version": "mcp_server_version", "sync_cron": "sync_cron",
               "sync_enabled": "sync_enabled", "database_path": "db_path"}
    return {aliases.get(k, k): v for k, v in flat.items()}
