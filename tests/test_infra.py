"""Config, cron scheduler, tracing/metrics, git helpers, synthetic repo
generators -- the supporting subsystems (application.yml,
ProjectSyncScheduler, GitRepositoryManager in the reference)."""
import json
import os
import subprocess
import threading
import time
from datetime import datetime

import pytest

from dmcp.config import Config, load_config_file, sqlite_path_from_url
from dmcp.index.git import GitClient, parse_name_status, read_readme
from dmcp.index.scheduler import CronExpression, CronScheduler
from dmcp.models.domain import RepositoryUrl
from dmcp.utils import synth
from dmcp.utils.tracing import METRICS, Metrics, span


# ----------------------------------------------------------------- config
def test_config_defaults_match_reference():
    c = Config()
    assert (c.server_port, c.enrich_batch_size, c.enrich_max_concurrent) == (8080, 20, 5)
    assert (c.claude_max_tokens, c.claude_timeout_seconds, c.claude_max_retries) == (16384, 240.0, 2)
    assert c.sync_cron == "0 0 2 * * *" and not c.sync_enabled
    assert c.mcp_server_name == "domain-mcp-server" and c.mcp_server_version == "1.0.1"
    assert (c.max_readme_length, c.description_length) == (10_000, 500)
    assert c.resolved_enrich_backend() == "none" and not c.has_api_key()


def test_config_from_env_and_file(tmp_path):
    env = {"DMCP_DB_PATH": "/x/db.sqlite", "SERVER_PORT": "9090", "SYNC_ENABLED": "true",
           "ANTHROPIC_API_KEY": "k", "ENRICH_BATCH_SIZE": "7", "CLAUDE_TIMEOUT_SECONDS": "1.5",
           "REQUIRE_ENRICHMENT_FOR_ANALYZE": "false", "IGNORED": "x"}
    c = Config.from_env(env)
    assert (c.db_path, c.server_port, c.sync_enabled, c.enrich_batch_size) == ("/x/db.sqlite", 9090, True, 7)
    assert c.claude_timeout_seconds == 1.5 and not c.require_enrichment_for_analyze
    assert c.resolved_enrich_backend() == "anthropic"
    yml = tmp_path / "c.yml"
    yml.write_text("claude:\n  api-key: fromfile\n  max-tokens: 99\nsync:\n  cron: '0 */5 * * * *'\n"
                   "server:\n  port: 7000\n")
    c2 = Config.from_env({"DMCP_CONFIG": str(yml), "SERVER_PORT": "7001"})
    assert c2.anthropic_api_key == "fromfile" and c2.claude_max_tokens == 99
    assert c2.sync_cron == "0 */5 * * * *" and c2.server_port == 7001  # env beats file
    toml = tmp_path / "c.toml"
    toml.write_text('[git]\nclone-base-path = "/srv/clones"\n[database]\npath = "/srv/db"\n')
    flat = load_config_file(str(toml))
    assert flat["git_clone_base_path"] == "/srv/clones" and flat["db_path"] == "/srv/db"


def test_database_url_mapping():
    assert sqlite_path_from_url("sqlite:///rel/path.db") == "rel/path.db"
    assert sqlite_path_from_url("sqlite:////abs/path.db") == "/abs/path.db"
    assert sqlite_path_from_url("/plain/path.db") == "/plain/path.db"
    with pytest.raises(ValueError):
        sqlite_path_from_url("jdbc:postgresql://localhost/x")
    assert Config.from_env({"DATABASE_URL": "sqlite:////tmp/u.db"}).db_path == "/tmp/u.db"


# ------------------------------------------------------------------- cron
def test_cron_expressions():
    c = CronExpression("0 0 2 * * *")
    assert c.next_after(datetime(2024, 1, 1, 1, 59, 59)) == datetime(2024, 1, 1, 2, 0, 0)
    assert c.next_after(datetime(2024, 1, 1, 2, 0, 0)) == datetime(2024, 1, 2, 2, 0, 0)
    every5 = CronExpression("0 */5 * * * *")
    assert every5.next_after(datetime(2024, 1, 1, 0, 3, 0)) == datetime(2024, 1, 1, 0, 5, 0)
    weekdays = CronExpression("30 15 9 * * MON-FRI")
    assert weekdays.next_after(datetime(2024, 1, 6, 12, 0, 0)) == datetime(2024, 1, 8, 9, 15, 30)  # Sat -> Mon
    monthly = CronExpression("0 0 0 1 JAN,JUL ?")
    assert monthly.next_after(datetime(2024, 2, 1)) == datetime(2024, 7, 1)
    five = CronExpression("15 10 * * *")  # classic 5-field
    assert five.next_after(datetime(2024, 1, 1, 9, 0)) == datetime(2024, 1, 1, 10, 15)
    # day-of-week 7 is Sunday, also as a range end (Spring accepts 1-7 and 5-7)
    sunday = CronExpression("0 0 0 * * 7")
    assert sunday.next_after(datetime(2024, 1, 6, 12, 0)) == datetime(2024, 1, 7)  # Sat -> Sun
    every_day = CronExpression("0 0 0 * * 1-7")
    assert every_day.dows == set(range(7))
    assert every_day.next_after(datetime(2024, 1, 6, 12, 0)) == datetime(2024, 1, 7)
    weekend = CronExpression("0 0 0 * * 5-7")
    assert weekend.dows == {5, 6, 0}
    assert weekend.next_after(datetime(2024, 1, 8, 12, 0)) == datetime(2024, 1, 12)  # Mon -> Fri
    for bad in ("* * *", "61 * * * * *", "0 0 25 * * *", "0 0 0 * * 8"):
        with pytest.raises(ValueError):
            CronExpression(bad)


def test_scheduler_runs_and_survives_failures():
    calls = []

    def job():
        calls.append(time.time())
        if len(calls) == 1:
            raise RuntimeError("first run fails")

    s = CronScheduler("* * * * * *", job)
    s.start()
    deadline = time.time() + 6
    while len(calls) < 2 and time.time() < deadline:
        time.sleep(0.05)
    s.stop()
    assert len(calls) >= 2 and len(s.runs) >= 2


# -------------------------------------------------------------- tracing
def test_metrics_and_span(tmp_path, monkeypatch):
    m = Metrics()
    for v in (1, 2, 3, 4, 100):
        m.observe_ms("op", v)
    m.inc("n", 2)
    assert m.percentile("op", 0.5) == 3 and m.percentile("op", 1.0) == 100 and m.percentile("x", 0.5) is None
    text = m.prometheus()
    assert "dmcp_n 2.0" in text and 'dmcp_op_ms_bucket{le="+Inf"} 5' in text and "dmcp_op_ms_count 5" in text
    snap = m.snapshot()
    assert snap["counters"]["n"] == 2 and snap["latencyMs"]["op"]["count"] == 5
    trace = tmp_path / "trace.jsonl"
    monkeypatch.setenv("DMCP_TRACE_FILE", str(trace))
    sink = {}
    with span("unit.test", sink, project="p") as info:
        info["rows"] = 3
    with pytest.raises(KeyError):
        with span("unit.fail"):
            raise KeyError("x")
    assert sink["unit.test"] >= 0 and METRICS.counters.get("unit.fail.errors", 0) >= 1
    lines = [json.loads(x) for x in trace.read_text().splitlines()]
    rec = next(r for r in lines if r["span"] == "unit.test")
    assert rec["project"] == "p" and rec["rows"] == 3 and "ms" in rec


# ------------------------------------------------------------------- git
def test_parse_name_status():
    d = parse_name_status("A\tsrc/New.java\nM\tsrc/Mod.java\nD\tsrc/Old.java\n"
                          "R087\tsrc/From.java\tsrc/To.java\nC100\tsrc/A.java\tsrc/Copy.java\nT\tsrc/T.java\n", "h")
    assert d.changed_files == {"src/New.java", "src/Mod.java", "src/To.java", "src/Copy.java", "src/T.java"}
    assert d.deleted_files == {"src/Old.java", "src/From.java"} and not d.full_resync_required


def test_git_client_clone_head_diff(tmp_path):
    repo = tmp_path / "r"
    synth.java_spring_repo(str(repo), 8)
    first = subprocess.run(["git", "-C", str(repo), "rev-parse", "HEAD"], capture_output=True, text=True).stdout.strip()
    (repo / "README.md").write_text("changed readme")
    subprocess.run(["git", "-C", str(repo), "-c", "user.email=a@b", "-c", "user.name=n", "commit", "-qam", "x"],
                   check=True)
    g = GitClient(str(tmp_path / "clones"))
    c = g.clone(RepositoryUrl.of(str(repo)), None, shallow=False)
    assert os.path.isdir(c.directory) and c.commit_hash == g.head(c.directory) != first
    d = g.diff(c.directory, first, c.commit_hash)
    assert d.changed_files == {"README.md"} and not d.full_resync_required
    assert g.diff(c.directory, None, c.commit_hash).full_resync_required
    assert g.diff(c.directory, "f" * 40, c.commit_hash).full_resync_required
    assert read_readme(c.directory) == "changed readme"
    assert read_readme(c.directory, 3) == "cha\n...(truncated)"
    g.cleanup(c.directory)
    assert not os.path.exists(c.directory)
    with pytest.raises(Exception):
        g.clone(RepositoryUrl.of(str(tmp_path / "missing")), None)


def test_synthetic_generators(tmp_path):
    fq = synth.java_spring_repo(str(tmp_path / "j"), 24, commit=False)
    assert len(fq) == 25 and fq[-1].endswith("Application")
    files = synth.nestjs_repo(str(tmp_path / "n"), 3, commit=False)
    assert files and os.path.exists(tmp_path / "n" / "package.json")
    synth.go_gin_repo(str(tmp_path / "g"), 2, commit=False)
    assert (tmp_path / "g" / "go.mod").exists()
    frames = synth.stack_trace_for(fq, 20)
    assert len(frames) == 20 and all({"className", "methodName", "lineNumber"} <= set(f) for f in frames)


def test_ssh_key_path_with_spaces_is_quoted(tmp_path):
    """GIT_SSH_COMMAND is run by a shell: a key path with spaces stays one argument."""
    import shlex
    from dmcp.index.git import GitClient
    key = str(tmp_path / "my keys" / "id rsa")
    cmd = GitClient(str(tmp_path), ssh_key_path=key)._env()["GIT_SSH_COMMAND"]
    argv = shlex.split(cmd)
    assert argv[:3] == ["ssh", "-i", key]
