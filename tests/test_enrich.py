"""Enrichment: JSON extraction / truncation repair / parsing (ClaudeApiClientTest
plus the private helpers the reference never tested), prompt building, backend
fan-out + failure isolation, and the Anthropic client against a local fake
HTTP server (retries, error mapping) -- no network."""
import json
import threading
import time
from http.server import BaseHTTPRequestHandler, HTTPServer

import pytest

from dmcp.config import Config
from dmcp.enrich.backend import (AnthropicBackend, FakeBackend, NullBackend, build_enrichment_prompt,
                                 create_backend)
from dmcp.enrich.jsonfix import (extract_json, loads_lenient, parse_enrichment_response, parse_string_list,
                                 repair_truncated_json)
from dmcp.enrich.types import EnrichmentInput, EnrichmentResult, normalize_method_name


def inp(name="co.a.OrderService", methods=("create",)):
    return EnrichmentInput("class OrderService { void create() {} }", name, "java", "SERVICE", list(methods))


# ---------------------------------------------------------------- jsonfix
@pytest.mark.parametrize("raw,expected", [
    (None, "{}"), ("   ", "{}"), ('{"a": 1}', '{"a": 1}'),
    ('```json\n{"a": 1}\n```', '{"a": 1}'), ('```\n{"a": 1}```', '{"a": 1}'),
    ('Sure! Here it is: {"a": {"b": 2}} hope it helps', '{"a": {"b": 2}}'),
    ("no json here", "no json here")])
def test_extract_json(raw, expected):
    assert extract_json(raw) == expected


def test_repair_truncated_json():
    assert repair_truncated_json('{"a": 1}') == '{"a": 1}'
    r = repair_truncated_json('{"description": "x", "methods": [{"methodName": "a"}, {"methodName": "b", "desc')
    assert json.loads(r) == {"description": "x", "methods": [{"methodName": "a"}]}
    nested = repair_truncated_json('{"a": [{"b": [1, 2]}, {"c": "d}]"')
    assert json.loads(nested)["a"][0] == {"b": [1, 2]}
    s = repair_truncated_json('{"a": ["x", "y')
    assert isinstance(json.loads(s), dict)


def test_loads_lenient_and_string_list():
    assert loads_lenient('```json\n{"a": [1, 2]}\n```') == {"a": [1, 2]}
    assert loads_lenient('{"m": [{"x": 1}, {"x": 2') == {"m": [{"x": 1}]}
    with pytest.raises(ValueError):
        loads_lenient("total garbage")
    assert parse_string_list(None) == [] and parse_string_list("  ") == []
    assert parse_string_list(" one ") == ["one"]
    assert parse_string_list(["a", 1, True, None, {"x": 1}]) == ["a", "1", "true", "null", ""]
    assert parse_string_list(42) == []


def test_parse_enrichment_response():
    raw = json.dumps({"description": "Handles orders", "classTypeCorrection": "SERVICE",
                      "methods": [{"methodName": "create(Order)", "description": "Creates",
                                   "businessLogic": ["validate", "persist"]},
                                  {"methodName": "list", "businessLogic": "single step"}, "junk"]})
    r = parse_enrichment_response("```json\n" + raw + "\n```", "co.a.X")
    assert r.success and r.description == "Handles orders" and r.class_type_correction == "SERVICE"
    assert [m.method_name for m in r.methods] == ["create(Order)", "list"]
    assert r.methods[1].business_logic == ["single step"] and r.methods[1].description == ""
    bad = parse_enrichment_response("not json at all", "co.a.X")
    assert not bad.success and bad.error_message.startswith("JSON parse error")
    arr = parse_enrichment_response("[1, 2]", "co.a.X")
    assert not arr.success
    empty = parse_enrichment_response("{}", "co.a.X")
    assert empty.success and empty.description == "" and empty.methods == []


def test_normalize_method_name():
    assert normalize_method_name("create(Order o)") == "create"
    assert normalize_method_name(" list ") == "list"
    assert normalize_method_name(None) is None


def test_prompt_contains_class_methods_and_readme():
    p = build_enrichment_prompt(inp(methods=("create", "cancel")), "# Shop readme")
    assert "co.a.OrderService" in p and "create" in p and "cancel" in p and "# Shop readme" in p
    assert "classTypeCorrection" in p
    big = EnrichmentInput("x" * 10000, "co.a.Big", "java", "OTHER", [])
    assert len(build_enrichment_prompt(big, None, max_source_chars=1000)) < 6000


# --------------------------------------------------------------- backends
def test_null_and_fake_backends():
    assert not NullBackend().enabled
    assert not NullBackend().enrich_batch([inp()], None)[0].success
    fb = FakeBackend(max_concurrent=3)
    res = fb.enrich_batch([inp(f"co.a.C{i}") for i in range(10)], None)
    assert all(r.success for r in res) and [r.full_class_name for r in res] == [f"co.a.C{i}" for i in range(10)]
    assert sorted(fb.calls) == sorted(f"co.a.C{i}" for i in range(10))


def test_batch_isolates_failures_and_bounds_concurrency():
    active, peak = [0], [0]
    lock = threading.Lock()

    def responder(i):
        with lock:
            active[0] += 1
            peak[0] = max(peak[0], active[0])
        time.sleep(0.02)
        with lock:
            active[0] -= 1
        if i.full_class_name.endswith("3"):
            raise RuntimeError("boom")
        return '{"description": "ok", "methods": []}'

    fb = FakeBackend(max_concurrent=4, responder=responder)
    res = fb.enrich_batch([inp(f"co.a.C{i}") for i in range(12)], None)
    assert [r.success for r in res] == [not str(i).endswith("3") for i in range(12)]
    assert "boom" in res[3].error_message and peak[0] <= 4


class _FakeAnthropic(BaseHTTPRequestHandler):
    script = []  # list of (status, body) consumed per request
    seen = []

    def do_POST(self):  # noqa: N802
        body = json.loads(self.rfile.read(int(self.headers["content-length"])))
        type(self).seen.append(({k.lower(): v for k, v in self.headers.items()}, body))
        status, payload = type(self).script.pop(0) if type(self).script else (200, None)
        if payload is None:
            payload = {"content": [{"type": "text", "text": json.dumps(
                {"description": "From fake API", "classTypeCorrection": None,
                 "methods": [{"methodName": "create", "description": "d", "businessLogic": ["s1"]}]})}]}
        data = json.dumps(payload).encode()
        self.send_response(status)
        self.send_header("content-type", "application/json")
        self.send_header("content-length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    def log_message(self, *a):
        pass


@pytest.fixture
def fake_api():
    _FakeAnthropic.script = []
    _FakeAnthropic.seen = []
    srv = HTTPServer(("127.0.0.1", 0), _FakeAnthropic)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    yield f"http://127.0.0.1:{srv.server_address[1]}"
    srv.shutdown()
    srv.server_close()


def test_anthropic_backend_success(fake_api):
    be = AnthropicBackend("sk-test", "test-model", max_tokens=123, base_url=fake_api, max_retries=0)
    r = be.enrich_class(inp(), "readme")
    assert r.success and r.description == "From fake API" and r.methods[0].business_logic == ["s1"]
    headers, body = _FakeAnthropic.seen[0]
    assert headers["x-api-key"] == "sk-test" and headers["anthropic-version"] == "2023-06-01"
    assert body["model"] == "test-model" and body["max_tokens"] == 123
    assert "co.a.OrderService" in body["messages"][0]["content"]


def test_anthropic_backend_retries_then_succeeds(fake_api):
    _FakeAnthropic.script = [(529, {"error": "overloaded"}), (429, {"error": "rate"})]
    be = AnthropicBackend("k", "m", base_url=fake_api, max_retries=2)
    t0 = time.time()
    assert be.enrich_class(inp(), None).success and len(_FakeAnthropic.seen) == 3
    assert time.time() - t0 < 10


def test_anthropic_backend_errors_are_isolated(fake_api):
    _FakeAnthropic.script = [(400, {"error": "bad request"})]
    be = AnthropicBackend("k", "m", base_url=fake_api, max_retries=3)
    res = be.enrich_batch([inp()], None)
    assert not res[0].success and "HTTP 400" in res[0].error_message and len(_FakeAnthropic.seen) == 1
    dead = AnthropicBackend("k", "m", base_url="http://127.0.0.1:9", max_retries=0, timeout_s=2)
    assert not dead.enrich_batch([inp()], None)[0].success
    with pytest.raises(ValueError):
        AnthropicBackend(" ", "m")


def test_analyze_class_legacy(fake_api):
    _FakeAnthropic.script = [(200, {"content": [{"type": "text", "text": '{"classType": "SERVICE"}'}]})]
    be = AnthropicBackend("k", "m", base_url=fake_api, max_retries=0)
    out = be.analyze_class("class A {}", "co.a.A", "A.java", None, "java")
    assert out.success and out.class_type == "SERVICE" and out.full_class_name == "co.a.A"
    assert out.source_file == "A.java" and out.methods == []


def test_create_backend_selection():
    assert create_backend(Config(enrich_backend="auto")).name == "null"
    assert create_backend(Config(enrich_backend="auto", anthropic_api_key="k")).name == "anthropic"
    assert create_backend(Config(enrich_backend="fake")).name == "fake"
    assert create_backend(Config(enrich_backend="null", anthropic_api_key="k")).name == "null"


def test_result_factories():
    ok = EnrichmentResult.ok("a.B", "d", None, [])
    assert ok.success and ok.error_message is None
    bad = EnrichmentResult.failure("a.B", "why")
    assert not bad.success and bad.methods == []


def test_analyze_batch_legacy_fans_out_in_input_order(fake_api):
    from dmcp.enrich.types import BatchClassInput
    be = AnthropicBackend("k", "m", base_url=fake_api, max_retries=0, max_concurrent=3)
    ins = [BatchClassInput(f"class C{i} {{}}", f"co.a.C{i}", f"C{i}.java", "java") for i in range(5)]
    out = be.analyze_batch(ins, "readme")
    assert [r.full_class_name for r in out] == [i.full_class_name for i in ins]
    assert all(r.success for r in out) and len(_FakeAnthropic.seen) == 5
    be.close()
