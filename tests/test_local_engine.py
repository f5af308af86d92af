"""Local enrichment engine on the CPU (reference ops): grammar-forced JSON,
continuous batching, jump-forward equivalence, template fitting and the
backend contract.  The same engine runs the gfx950 kernels on the GPU
(tests/test_gpu_model.py)."""
import json

import pytest
import torch

from dmcp.enrich.local import (LocalEngine, LocalLLMBackend, build_template, fit_template, template_budget,
                               _json_safe_mask)
from dmcp.enrich.types import EnrichmentInput
from dmcp.models.llm import LocalLM, preset


@pytest.fixture(scope="module")
def tiny():
    torch.manual_seed(0)
    return LocalLM(preset("tiny", max_batch=4, max_rows=16, max_seq=768), device="cpu", seed=1)


def _inputs(n):
    return [EnrichmentInput("public class S%d { void a() {} void b() {} }" % i, f"co.x.S{i}", "java", "SERVICE",
                            ["a", "b", "c"][: 1 + i % 3]) for i in range(n)]


def test_json_safe_mask():
    m = _json_safe_mask(320, False)
    bits = [(m[v >> 5] >> (v & 31)) & 1 for v in range(320)]
    assert bits[ord("a")] and bits[ord(" ")] and not bits[ord('"')] and not bits[ord("\\")]
    assert not bits[10] and not bits[256] and sum(bits) == 95 - 2
    q = _json_safe_mask(320, True)
    assert (q[ord('"') >> 5] >> (ord('"') & 31)) & 1


def test_template_budget_and_fit():
    inp = _inputs(3)[2]
    segs = build_template(inp)
    assert segs[0].forced == b'{"description": "' and segs[1].forced is None
    assert all(not (a.forced is not None and b.forced is not None) for a, b in zip(segs, segs[1:]))
    big = template_budget(segs)
    small = fit_template(inp, big // 2)
    assert template_budget(small) <= big // 2
    many = EnrichmentInput("x", "a.B", "java", "OTHER", [f"m{i}" for i in range(200)])
    assert template_budget(fit_template(many, 300)) <= 300


def test_engine_valid_json_and_continuous_batching(tiny):
    eng = LocalEngine(tiny)
    inputs = _inputs(7)  # > max_batch 4 -> slots are recycled
    raw = eng.generate(inputs, "A readme")
    for r, inp in zip(raw, inputs):
        doc = json.loads(r)
        assert [m["methodName"] for m in doc["methods"]] == inp.method_names
        assert doc["classTypeCorrection"] is None and len(doc["methods"][0]["businessLogic"]) == 2
    assert eng.stats["prefills"] == 7 and eng.stats["decode_steps"] > 0


def test_jump_forward_is_exact_on_cpu(tiny):
    a = LocalEngine(tiny, jump_forward=False)
    b = LocalEngine(tiny, jump_forward=True)
    inputs = _inputs(4)
    ra, rb = a.generate(inputs, None), b.generate(inputs, None)
    assert sum(x == y for x, y in zip(ra, rb)) >= 3
    assert b.stats["decode_steps"] < 0.8 * a.stats["decode_steps"]
    assert b.stats["decode_rows"] == b.stats["generated_tokens"]


def test_backend_contract(tiny):
    be = LocalLLMBackend([LocalEngine(tiny)])
    res = be.enrich_batch(_inputs(3), None)
    assert all(r.success for r in res) and res[2].methods[2].method_name == "c"
    assert be.enrich_batch([], None) == []
    assert be.stats()["prefills"] == 3
    one = be.enrich_class(_inputs(1)[0], None)
    assert one.success and one.full_class_name == "co.x.S0"


def test_prompt_too_long_is_truncated_not_failed(tiny):
    eng = LocalEngine(tiny)
    long_src = "class L { " + "int x; " * 2000 + "}"
    out = eng.generate([EnrichmentInput(long_src, "co.x.L", "java", "OTHER", ["x"])], None)
    assert json.loads(out[0])["methods"][0]["methodName"] == "x"
