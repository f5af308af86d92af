"""Local enrichment model on the GPU: decode path vs fp32 reference, hipGraph
replay vs eager, and the JSON-constrained engine end to end."""
import json

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def model():
    from dmcp.models.llm import LocalLM, preset
    from dmcp.ops import hip
    hip.lib()
    return LocalLM(preset("tiny", max_batch=16), device="cuda")


def _rel_err(a, b):
    return (a.float() - b.float()).abs().max().item() / max(1.0, b.float().abs().max().item())


def test_prefill_matches_reference(model):
    toks = [256] + list(b"public class UserController { void list() {} }")
    got = model.forward_tokens(torch.tensor(toks, dtype=torch.int32), 2, 0)
    ref = model.reference_logits(toks)[-1]
    assert _rel_err(got, ref) < 0.03


def test_decode_and_extend_match_reference(model):
    toks = [256] + list(b"@Service class A {")
    model.forward_tokens(torch.tensor(toks, dtype=torch.int32), 1, 0)
    nxt = [ord("x"), ord("y")]
    d = model.decode(torch.tensor([nxt[0]], dtype=torch.int32, device="cuda"),
                     torch.tensor([1], dtype=torch.int32, device="cuda"),
                     torch.tensor([len(toks)], dtype=torch.int32, device="cuda"))[0]
    assert _rel_err(d, model.reference_logits(toks + nxt[:1])[-1]) < 0.03
    e = model.forward_tokens(torch.tensor(nxt[1:], dtype=torch.int32), 1, len(toks) + 1)
    assert _rel_err(e, model.reference_logits(toks + nxt)[-1]) < 0.03


def test_graph_replay_equals_eager(model):
    from dmcp.models.llm import DecodeGraphs
    for s in range(3):
        model.forward_tokens(torch.tensor([256, 65 + s, 66], dtype=torch.int32), s, 0)
    tok = torch.tensor([70, 71, 72], dtype=torch.int32, device="cuda")
    sl = torch.tensor([0, 1, 2], dtype=torch.int32, device="cuda")
    ps = torch.tensor([3, 3, 3], dtype=torch.int32, device="cuda")
    eager = model.decode(tok, sl, ps).clone()
    graphs = DecodeGraphs(model)
    replay = graphs.run(tok, sl, ps).clone()
    torch.testing.assert_close(replay.float(), eager.float(), atol=1e-2, rtol=1e-2)


def test_engine_generates_valid_json(model):
    from dmcp.enrich.local import LocalEngine, LocalLLMBackend
    from dmcp.enrich.types import EnrichmentInput
    eng = LocalEngine(model)
    be = LocalLLMBackend([eng])
    inputs = [EnrichmentInput("class C%d { void run() {} }" % i, f"co.acme.C{i}", "java", "SERVICE",
                              ["run", "stop"][: 1 + i % 2]) for i in range(20)]  # > max_batch: continuous batching
    raw = eng.generate(inputs, "readme")
    for r, inp in zip(raw, inputs):
        doc = json.loads(r)
        assert [m["methodName"] for m in doc["methods"]] == inp.method_names
    res = be.enrich_batch(inputs, None)
    assert all(x.success for x in res)
    assert eng.stats["decode_steps"] > 0 and eng.stats["prefills"] == 40
