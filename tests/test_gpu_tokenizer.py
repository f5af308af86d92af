"""A Llama-format checkpoint with its own BPE tokenizer on the GPU: the
engine's hipGraph decode (gfx950 kernels, vocabulary-sized grammar masks)
produces schema-valid replies, and the checkpoint's prefill matches the fp32
reference.  The checkpoint and tokenizer are written by the test (random
weights; no download)."""
import json
import os

import pytest
import torch

from tests.test_tokenizer import _train_bpe, _write_checkpoint

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("gpu_ckpt"))
    _train_bpe(os.path.join(d, "tokenizer.json"))
    _write_checkpoint(d, vocab=512, bos=0)
    return d


def test_checkpoint_prefill_matches_reference(ckpt):
    from dmcp.enrich.tokenizer import load_local_model
    from dmcp.ops import hip
    hip.lib()
    model, tok = load_local_model(ckpt, device="cuda", max_batch=8, max_rows=64, max_seq=2048)
    toks = [0] + tok.encode("public class OrderService { void create() {} }")
    got = model.forward_tokens(torch.tensor(toks, dtype=torch.int32), 1, 0).float()
    ref = model.reference_logits(toks)[-1].float()
    assert (got - ref).abs().max().item() < 0.05 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("kv_dtype", ["bf16", "fp8"])
def test_checkpoint_engine_on_gpu(ckpt, kv_dtype):
    from dmcp.enrich.local import LocalEngine
    from dmcp.enrich.tokenizer import load_local_model
    from dmcp.enrich.types import EnrichmentInput
    model, tok = load_local_model(ckpt, device="cuda", max_batch=8, max_rows=64, max_seq=2048, kv_dtype=kv_dtype)
    eng = LocalEngine(model, tokenizer=tok)
    # free-text masks (no quote / quote) + one row per choice trie state
    assert eng.graphs is not None and eng.masks.shape[1] == 512 // 32 and eng.masks.shape[0] > 2
    readme = "Shop service: orders, payments and stock reservations. " * 4
    inputs = [EnrichmentInput("public class S%d { void create() {} void cancel() {} }" % i, f"co.x.S{i}", "java",
                              "SERVICE", ["create", "cancel"][: 1 + i % 2]) for i in range(12)]
    raw = eng.generate(inputs, readme)
    for r, inp in zip(raw, inputs):
        doc = json.loads(r)
        assert [m["methodName"] for m in doc["methods"]] == inp.method_names
        assert '"' not in doc["description"] and "\\" not in doc["description"]
    assert eng.stats["prefix_tokens"] > 0 and eng.stats["decode_steps"] > 0
