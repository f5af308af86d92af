"""Checkpoint tokenizers for the local enrichment engine (CPU, reference ops):
a byte-level BPE ``tokenizer.json`` trained here with the ``tokenizers``
library, a Llama-format safetensors checkpoint written here (random weights),
JSON-safe vocabulary masks, and the engine producing schema-valid replies
through that vocabulary -- the path a real checkpoint takes
(``LOCAL_LLM_MODEL_PATH``).  No network: nothing is downloaded."""
import json
import os

import pytest
import torch

from dmcp.enrich.local import LocalEngine, LocalLLMBackend, build_model
from dmcp.enrich.tokenizer import ByteTokenizer, HFTokenizer, load_local_model, load_tokenizer
from dmcp.enrich.types import EnrichmentInput

CORPUS = [
    "public class OrderService { private final OrderRepository repo; public Order create(Order o) {} }",
    "Describe the business purpose of this class and each of its methods in JSON.",
    '{"description": "Creates orders", "classTypeCorrection": null, "methods": [{"methodName": "create"}]}',
    "The service validates the payment, reserves the stock and publishes an OrderCreated event.",
    "package co.fanki.shop; import java.util.List; @Service @Transactional",
] * 20


def _train_bpe(path: str, vocab: int = 512, metaspace: bool = False) -> None:
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    if metaspace:
        tk = Tokenizer(models.BPE(unk_token="<unk>", byte_fallback=True))
        tk.pre_tokenizer = pre_tokenizers.Metaspace()
        tk.decoder = decoders.Sequence([decoders.Replace("▁", " "), decoders.ByteFallback(), decoders.Fuse()])
        alphabet = [chr(c) for c in range(0x20, 0x7F)] + ["▁"]
        trainer = trainers.BpeTrainer(vocab_size=vocab, special_tokens=["<unk>", "<s>", "</s>"]
                                      + [f"<0x{b:02X}>" for b in range(256)], initial_alphabet=alphabet)
    else:
        tk = Tokenizer(models.BPE())
        tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
        tk.decoder = decoders.ByteLevel()
        trainer = trainers.BpeTrainer(vocab_size=vocab, special_tokens=["<|bos|>", "<|eos|>"],
                                      initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tk.train_from_iterator(CORPUS, trainer)
    tk.save(path)


def _write_checkpoint(d: str, vocab: int, hidden=256, layers=2, heads=4, kv=2, inter=512, bos=None) -> None:
    from safetensors.torch import save_file
    g = torch.Generator().manual_seed(3)

    def rnd(*s, std=0.02):
        return (torch.randn(*s, generator=g) * std).to(torch.bfloat16)
    hd = hidden // heads
    t = {"model.embed_tokens.weight": rnd(vocab, hidden, std=1.0), "model.norm.weight": torch.ones(hidden).bfloat16(),
         "lm_head.weight": rnd(vocab, hidden)}
    for i in range(layers):
        p = f"model.layers.{i}."
        t[p + "input_layernorm.weight"] = torch.ones(hidden).bfloat16()
        t[p + "post_attention_layernorm.weight"] = torch.ones(hidden).bfloat16()
        t[p + "self_attn.q_proj.weight"] = rnd(heads * hd, hidden)
        t[p + "self_attn.k_proj.weight"] = rnd(kv * hd, hidden)
        t[p + "self_attn.v_proj.weight"] = rnd(kv * hd, hidden)
        t[p + "self_attn.o_proj.weight"] = rnd(hidden, heads * hd)
        t[p + "mlp.gate_proj.weight"] = rnd(inter, hidden)
        t[p + "mlp.up_proj.weight"] = rnd(inter, hidden)
        t[p + "mlp.down_proj.weight"] = rnd(hidden, inter)
    save_file(t, os.path.join(d, "model.safetensors"))
    cfg = {"vocab_size": vocab, "hidden_size": hidden, "num_hidden_layers": layers, "num_attention_heads": heads,
           "num_key_value_heads": kv, "intermediate_size": inter, "rms_norm_eps": 1e-5, "rope_theta": 10000.0}
    if bos is not None:
        cfg["bos_token_id"] = bos
    with open(os.path.join(d, "config.json"), "w") as f:
        json.dump(cfg, f)


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("ckpt"))
    _train_bpe(os.path.join(d, "tokenizer.json"))
    _write_checkpoint(d, vocab=512, bos=0)
    return d


def _bits(words, n):
    return [(words[v >> 5] >> (v & 31)) & 1 for v in range(n)]


def test_byte_tokenizer_matches_builtin_vocabulary():
    from dmcp.enrich.local import _json_safe_mask
    bt = ByteTokenizer(320)
    assert bt.encode('a"b') == [97, 34, 98] and bt.bos == 256 and bt.quote == 34
    nq, q = bt.json_masks(320)
    assert nq == _json_safe_mask(320, False) and q == _json_safe_mask(320, True)
    ids, split = bt.encode_split("README text. Source of A.java", "Source of ")
    assert ids[0] == 256 and bytes(ids[1:split]) == b"README text. " and bt.decode(ids[1:]).endswith("A.java")


def test_hf_byte_level_bpe_masks_and_roundtrip(ckpt):
    tk = load_tokenizer(ckpt)
    assert tk.bos == 0 and 300 < len(tk.token_bytes) <= 512  # the model pads its vocabulary past the tokenizer's
    text = 'public class OrderService { "quoted" \\ }'
    assert tk.decode(tk.encode(text)) == text
    assert tk.token_bytes[tk.quote] == b'"'
    nq, q = tk.json_masks(512)
    allowed = [i for i, b in enumerate(_bits(nq, 512)) if b]
    assert len(allowed) > 100  # merged multi-byte tokens are allowed, not just single bytes
    assert any(len(tk.token_bytes[i]) > 3 for i in allowed)
    for i in allowed:
        b = tk.token_bytes[i]
        assert b and b'"' not in b and b"\\" not in b and all(0x20 <= c < 0x7F for c in b)
    assert not _bits(nq, 512)[tk.quote] and _bits(q, 512)[tk.quote]
    assert not _bits(q, 512)[0] and not _bits(q, 512)[1]  # special tokens never sampled
    ids, split = tk.encode_split("Shared README. Source of B.java", "Source of ")
    assert ids[0] == 0 and tk.decode(ids[1:split]) == "Shared README. "


def test_sentencepiece_style_tokenizer(tmp_path):
    p = str(tmp_path / "tokenizer.json")
    _train_bpe(p, vocab=400, metaspace=True)
    tk = HFTokenizer(p)
    assert tk.bos is None and tk.token_bytes[tk.quote] == b'"'
    assert tk.decode(tk.encode("create the order")).strip() == "create the order"
    nq, _ = tk.json_masks(len(tk.token_bytes))
    allowed = [i for i, b in enumerate(_bits(nq, len(tk.token_bytes))) if b]
    assert any(tk.token_bytes[i].startswith(b" ") for i in allowed)  # '▁' became a space
    assert all(b'"' not in tk.token_bytes[i] for i in allowed)


def test_checkpoint_engine_generates_schema_valid_json(ckpt):
    model, tok = load_local_model(ckpt, device="cpu", max_batch=3, max_rows=24, max_seq=2048)
    assert model.cfg.vocab_size == 512 and model.cfg.hidden == 256
    eng = LocalEngine(model, tokenizer=tok, use_graphs=False)
    readme = "Shop service: orders, payments and stock reservations. " * 3
    inputs = [EnrichmentInput("public class S%d { void create() {} void cancel() {} }" % i, f"co.x.S{i}", "java",
                              "SERVICE", ["create", "cancel"][: 1 + i % 2]) for i in range(5)]
    raw = eng.generate(inputs, readme)
    for r, inp in zip(raw, inputs):
        doc = json.loads(r)
        assert [m["methodName"] for m in doc["methods"]] == inp.method_names
        assert isinstance(doc["description"], str)
    # the forced skeleton is tokenized: fewer tokens than bytes went through the model
    assert eng.stats["generated_tokens"] < sum(len(r.encode()) for r in raw)
    assert eng.stats["prefix_tokens"] > 0 and eng.stats["prefills"] == 5
    # the same replies with jump-forward off (an exact multi-token extend)
    slow = LocalEngine(model, tokenizer=tok, use_graphs=False, jump_forward=False)
    assert sum(a == b for a, b in zip(slow.generate(inputs, readme), raw)) >= 4


def test_backend_from_checkpoint_spec(ckpt):
    model, tok = build_model({"path": ckpt, "max_batch": 2, "max_rows": 16, "max_seq": 512}, "cpu")
    assert isinstance(tok, HFTokenizer) and model.cfg.max_batch == 2
    be = LocalLLMBackend([LocalEngine(model, tokenizer=tok, use_graphs=False)])
    res = be.enrich_batch([EnrichmentInput("class A { void run() {} }", "co.A", "java", "OTHER", ["run"])], None)
    assert res[0].success and res[0].methods[0].method_name == "run"
    m2, t2 = build_model({"preset": "tiny", "max_batch": 2, "max_rows": 16}, "cpu")
    assert t2 is None and m2.cfg.name == "tiny"


def test_config_reads_model_path(tmp_path):
    from dmcp.config import Config
    assert Config.from_env({"LOCAL_LLM_MODEL_PATH": str(tmp_path)}).local_llm_model_path == str(tmp_path)
    assert Config.from_env({}).local_llm_model_path == ""


def test_worker_process_serves_a_checkpoint(ckpt):
    """The service path (one worker process per device) with LOCAL_LLM_MODEL_PATH:
    the worker loads the checkpoint and its tokenizer, replies parse."""
    from dmcp.enrich.workers import GpuWorkerPool, ProcessLLMBackend
    pool = GpuWorkerPool(["cpu"], {"path": ckpt, "max_batch": 2, "max_rows": 16, "max_seq": 2048},
                         engine={"use_graphs": False}, start_timeout_s=300, env_extra={"OMP_NUM_THREADS": "2"})
    try:
        be = ProcessLLMBackend(pool)
        inputs = [EnrichmentInput("class A%d { void run() {} }" % i, f"co.A{i}", "java", "OTHER", ["run"])
                  for i in range(3)]
        res = be.enrich_batch(inputs, "Shop README. " * 4)
        assert all(r.success for r in res), [r.error_message for r in res]
        assert [r.methods[0].method_name for r in res] == ["run"] * 3
    finally:
        pool.close()


def test_sentencepiece_split_prompt_round_trips_exactly(tmp_path):
    """Metaspace tokenizers add a dummy-prefix space to each encode: the
    per-class half of a split prompt must still spell exactly the prompt's
    bytes (no extra space before 'Source of'), so the local model sees what
    an API backend gets."""
    from dmcp.enrich.tokenizer import HFTokenizer
    path = str(tmp_path / "sp.json")
    _train_bpe(path, vocab=400, metaspace=True)
    tok = HFTokenizer(path, bos=1)
    text = "Project context (README):\nA shop.\n\nSource of co.x.OrderService:\n```java\nclass A {}\n```\n"
    ids, split = tok.encode_split(text, "Source of ")
    assert ids[0] == 1 and split > 1
    # the prompt's first piece carries SentencePiece's usual dummy-prefix
    # space (as any encode of the whole prompt does); nothing else is added
    assert b"".join(tok.token_bytes[i] for i in ids[1:]) == b" " + text.encode()
    assert b"".join(tok.token_bytes[i] for i in ids[split:]) == text[text.find("Source of "):].encode()


def test_checkpoint_keeps_bf16_prefill_and_makes_type_choices(ckpt):
    """A loaded checkpoint resolves prefill_dtype "auto" to bf16 (MXFP8
    parity is pinned on random-init weights only; fp8 stays available by
    name) and gets the classTypeCorrection choice a random preset does not."""
    model, tok = load_local_model(ckpt, device="cpu", max_batch=2, max_rows=8, max_seq=1024, prefill_dtype="auto")
    assert model.checkpoint == ckpt and model.cfg.prefill_dtype == "bf16" and not model.prefill_fp8
    assert LocalEngine(model, tokenizer=tok, use_graphs=False).type_choice
    fp8, _ = load_local_model(ckpt, device="cpu", max_batch=2, max_rows=8, max_seq=1024, prefill_dtype="fp8")
    assert fp8.cfg.prefill_dtype == "fp8"


@pytest.mark.parametrize("metaspace", [False, True])
def test_continuation_batch_equals_one_by_one(tmp_path, metaspace):
    """The engine tokenises an admission's per-class prompts in one batched
    call (LocalEngine._pretokenize): the ids equal encoding each alone."""
    from dmcp.enrich.tokenizer import HFTokenizer
    path = str(tmp_path / "t.json")
    _train_bpe(path, vocab=400, metaspace=metaspace)
    tok = HFTokenizer(path, bos=1)
    texts = [f"Source of co.x.Svc{i}:\n```java\nclass Svc{i} {{ void run() {{ call({i}); }} }}\n```\n" * (1 + i % 3)
             for i in range(12)] + ["Source of ", "Source of é方法\n"]
    assert tok.encode_continuation_batch(texts) == [tok.encode_continuation(t) for t in texts]


def test_engine_batched_prompt_tokenisation_matches(ckpt):
    """Prompts built from the admission's batched tokenisation equal the
    one-class-at-a-time prompts (same replies from the same model)."""
    model, tok = load_local_model(ckpt, device="cpu", max_batch=4, max_rows=24, max_seq=2048)
    from dmcp.enrich.types import EnrichmentInput
    eng = LocalEngine(model, tokenizer=tok, use_graphs=False)
    inputs = [EnrichmentInput(f"class Svc{i} {{ void run() {{}} }}\n" * (1 + i), f"co.x.Svc{i}", "java", "SERVICE",
                              ["run"]) for i in range(5)]
    items = [(i, x) for i, x in enumerate(inputs)]
    eng._pretokenize(items, "A README.")
    assert len(eng._cont_cache) == 5
    from dmcp.enrich.local import _Seq
    batched = [eng._prompt(_Seq(x, i, []), "A README.", 64) for i, x in enumerate(inputs)]
    eng._cont_cache.clear()
    single = [eng._prompt(_Seq(x, i, []), "A README.", 64) for i, x in enumerate(inputs)]
    assert batched == single
