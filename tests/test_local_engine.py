"""Local enrichment engine on the CPU (reference ops): grammar-forced JSON,
continuous batching, jump-forward equivalence, template fitting and the
backend contract.  The same engine runs the gfx950 kernels on the GPU
(tests/test_gpu_model.py)."""
import json

import pytest
import torch

from dmcp.enrich.local import (CLASS_TYPES, LocalEngine, LocalLLMBackend, build_template, fit_template, merge_parts,
                               plan_reply, template_budget, _json_safe_mask)
from dmcp.enrich.types import EnrichmentInput
from dmcp.models.llm import LocalLM, preset


@pytest.fixture(scope="module")
def tiny():
    torch.manual_seed(0)
    return LocalLM(preset("tiny", max_batch=4, max_rows=16, max_seq=2048), device="cpu", seed=1)


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
    segs = build_template(inp.method_names)
    assert segs[0].forced == b'{"description": "' and segs[1].forced is None
    assert all(not (a.forced is not None and b.forced is not None) for a, b in zip(segs, segs[1:]))
    assert segs[3].choice == 0 and len(segs[3].then) == 11  # classTypeCorrection: null | 10 types
    big = template_budget(segs)
    small = fit_template(inp, big // 2)
    assert template_budget(small) <= big // 2
    many = EnrichmentInput("x", "a.B", "java", "OTHER", [f"m{i}" for i in range(200)])
    assert template_budget(fit_template(many, 300)) <= 300


def test_plan_reply_splits_instead_of_dropping():
    """No silent drops: methods that do not fit one reply go to continuation
    parts, each within the budget, together covering every method in order."""
    names = [f"method{i}" for i in range(60)]
    parts, dropped = plan_reply(names, 1024)
    assert dropped == 0 and len(parts) > 1
    assert all(template_budget(p) <= 1024 for p in parts)
    covered = []
    for p in parts:
        for seg in p:
            if seg.forced and b'"methodName": ' in seg.forced:
                covered += [json.loads(x.split(b", ")[0]) for x in seg.forced.split(b'"methodName": ')[1:]]
    assert covered == names
    assert parts[1][0].forced.startswith(b'{"description": "", "classTypeCorrection": null')
    merged = json.loads(merge_parts(['{"description": "d", "classTypeCorrection": "DTO", "methods": [{"methodName": "a"}]}',
                                     '{"description": "", "classTypeCorrection": null, "methods": [{"methodName": "b"}]}']))
    assert merged["description"] == "d" and merged["classTypeCorrection"] == "DTO"
    assert [m["methodName"] for m in merged["methods"]] == ["a", "b"]
    one, d1 = plan_reply(["x" * 5000], 1024)
    assert d1 == 1  # a method name longer than the budget is the only drop, and it is counted


def test_engine_valid_json_and_continuous_batching(tiny):
    eng = LocalEngine(tiny)
    inputs = _inputs(7)  # > max_batch 4 -> slots are recycled
    raw = eng.generate(inputs, "A readme")
    for r, inp in zip(raw, inputs):
        doc = json.loads(r)
        assert [m["methodName"] for m in doc["methods"]] == inp.method_names
        assert doc["classTypeCorrection"] is None or doc["classTypeCorrection"] in CLASS_TYPES
        assert all(1 <= len(m["businessLogic"]) <= 3 for m in doc["methods"])
    assert eng.stats["prefills"] == 7 and eng.stats["decode_steps"] > 0


def test_two_admissions_in_flight_match_one(tiny):
    """Up to ``admit_depth`` batched prefills in flight (the next admission's
    host work under the previous prefill) and a feed refilled a chunk at a
    time generate what one admission at a time and a whole refill do."""
    a = LocalEngine(tiny)
    a.admit_depth, a.refill_chunk, a.admit_min = 1, 0, 1
    b = LocalEngine(tiny)
    b.admit_depth, b.refill_chunk, b.admit_min = 2, 2, 1
    inputs = _inputs(9)
    ra, rb = a.generate(inputs, "A readme"), b.generate(inputs, "A readme")
    for r in rb:
        json.loads(r)
    assert sum(x == y for x, y in zip(ra, rb)) >= len(ra) - 1
    assert b.stats["prefills"] == a.stats["prefills"] == 9


@pytest.mark.parametrize("native", [False, True])
def test_host_work_under_the_step_generates_the_same(tiny, native):
    """The look-ahead refill and the admissions run after the step launch
    (under the steps in flight) or at the loop iteration's top: the same
    replies, every class admitted once, and the slowest iterations recorded
    with their phases."""
    a = LocalEngine(tiny, native_grammar=native)
    a.host_under_step = False
    b = LocalEngine(tiny, native_grammar=native)
    b.host_under_step = True
    a.refill_chunk = b.refill_chunk = 2
    inputs = _inputs(9)
    ra, rb = a.generate(inputs, "A readme"), b.generate(inputs, "A readme")
    for r in rb:
        json.loads(r)
    assert sum(x == y for x, y in zip(ra, rb)) >= len(ra) - 1
    assert a.stats["prefills"] == b.stats["prefills"] == 9
    assert b.stats["under_s"] > a.stats["under_s"]  # refill + admission time spent under the steps
    assert b.slow_iters and all(ms >= 0 and all(v >= 0 for v in ph.values()) for ms, ph in b.slow_iters)


def test_session_defers_full_gc_and_restores_threshold(tiny):
    """A session raises the full-collection threshold while it runs (a full
    pass over the run's objects paused the GPU loop) and restores the
    interpreter's own afterwards -- also when the consumer stops early."""
    import gc
    before = gc.get_threshold()
    eng = LocalEngine(tiny)
    eng.gc_full_every = 5000
    seen = [gc.get_threshold() for _ in eng.stream(enumerate(_inputs(3)), None)]
    assert len(seen) == 3 and all(t[2] == max(before[2], 5000) for t in seen)
    assert gc.get_threshold() == before
    it = eng.stream(enumerate(_inputs(3)), None)
    next(it)
    assert gc.get_threshold()[2] == max(before[2], 5000)
    it.close()  # the consumer stops early: the session's finally restores it
    assert gc.get_threshold() == before


def test_gc_deferral_is_process_wide_across_engines(tiny):
    """Sessions of several engines overlap (``_threaded_stream``): the first
    to enter saves the interpreter's threshold and the last to leave
    restores it, whatever the interleaving (advisor r5: per-session
    save/restore could leave full collections deferred for good)."""
    import gc
    from dmcp.enrich import local as L
    before = gc.get_threshold()
    # the interleaving that broke per-session save/restore: A in, B in, A out, B out
    L._gc_defer_enter(1000)
    L._gc_defer_enter(5000)
    assert gc.get_threshold()[2] == max(before[2], 5000)
    L._gc_defer_exit()
    assert gc.get_threshold()[2] == max(before[2], 5000)  # B still runs
    L._gc_defer_exit()
    assert gc.get_threshold() == before
    # two engines through the threaded multi-replica stream
    other = LocalLM(preset("tiny", max_batch=4, max_rows=16, max_seq=2048), device="cpu", seed=1)
    engines = [LocalEngine(tiny), LocalEngine(other)]  # one model (KV cache) per engine, as one per GPU
    for e in engines:
        e.gc_full_every = 7000
    out = list(L._threaded_stream(engines, enumerate(_inputs(6)), None))
    assert sorted(i for i, _ in out) == list(range(6)) and all(r.success for _, r in out)
    assert gc.get_threshold() == before


def test_jump_forward_is_exact_on_cpu(tiny):
    a = LocalEngine(tiny, jump_forward=False)
    b = LocalEngine(tiny, jump_forward=True)
    inputs = _inputs(4)
    ra, rb = a.generate(inputs, None), b.generate(inputs, None)
    assert sum(x == y for x, y in zip(ra, rb)) >= 3
    assert b.stats["decode_steps"] < 0.8 * a.stats["decode_steps"]
    assert b.stats["decode_rows"] == b.stats["generated_tokens"]


def test_pipelined_loop_matches_synchronous_loop(tiny):
    """The one-step pipeline (device-side gather of the previous selections,
    grammar one step behind) generates what the synchronous loop does."""
    sync = LocalEngine(tiny, pipeline=False)
    pipe = LocalEngine(tiny, pipeline=True)
    inputs = _inputs(7)
    ra, rb = sync.generate(inputs, "A readme"), pipe.generate(inputs, "A readme")
    assert sum(x == y for x, y in zip(ra, rb)) >= 6
    for r in rb:
        json.loads(r)
    # forced bytes after a sampled quote start a step later: a few more steps
    assert sync.stats["decode_steps"] <= pipe.stats["decode_steps"] <= 1.3 * sync.stats["decode_steps"]
    assert pipe.stats["generated_tokens"] == sync.stats["generated_tokens"] or \
        sum(x == y for x, y in zip(ra, rb)) < len(ra)


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


def test_shared_prefix_cpu_matches_full_prompt(tiny):
    """CPU reference path of the shared prefix: prefix prefill once + suffix
    prefill + decode == full-prompt prefill + decode."""
    prefix = [256] + list(b"Shared instructions and README text for every class of the project. " * 2)
    tails = [list(b"class A {}"), list(b"class Bb { int x; }")]
    full = []
    for s, t in enumerate(tails):
        full.append(tiny.forward_tokens(torch.tensor(prefix + t, dtype=torch.int32), s, 0))
    d_full = tiny.decode(torch.tensor([65, 66], dtype=torch.int32), torch.tensor([0, 1], dtype=torch.int32),
                         torch.tensor([len(prefix) + len(t) for t in tails], dtype=torch.int32))
    P = tiny.set_prefix(prefix)
    try:
        for s, t in enumerate(tails):
            tiny.fork_prefix(s + 2)
            lg = tiny.forward_tokens(torch.tensor(t, dtype=torch.int32), s + 2, P)
            torch.testing.assert_close(lg.float(), full[s].float(), atol=3e-2, rtol=3e-2)
        d = tiny.decode(torch.tensor([65, 66], dtype=torch.int32), torch.tensor([2, 3], dtype=torch.int32),
                        torch.tensor([len(prefix) + len(t) for t in tails], dtype=torch.int32))
        torch.testing.assert_close(d.float(), d_full.float(), atol=3e-2, rtol=3e-2)
    finally:
        tiny.clear_prefix()


def test_engine_prompt_prefix_detection(tiny):
    """The shared prefix is everything before 'Source of' (instructions +
    README: the same for every class of a project)."""
    from dmcp.enrich.local import _Seq
    eng = LocalEngine(tiny, use_graphs=False)
    readme = "A README shared by every prompt of the batch. " * 3

    def seq(inp):
        return eng._seqs_for(0, inp, readme)[0]
    sa, sb = seq(_inputs(1)[0]), seq(_inputs(2)[1])
    a, b = sa.prompt, sb.prompt
    P = eng._seq_prefix_len(sa)
    assert P > 64 and bytes(a[P:P + 10]) == b"Source of " and eng._seq_prefix_len(sb) == P
    assert a[:P] == b[:P] and a[P + 10:] != b[P + 10:]
    short = _Seq(_inputs(1)[0], 0, [], prompt=[256] + list(b"Source of x"), prefix_split=1)
    assert eng._seq_prefix_len(short) == 0  # below the minimum
    assert LocalEngine(tiny, use_graphs=False, shared_prefix=False)._seq_prefix_len(sa) == 0
    out = eng.generate(_inputs(5), readme)
    assert eng.stats["prefix_tokens"] == P and all(json.loads(o) for o in out)
    assert eng.stats["prefill_batches"] < eng.stats["prefills"]  # admitted classes share one prefill pass
    assert tiny.prefix_len == 0  # cleared after the stream


def test_engine_streams_results_as_they_finish(tiny):
    """stream() pulls inputs lazily (never more than free slots + look-ahead
    ahead of what finished) and yields each reply as its sequence ends."""
    eng = LocalEngine(tiny, use_graphs=False)
    pulled = []

    def src():
        for i, inp in enumerate(_inputs(12)):
            pulled.append(i)
            yield i, inp
    seen = []
    for key, raw in eng.stream(src(), "readme text"):
        seen.append(key)
        if len(seen) == 1:
            assert len(pulled) < 12  # the first reply came before the feed was drained
        json.loads(raw)
    assert sorted(seen) == list(range(12))


def test_engine_admits_other_prefixes_unshared(tiny):
    """A prompt whose prefix differs (another project's README) runs next to
    the others with its whole prompt in its own slot -- never attending to
    the wrong prefix -- and equals its reply generated alone."""
    readme = "A README shared by every prompt of the batch. " * 3
    other = "Another project entirely, with its own README text. " * 3
    inputs = _inputs(4)
    mixed = [(i, inp, other if i == 2 else readme) for i, inp in enumerate(inputs)]
    eng = LocalEngine(tiny, use_graphs=False)
    out = dict(eng.stream(mixed, None))
    assert all(json.loads(o) for o in out.values())
    assert eng.stats["unshared_prefills"] >= 1
    alone = LocalEngine(tiny, use_graphs=False, shared_prefix=False).generate([inputs[2]], other)[0]
    assert out[2] == alone


def test_prefill_batch_matches_single_prefills(tiny):
    """Packed multi-sequence prefill (one pass over every token, varlen
    attention) == one forward_tokens per sequence, with and without the
    shared prefix."""
    seqs = [list(b"class A { void a() {} }"), list(b"class Bee { int b; long c; }"), list(b"x")]
    single = [tiny.forward_tokens(torch.tensor([256] + t, dtype=torch.int32), s, 0) for s, t in enumerate(seqs)]
    got = tiny.prefill_batch([([256] + t, s, 0) for s, t in enumerate(seqs)])
    torch.testing.assert_close(got.float(), torch.stack(single).float(), atol=3e-2, rtol=3e-2)
    prefix = [256] + list(b"Shared instructions and README text for every class of the project. " * 2)
    P = tiny.set_prefix(prefix)
    try:
        ref = []
        for s, t in enumerate(seqs):
            tiny.fork_prefix(s)
            ref.append(tiny.forward_tokens(torch.tensor(t, dtype=torch.int32), s, P))
        for s in range(len(seqs)):
            tiny.fork_prefix(s)
        got = tiny.prefill_batch([(t, s, P) for s, t in enumerate(seqs)])
        torch.testing.assert_close(got.float(), torch.stack(ref).float(), atol=3e-2, rtol=3e-2)
    finally:
        tiny.clear_prefix()


def test_prefill_reference_matches_sdpa_extend():
    """reference.prefill_attention (the fp32 oracle of the MFMA prefill
    kernel) == the SDPA + log-sum-exp merge path it replaces, with the
    prefix keys taken from another slot."""
    import math
    from dmcp.models.llm import _extend_attention
    from dmcp.ops import reference
    g = torch.Generator().manual_seed(0)
    T, Hq, Hkv, D, start, P, MAXS = 19, 8, 2, 16, 23, 11, 64
    q = torch.randn(T, Hq, D, generator=g)
    kc = torch.randn(3, Hkv, MAXS, D, generator=g)
    vc = torch.randn(3, Hkv, MAXS, D, generator=g)
    got = reference.prefill_attention(q, kc, vc, 1, start, 2, P, 1 / math.sqrt(D))
    k = torch.cat([kc[2, :, :P], kc[1, :, P:start + T]], 1).unsqueeze(0)
    v = torch.cat([vc[2, :, :P], vc[1, :, P:start + T]], 1).unsqueeze(0)
    exp = _extend_attention(q.transpose(0, 1).unsqueeze(0), k, v, start, 1 / math.sqrt(D))[0].transpose(0, 1)
    torch.testing.assert_close(got, exp, atol=1e-4, rtol=1e-4)
    # start 0: plain causal prefill
    got0 = reference.prefill_attention(q, kc, vc, 0, 0, None, 0, 0.25)
    k0 = kc[0, :, :T].repeat_interleave(Hq // Hkv, 0)
    v0 = vc[0, :, :T].repeat_interleave(Hq // Hkv, 0)
    exp0 = torch.nn.functional.scaled_dot_product_attention(q.transpose(0, 1), k0, v0, is_causal=True, scale=0.25)
    torch.testing.assert_close(got0, exp0.transpose(0, 1), atol=1e-4, rtol=1e-4)


def test_fp8_kv_codec():
    """e4m3 storage: exact on representable values, saturating at +-448,
    relative error <= 2^-4 on normal values."""
    from dmcp.ops.reference import kv_encode, kv_float
    x = torch.tensor([0.0, 1.0, -1.5, 448.0, 1000.0, -1e9, 0.3, 2 ** -6])
    b = kv_encode(x, torch.uint8)
    assert b.dtype == torch.uint8
    y = kv_float(b)
    assert y[:4].tolist() == [0.0, 1.0, -1.5, 448.0] and y[4].item() == 448.0 and y[5].item() == -448.0
    assert abs(y[6].item() - 0.3) <= 0.3 * 2 ** -4 and y[7].item() == 2 ** -6
    assert kv_encode(x, torch.bfloat16).dtype == torch.bfloat16


def test_fp8_kv_model_tracks_bf16_model():
    """The tiny model with an fp8 KV cache (CPU reference ops) stays close to
    the bf16-cache model on prefill + shared-prefix extend + decode."""
    a = LocalLM(preset("tiny", max_batch=4, max_rows=16, max_seq=768), device="cpu", seed=1)
    b = LocalLM(preset("tiny", max_batch=4, max_rows=16, max_seq=768, kv_dtype="fp8"), device="cpu", seed=1,
                weights=a.w)
    assert b.k_cache.dtype == torch.uint8 and b.cfg.kv_bytes() * 2 == a.cfg.kv_bytes()
    toks = torch.tensor([256] + list(b"public class OrderService { void create() {} }"), dtype=torch.int32)
    la, lb = a.forward_tokens(toks, 0, 0).float(), b.forward_tokens(toks, 0, 0).float()
    assert torch.nn.functional.cosine_similarity(la, lb, dim=0) > 0.99
    for m in (a, b):
        m.set_prefix(toks[:20].tolist())
        m.fork_prefix(1)
        m.forward_tokens(toks[20:], 1, 20)
    step = [m.decode(torch.tensor([65, 66], dtype=torch.int32), torch.tensor([0, 1], dtype=torch.int32),
                     torch.tensor([len(toks), len(toks)], dtype=torch.int32)).float() for m in (a, b)]
    assert torch.nn.functional.cosine_similarity(step[0], step[1], dim=1).min() > 0.99


def test_fused_shape_contract():
    from dmcp.models.llm import fused_shapes_ok
    assert fused_shapes_ok(preset("dmcp-coder-1b")) and fused_shapes_ok(preset("tiny"))
    assert not fused_shapes_ok(preset("tiny", vocab_size=32001))
    assert not fused_shapes_ok(preset("tiny", vocab_size=50257))
    assert not fused_shapes_ok(preset("tiny", intermediate=520))


class _Forcing(LocalLM):
    """The tiny model with a fixed bias added to every logit row: greedy
    decoding then follows the bias wherever the grammar leaves a choice."""

    def __init__(self, bias, **kw):
        super().__init__(preset("tiny", max_batch=4, max_rows=16, max_seq=2048), device="cpu", seed=1, **kw)
        self.bias = torch.zeros(self.cfg.vocab_size)
        for ch, v in bias.items():
            self.bias[ord(ch)] = v

    def _biased(self, logits):
        return (logits.float() + self.bias).to(logits.dtype)

    def decode(self, *a, **kw):
        return self._biased(super().decode(*a, **kw))

    def prefill_batch(self, reqs):
        return self._biased(super().prefill_batch(reqs))


@pytest.mark.parametrize("pipeline", [False, True])
def test_class_type_correction_is_the_models_choice(pipeline):
    """classTypeCorrection is a grammar choice (null or one of the 10 types,
    ClaudeApiClient.java:101-120): a model that prefers '"', 'E', 'N' writes
    "ENTITY"; one that prefers 'n' writes null."""
    ent = LocalEngine(_Forcing({'"': 30.0, "E": 25.0, "N": 20.0}), pipeline=pipeline, type_choice=True)
    doc = json.loads(ent.generate(_inputs(2)[1:], None)[0])
    assert doc["classTypeCorrection"] == "ENTITY" and ent.stats["type_corrections"] == 1
    keep = LocalEngine(_Forcing({"n": 30.0, "]": 20.0}), pipeline=pipeline, type_choice=True)
    doc = json.loads(keep.generate(_inputs(2)[1:], None)[0])
    assert doc["classTypeCorrection"] is None


@pytest.mark.parametrize("pipeline", [False, True])
def test_business_logic_length_is_the_models_choice(pipeline):
    """1..3 steps, closed when the model picks ']' (any length) or ', "'."""
    stop = LocalEngine(_Forcing({'"': 30.0, "]": 25.0, "n": 26.0}), pipeline=pipeline)
    doc = json.loads(stop.generate(_inputs(3)[2:], None)[0])
    assert [len(m["businessLogic"]) for m in doc["methods"]] == [1, 1, 1]
    more = LocalEngine(_Forcing({'"': 30.0, ",": 25.0, "n": 26.0}), pipeline=pipeline)
    doc = json.loads(more.generate(_inputs(3)[2:], None)[0])
    assert [len(m["businessLogic"]) for m in doc["methods"]] == [3, 3, 3]
    assert more.stats["choice_waits" if pipeline else "decode_steps"] > 0


def test_large_class_gets_every_method_within_max_new_tokens(tiny):
    """A 60-method class under a 1,024-token reply budget: split into parts,
    generated side by side, merged -- every method described, in order."""
    names = [f"handleEvent{i}" for i in range(60)]
    inp = EnrichmentInput("class Big {}", "co.x.Big", "java", "LISTENER", names)
    eng = LocalEngine(tiny, max_new_tokens=1024, fork_methods=False)
    doc = json.loads(eng.generate([inp], None)[0])
    assert [m["methodName"] for m in doc["methods"]] == names
    assert all(m["description"] for m in doc["methods"])
    assert eng.stats["split_classes"] == 1 and eng.stats["reply_parts"] > 1 and eng.stats["methods_dropped"] == 0
    assert eng.reply_budget == 1024
    # method branches: the same class as a head + 60 branches on 4 KV slots
    # (branches hand their slot to the next; never a deadlock)
    fk = LocalEngine(tiny, max_new_tokens=1024)
    doc = json.loads(fk.generate([inp], None)[0])
    assert [m["methodName"] for m in doc["methods"]] == names and all(m["description"] for m in doc["methods"])
    assert fk.stats["forks"] == 1 and fk.stats["fork_branches"] == 60


def test_method_branches_shorten_the_critical_path():
    """With fork_methods each method decodes as its own sequence from a copy
    of the class head's KV: with slots to spare (a latency-bound batch),
    fewer decode steps for the same classes, every reply complete."""
    roomy = LocalLM(preset("tiny", max_batch=32, max_rows=128, max_seq=2048), device="cpu", seed=1)
    inputs = [EnrichmentInput("class S%d {}" % i, f"co.x.S{i}", "java", "SERVICE",
                              ["alpha", "beta", "gamma", "delta"][: 1 + i % 4]) for i in range(6)]
    seq = LocalEngine(roomy, fork_methods=False)
    fk = LocalEngine(roomy, fork_methods=True)
    a, b = seq.generate(inputs, "readme"), fk.generate(inputs, "readme")
    for r, inp in zip(b, inputs):
        doc = json.loads(r)
        assert [m["methodName"] for m in doc["methods"]] == inp.method_names
        assert doc["classTypeCorrection"] is None or doc["classTypeCorrection"] in CLASS_TYPES
    assert fk.stats["forks"] == 6 and fk.stats["fork_branches"] == sum(len(i.method_names) for i in inputs)
    assert fk.stats["decode_steps"] < 0.7 * seq.stats["decode_steps"]
    # the first method of each class sees exactly the sequential context: same text
    for ra, rb in zip(a, b):
        assert json.loads(ra)["methods"][0] == json.loads(rb)["methods"][0]


def test_fork_skipped_for_long_own_context():
    """In a full batch, a class whose own prompt exceeds fork_max_context
    decodes its methods in one sequence: the same replies as
    fork_methods=False, counted in stats["fork_skipped"].  A small
    (latency-bound) batch -- every class fits in 3/4 of the slots -- forks
    it anyway (its branches read the head's KV in place)."""
    tight = LocalLM(preset("tiny", max_batch=4, max_rows=128, max_seq=2048), device="cpu", seed=1)
    inputs = [EnrichmentInput("class S%d {}" % i, f"co.x.S{i}", "java", "SERVICE",
                              ["alpha", "beta", "gamma"][: 1 + i % 3]) for i in range(4)]
    seq = LocalEngine(tight, fork_methods=False)
    capped = LocalEngine(tight, fork_methods=True, fork_max_context=8)
    assert capped.generate(inputs, "readme") == seq.generate(inputs, "readme")
    assert capped.stats["fork_skipped"] == 4 and capped.stats["forks"] == 0
    both = LocalEngine(tight, fork_methods=True, fork_max_context=100000)
    out = both.generate(inputs, "readme")
    assert both.stats["fork_skipped"] == 0 and both.stats["forks"] == 4
    assert all(json.loads(o) for o in out)
    roomy = LocalLM(preset("tiny", max_batch=32, max_rows=128, max_seq=2048), device="cpu", seed=1)
    small = LocalEngine(roomy, fork_methods=True, fork_max_context=8)
    out = small.generate(inputs, "readme")
    assert small.stats["fork_skipped"] == 0 and small.stats["forks"] == 4
    assert all(json.loads(o) for o in out)


def test_class_type_correction_reaches_the_database(tmp_path):
    """The model's correction is applied to source_classes.class_type
    (CodeContextService.java:635-637) through the real pipeline."""
    from conftest import make_app
    from dmcp.utils import synth
    repo = tmp_path / "shop"
    synth.java_spring_repo(str(repo), 8)
    be = LocalLLMBackend([LocalEngine(_Forcing({'"': 30.0, "D": 25.0, "]": 20.0}), type_choice=True)])
    app = make_app(tmp_path, backend=be)
    r = app.indexer.analyze_project(str(repo))
    assert r.success and r.stats["enriched"] == r.classes_analyzed
    types = {c.class_type.value for c in app.repos.classes.find_by_project_id(r.project_id)}
    assert types == {"DTO"}
    g = app.cache.get_graph(r.project_id)
    assert g.node_info("co.acme.shop.order.OrderService").class_type == "DTO"
    app.db.close()


def test_bpe_vocabulary_engine_on_cpu():
    """The 128,256-id code tokenizer drives the same engine: forced skeleton,
    choice masks and free strings over BPE pieces; replies parse."""
    from dmcp.enrich.local import build_model
    model, tok = build_model({"preset": "tiny-bpe", "seed": 3}, "cpu")
    assert model.cfg.vocab_size == 128256 and tok.bos == 128000
    eng = LocalEngine(model, tokenizer=tok)
    out = eng.generate(_inputs(3), "A readme")
    for r, inp in zip(out, _inputs(3)):
        doc = json.loads(r)
        assert [m["methodName"] for m in doc["methods"]] == inp.method_names
    text = open(__file__).read()
    assert len(text.encode()) / len(tok.encode(text)) > 3.0  # ~4 bytes per token on source code


@pytest.mark.parametrize("pipeline", [True, False])
def test_native_grammar_engine_matches_the_python_engine(tiny, pipeline):
    """native/grammar/engine.cpp (the production step builder) generates
    exactly what the Python reference implementation does: forced skeleton,
    choices, split parts, jump-forward, mixed projects."""
    from dmcp.enrich.local import _SharedFeed  # noqa: F401  (module imports fine)
    readme, other = "A README shared by every prompt. " * 4, "Another project's README. " * 4
    inputs = _inputs(9) + [EnrichmentInput("class Big {}", "co.x.Big", "java", "LISTENER",
                                           [f"onEvent{i}" for i in range(30)])]
    items = [(i, inp, other if i % 4 == 3 else readme) for i, inp in enumerate(inputs)]
    py = LocalEngine(tiny, pipeline=pipeline, native_grammar=False, max_new_tokens=900, type_choice=True)
    nat = LocalEngine(tiny, pipeline=pipeline, native_grammar=True, max_new_tokens=900, type_choice=True)
    assert py._native is None and nat._native is not None
    a, b = dict(py.stream(items, None)), dict(nat.stream(items, None))
    assert a == b
    for k in ("decode_steps", "decode_rows", "choice_waits", "type_corrections", "split_classes"):
        assert py.stats[k] == nat.stats[k], k
    for k in ("forks", "fork_branches"):
        assert py.stats[k] == nat.stats[k], k
    assert nat.stats["forks"] > 0 and nat._native.n_templates() == 0  # all released
    # an abandoned stream leaves nothing behind for the next one
    g = nat.stream(items, None)
    next(g)
    g.close()
    assert nat._native.n_active() == 0 and nat._native.n_templates() == 0
    assert dict(nat.stream(items[:3], None)) == {k: v for k, v in a.items() if k < 3}


def test_prefill_fp8_close_to_bf16():
    """prefill_dtype fp8 (MXFP8 activations x e4m3 weights, the CPU references
    of csrc/pgemm.hip) stays close to the bf16 prefill of the same weights,
    and the engine decodes valid replies after it."""
    cfg = dict(max_batch=4, max_rows=16, max_seq=2048)
    a = LocalLM(preset("tiny", **cfg), device="cpu", seed=3)
    b = LocalLM(preset("tiny", prefill_dtype="fp8", **cfg), device="cpu", seed=3)
    assert b.prefill_fp8 and set(b.w8) == {f"l{i}.{n}" for i in range(b.cfg.layers)
                                          for n in ("wqkv", "wo", "wgu", "wdown")}
    seqs = [[256] + list(b"class A { void a() {} }"), [256] + list(b"interface Bee { int b(); }"), [256, 65]]
    la = a.prefill_batch([(t, s, 0) for s, t in enumerate(seqs)]).float()
    lb = b.prefill_batch([(t, s, 0) for s, t in enumerate(seqs)]).float()
    cos = torch.nn.functional.cosine_similarity(la, lb, dim=-1)
    assert (cos > 0.98).all(), cos
    ka, kb = a.k_cache[:, :3].float(), b.k_cache[:, :3].float()
    assert (ka - kb).norm() / ka.norm() < 0.1
    one = b.prefill_batch([(seqs[0], 3, 0)]).float()  # a single sequence takes the fp8 path too
    torch.testing.assert_close(one[0], lb[0], atol=2e-2, rtol=2e-2)
    eng = LocalEngine(b, use_graphs=False)
    out = eng.generate(_inputs(3), "readme")
    assert all(json.loads(o) for o in out)


def test_decode_fp8_greedy_agreement_with_bf16():
    """decode_dtype fp8 (e4m3 weights x MXFP8 activations; the CPU references
    of csrc/pgemm.hip's decode GEMM) against bf16 decode of the same weights:
    the step's final hidden rows stay close, greedy tokens mostly agree, and
    the engine's replies stay valid JSON."""
    cfg = dict(max_batch=4, max_rows=16, max_seq=2048)
    a = LocalLM(preset("tiny", **cfg), device="cpu", seed=5)
    b = LocalLM(preset("tiny", decode_dtype="fp8", **cfg), device="cpu", seed=5)
    assert b.decode_fp8 and not b.prefill_fp8
    prompt = [256] + list(b"public class Agreement { void run() {} }")
    for m in (a, b):
        m.prefill_batch([(prompt, 0, 0)])
    # 20 greedy steps: each model from its own token (the usual fp8 deployment check)
    ta, tb = [65], [65]
    agree = 0
    for step in range(20):
        p = len(prompt) + step
        la = a.decode(torch.tensor([ta[-1]], dtype=torch.int32), torch.tensor([0], dtype=torch.int32),
                      torch.tensor([p], dtype=torch.int32)).float()
        lb = b.decode(torch.tensor([tb[-1]], dtype=torch.int32), torch.tensor([0], dtype=torch.int32),
                      torch.tensor([p], dtype=torch.int32)).float()
        if step == 0:
            assert torch.nn.functional.cosine_similarity(la, lb, dim=-1).item() > 0.98
        ta.append(int(la.argmax()))
        tb.append(int(lb.argmax()))
        agree += ta[-1] == tb[-1]
    assert agree >= 14, (ta, tb)
    out = LocalEngine(b, use_graphs=False).generate(_inputs(3), "readme")
    assert all(json.loads(o) for o in out)


def test_prefill_dtype_auto_is_bf16_off_gpu():
    """prefill_dtype "auto" (the service default) picks the MX kernels only on
    a gfx950 device; on the CPU it is the bf16 path, and unknown names fail."""
    import pytest as _pytest
    from dmcp.config import Config
    from dmcp.models.llm import LocalLM, preset
    assert Config().local_llm_prefill_dtype == "auto"
    m = LocalLM(preset("tiny", prefill_dtype="auto", max_batch=2, max_seq=256), device="cpu", seed=0)
    assert not m.prefill_fp8
    with _pytest.raises(ValueError):
        LocalLM(preset("tiny", prefill_dtype="int8", max_batch=2, max_seq=256), device="cpu", seed=0)


def test_branches_read_the_head_kv_in_place_as_a_copy_would():
    """Method branches read their class head's keys from the anchor slot in
    place (LocalLM.fork_share + the fork table of the decode attention):
    the replies equal an engine whose branches get a copy of the head's KV
    (fork_kv), with the slots handed around on 4 KV slots; every slot owns
    its keys again afterwards."""
    names = [f"m{i}" for i in range(9)]
    inputs = [EnrichmentInput("class S%d { int x; }" % i, f"co.x.S{i}", "java", "SERVICE", names[: 3 + 2 * i])
              for i in range(3)]
    m = LocalLM(preset("tiny", max_batch=4, max_rows=64, max_seq=2048), device="cpu", seed=2)
    shared = LocalEngine(m, use_graphs=False).generate(inputs, "readme")
    assert int(m.fork_tab[:, 1].max()) == 0

    class Copying(LocalLM):
        def fork_share(self, src, dsts, end):  # the pre-sharing behaviour: copy [P, end)
            self.fork_kv(src, dsts, self.prefix_len, end)

    c = Copying(preset("tiny", max_batch=4, max_rows=64, max_seq=2048), device="cpu", seed=2)
    copied = LocalEngine(c, use_graphs=False).generate(inputs, "readme")
    assert shared == copied


def test_decode_attention_fork_table_matches_copied_kv():
    """reference decode_attention: a row whose slot has a parent reads the
    keys below the fork end from the parent slot -- the same as copying them."""
    from dmcp.ops import reference as R
    g = torch.Generator().manual_seed(0)
    S, H, T, D, G = 6, 2, 64, 16, 2
    kc, vc = torch.randn(S, H, T, D, generator=g).bfloat16(), torch.randn(S, H, T, D, generator=g).bfloat16()
    q = torch.randn(3, H * G, D, generator=g).bfloat16()
    slot = torch.tensor([1, 3, 4], dtype=torch.int32)
    seq = torch.tensor([40, 50, 9], dtype=torch.int32)
    fork = torch.stack([torch.arange(S), torch.zeros(S, dtype=torch.long)], 1).to(torch.int32)
    fork[3] = torch.tensor([0, 30])
    fork[4] = torch.tensor([0, 30])  # end past the row's length: all its keys from the parent
    got = R.decode_attention(q, kc, vc, slot, seq, 0.25, fork=fork)
    k2, v2 = kc.clone(), vc.clone()
    k2[3, :, :30], v2[3, :, :30] = kc[0, :, :30], vc[0, :, :30]
    k2[4, :, :9], v2[4, :, :9] = kc[0, :, :9], vc[0, :, :9]
    exp = R.decode_attention(q, k2, v2, slot, seq, 0.25)
    assert torch.equal(got, exp)


def test_random_weights_never_correct_class_types(tmp_path):
    """A random-initialised preset (no checkpoint) gets a forced
    ``"classTypeCorrection": null``: a model that would pick "DTO" given the
    choice leaves every statically inferred class type as it was, through
    the real pipeline."""
    from conftest import make_app
    from dmcp.utils import synth
    forcing = _Forcing({'"': 30.0, "D": 25.0, "]": 20.0})
    assert forcing.checkpoint is None
    eng = LocalEngine(forcing)
    assert not eng.type_choice
    doc = json.loads(eng.generate(_inputs(2)[1:], None)[0])
    assert doc["classTypeCorrection"] is None and eng.stats["type_corrections"] == 0
    repo = tmp_path / "shop"
    synth.java_spring_repo(str(repo), 8)
    app = make_app(tmp_path, backend=LocalLLMBackend([LocalEngine(_Forcing({'"': 30.0, "D": 25.0, "]": 20.0}))]))
    r = app.indexer.analyze_project(str(repo))
    assert r.success and r.stats["enriched"] == r.classes_analyzed
    types = {c.full_class_name: c.class_type.value for c in app.repos.classes.find_by_project_id(r.project_id)}
    assert types["co.acme.shop.order.OrderService"] == "SERVICE" and "DTO" not in set(types.values()) - {"DTO"}
    assert len(set(types.values())) > 1  # the static types, not one forced type
    app.db.close()
    forcing.checkpoint = "/some/checkpoint"
    assert LocalEngine(forcing).type_choice  # a loaded checkpoint makes its own choice


def test_reply_shape_derives_from_the_budget_and_config():
    """String caps and the step count scale with the reply budget (the
    reference's free-length contract, ClaudeApiClient.java:40, 101-113) and
    each can be set; the legacy caps are the 1,536-token floor."""
    from dmcp.config import Config
    from dmcp.enrich.local import ReplyShape
    from dmcp.enrich.workers import engine_spec
    assert ReplyShape.from_budget(1536) == ReplyShape.LEGACY == ReplyShape(96, 64, 40, 3)
    assert ReplyShape.from_budget(4096) == ReplyShape(256, 128, 64, 4)
    assert ReplyShape.from_budget(16384) == ReplyShape(512, 256, 160, 6)
    assert ReplyShape.from_budget(4096, desc=1000, max_steps=2) == ReplyShape(1000, 128, 64, 2)
    cfg = Config.from_env({"LOCAL_LLM_DESC_MAX_BYTES": "300", "LOCAL_LLM_MAX_STEPS": "5"})
    spec = engine_spec(cfg)
    assert spec["reply_shape"] == {"desc": 300, "method": 0, "step": 0, "max_steps": 5}
    tiny = LocalLM(preset("tiny", max_batch=4, max_rows=16, max_seq=8192), device="cpu", seed=1)
    eng = LocalEngine(tiny, use_graphs=False, **spec)
    assert eng.reply_budget == 4096
    assert eng.reply_shape == ReplyShape(300, 128, 64, 5)
    segs = build_template(["a"], *eng.reply_shape.scaled(1.0), eng.reply_shape.max_steps)
    assert max(s.max_len for s in segs if s.is_free) == 300


class _Pattern(_Forcing):
    """Greedy text "abc abc ..." by position (row bias = one byte of the
    4-byte cycle at the row's position)."""

    def __init__(self):
        super().__init__({})
        self.cycle = [ord(c) for c in "abc "]

    def decode(self, tokens, slots, positions, *a, **kw):
        lg = LocalLM.decode(self, tokens, slots, positions, *a, **kw).float()
        for r, p in enumerate(positions.tolist()):
            lg[r, self.cycle[p % 4]] += 40.0
        return lg.to(torch.bfloat16)


@pytest.mark.parametrize("native", [False, True])
def test_capped_string_closes_at_a_word_boundary(native):
    """A free string that reaches its byte cap ends at its last space (never
    mid-word, no trailing space); the native grammar engine cuts the same."""
    from dmcp.enrich.local import ReplyShape, _trim_to_word
    eng = LocalEngine(_Pattern(), use_graphs=False, native_grammar=native, reply_shape=ReplyShape(41, 30, 22, 1))
    doc = json.loads(eng.generate(_inputs(2)[1:], None)[0])
    texts = [(doc["description"], 41)] + [(m["description"], 30) for m in doc["methods"]] + \
        [(st, 22) for m in doc["methods"] for st in m["businessLogic"]]
    for text, cap in texts:
        # byte tokens reach the cap exactly; the cut shortens every string
        assert 0 < len(text.encode()) < cap and text[-1] != " " and " " in text, (text, cap)
        assert set(text.split(" ")[-1]) <= set("abc")
    b = bytearray(b'{"x": "alpha beta gam')
    _trim_to_word(b, 7)
    assert bytes(b) == b'{"x": "alpha beta'
    b = bytearray(b'{"x": "al phabetagam')  # the last space is in the first half: cut at the cap
    _trim_to_word(b, 7)
    assert bytes(b) == b'{"x": "al phabetagam'
