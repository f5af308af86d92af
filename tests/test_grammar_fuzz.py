"""Seeded fuzzing of the native grammar engine (native/grammar/engine.cpp)
against the Python state machine of dmcp/enrich/local.py.

The native engine parses templates, choice tables and id streams handed over
from Python and indexes its vectors on every decode step of the GPU worker
(native C++ under sanitizers and fuzz).  Each iteration draws a
random reply grammar -- method names (escaped and unicode ones included),
string caps, step counts, the class-type choice on or off, reply budgets
small enough to split classes into parts or shrink their branches -- and a
random engine configuration (one-step pipeline, jump-forward, method forks,
shared prefix over two projects, batch and row limits), then streams the
classes through two engines that differ only in the grammar implementation.
The "model" is a hash of (token, position, slot) into a table of random
logits with a random bias toward closing strings, so thousands of
iterations run in seconds; the replies and step statistics must be equal.

``DMCP_GRAMMAR_FUZZ_ITERS`` scales the run (default 300; scripts/asan_tests.sh
runs 6,000 with the ASan/UBSan build of the module loaded through
``DMCP_GRAMMAR_SO``).
"""
import json
import os
import random

import numpy as np
import pytest
import torch

from dmcp.enrich.local import LocalEngine, ReplyShape
from dmcp.enrich.types import EnrichmentInput
from dmcp.models.llm import LocalLM, preset

ITERS = int(os.environ.get("DMCP_GRAMMAR_FUZZ_ITERS", "300"))
NT = 4093  # rows of the logit table (prime)


class _HashLM(LocalLM):
    """The tiny preset's shapes and KV bookkeeping with a hashed "model":
    the logits of a (token, position, slot) row are a fixed random table row
    plus a bias toward the quote (strings close at random lengths)."""

    def __init__(self, max_batch: int, max_rows: int):
        super().__init__(preset("tiny", max_batch=max_batch, max_rows=max_rows, max_seq=1024), device="cpu", seed=0)
        self.table = torch.zeros(NT, self.cfg.vocab_size)
        self.reseed(0, 0.0)

    def reseed(self, seed: int, quote_bias: float) -> None:
        g = torch.Generator().manual_seed(seed)
        t = torch.randn(NT, self.cfg.vocab_size, generator=g)
        t[:, ord('"')] += quote_bias
        self.table = t.to(torch.bfloat16)
        self.np_table = self.table.float().numpy()

    def _hash(self, toks, pos, slots):
        return (np.asarray(toks, np.int64) * 7919 + np.asarray(pos, np.int64) * 104729
                + np.asarray(slots, np.int64) * 13) % NT

    def forward_tokens(self, tokens, slot, start_pos):  # the shared prefix prefill
        return self.table[int(self._hash(int(tokens[-1]), start_pos + len(tokens) - 1, slot))]

    def prefill_batch(self, reqs):
        h = self._hash([int(t[-1]) for t, _, _ in reqs], [st + len(t) - 1 for t, _, st in reqs],
                       [sl for _, sl, _ in reqs])
        return self.table[torch.from_numpy(h)]

    _bits_cache = {}

    def _allowed(self, masks):
        key = masks.numpy().tobytes()  # every engine over this vocabulary builds the same rows
        if key not in self._bits_cache:
            V = self.cfg.vocab_size
            w = masks.numpy().astype(np.int64) & 0xFFFFFFFF
            idx = np.arange(V)
            self._bits_cache[key] = ((w[:, idx // 32] >> (idx % 32)) & 1).astype(bool)
        return self._bits_cache[key]

    def decode_select_gather(self, tokens, src, last_ids, slots, positions, masks, mask_idx, mask_alt=None,
                             alt_token=-1, prefix_rows=None):
        """The engine's step contract (reference.decode_embed_norm's gather and
        mask switch, then the masked greedy selection) on the hashed logits."""
        B = tokens.shape[0]
        s, li, mi = src.numpy(), last_ids.numpy(), mask_idx.numpy()
        gathered = li[np.clip(s, 0, li.size - 1)]
        toks = np.where(s >= 0, gathered, tokens.numpy())
        if mask_alt is not None:
            ma = mask_alt.numpy()
            mi[:] = np.where((s >= 0) & (gathered == alt_token) & (ma >= 0), ma, mi)
        allowed = self._allowed(masks)
        rows = self.np_table[self._hash(toks, positions.numpy(), slots.numpy())]
        x = np.where(allowed[np.clip(mi, 0, allowed.shape[0] - 1)], rows, -np.inf)
        li[:B] = np.argmax(x, axis=1)  # first index among ties; 0 when nothing is allowed
        return None, last_ids[:B]


_MODELS = {}


def _model(max_batch: int, max_rows: int) -> _HashLM:
    key = (max_batch, max_rows)
    if key not in _MODELS:
        _MODELS[key] = _HashLM(max_batch, max_rows)
    return _MODELS[key]


_NAME_CHARS = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789_$"
_ODD_NAMES = ["<init>", "get\"quoted\"", "back\\slash", "méthode", "方法", "tab\there", "x" * 40, "a b"]


def _names(rng: random.Random):
    out = []
    for _ in range(rng.choice([0, 1, 1, 2, 3, 4, 6])):
        if rng.random() < 0.15:
            out.append(rng.choice(_ODD_NAMES))
        else:
            out.append("".join(rng.choice(_NAME_CHARS) for _ in range(rng.randint(1, 14))))
    if out and rng.random() < 0.2:
        out.append(out[0])  # duplicates collapse (dict.fromkeys)
    return out


def _case(seed: int):
    rng = random.Random(seed)
    model = _model(rng.choice([3, 4, 8]), rng.choice([8, 24, 64]))
    model.reseed(seed, rng.uniform(-1.0, 4.0))
    shape = ReplyShape(rng.randint(4, 40), rng.randint(4, 30), rng.randint(4, 20), rng.randint(1, 4))
    kw = dict(use_graphs=False, pipeline=rng.random() < 0.6, jump_forward=rng.random() < 0.8,
              fork_methods=rng.random() < 0.6, fork_max_context=rng.choice([0, 8, 100000]),
              shared_prefix=rng.random() < 0.7, max_new_tokens=rng.choice([None, 200, 300, 500, 900]),
              reply_shape=shape, type_choice=rng.random() < 0.5, longest_first=rng.random() < 0.5)
    readmes = ["Project one README. " * rng.randint(2, 5), "Another project, another README. " * rng.randint(2, 5)]
    items = []
    for i in range(rng.randint(1, 7)):
        src = "class C%d { %s }" % (i, " ".join("void m%d() {}" % k for k in range(rng.randint(0, 3))))
        inp = EnrichmentInput(src, f"co.f.C{i}", "java", rng.choice(["SERVICE", "DTO", "OTHER"]), _names(rng))
        items.append((i, inp, readmes[0] if rng.random() < 0.75 else readmes[1]))
    return model, kw, items


def _run(model, kw, items, native: bool):
    eng = LocalEngine(model, native_grammar=native, **kw)
    out = dict(eng.stream(list(items), None))
    if native:
        assert eng._native.n_active() == 0 and eng._native.n_templates() == 0
    return out, {k: eng.stats[k] for k in ("decode_steps", "decode_rows", "choice_waits", "type_corrections",
                                           "split_classes", "forks", "fork_branches", "generated_tokens",
                                           "methods_dropped")}


@pytest.mark.timeout(3600)  # 6,000 iterations under ASan (scripts/asan_tests.sh)
def test_grammar_fuzz_native_matches_python():
    from dmcp.enrich.local import _grammar_module
    mod = _grammar_module()
    if os.environ.get("DMCP_GRAMMAR_SO"):
        assert mod.__file__ == os.environ["DMCP_GRAMMAR_SO"]
    bad = []
    for it in range(ITERS):
        model, kw, items = _case(1000 + it)
        a, sa = _run(model, kw, items, native=False)
        b, sb = _run(model, kw, items, native=True)
        if a != b or sa != sb:
            bad.append((1000 + it, kw, sa, sb))
            continue
        missing = 0
        for k, raw in a.items():
            doc = json.loads(raw)  # every reply parses; its methods in order, none but the counted drops missing
            got = [m["methodName"] for m in doc["methods"]]
            want = list(dict.fromkeys(items[k][1].method_names))
            it_w = iter(want)
            assert all(n in it_w for n in got), (got, want)
            missing += len(want) - len(got)
        assert missing == sa["methods_dropped"]
    assert not bad, bad[:3]


def test_native_engine_rejects_malformed_templates():
    """Out-of-range choice ids and branch indices are refused by add_template
    (no out-of-bounds access later)."""
    from dmcp.enrich.local import _grammar_module
    eng = _grammar_module().Engine([b"a", b'"'], 1, [[b"null", b'"X"']], {(0, b""): 2}, {}, True, True, 8)
    with pytest.raises(ValueError):
        eng.add_template([[(2, [], 0, 0, 5, [])]])
    with pytest.raises(ValueError):
        eng.add_template([[(2, [], 0, 0, 0, [7])]])
    with pytest.raises(ValueError):
        eng.add_template([])
    t = eng.add_template([[(0, [0], 0, 0, -1, []), (1, [], 0, 3, -1, [])]])
    h = eng.new_seq(t)
    assert eng.admit(h, 0, 5, False) == 1  # free string with min_len 0: the quote is allowed
    import numpy as np
    with pytest.raises(ValueError):
        eng.build(np.zeros((3, 4), dtype=np.int32), 0)  # fewer than the 7 step rows
