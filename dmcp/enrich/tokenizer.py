"""Tokenizers of the local enrichment engine -- MI355X extension.

The engine (:class:`dmcp.enrich.local.LocalEngine`) forces the JSON skeleton
of every reply and samples only string contents under a per-row vocabulary
mask.  It needs four things from a tokenizer, all precomputed here so the
per-step grammar loop stays table lookups:

* ``encode(text)`` -- prompt and forced-skeleton ids;
* ``token_bytes[id]`` -- the bytes a token appends to the reply;
* ``quote`` -- the id of the lone ``"`` token that closes a free string;
* :meth:`json_masks` -- bit masks over the model vocabulary of the tokens a
  JSON string may contain (printable ASCII, no ``"`` / ``\\`` / control
  characters, no special tokens), without and with the closing quote.

:class:`ByteTokenizer` is the built-in byte-level vocabulary of the
random-initialised presets (``BOS`` + one id per byte).
:class:`HFTokenizer` reads a checkpoint's ``tokenizer.json`` (byte-level BPE
as in GPT-2 / Llama 3 / Qwen, or SentencePiece-style ``▁`` + ``<0xNN>``
byte fallback) through the ``tokenizers`` library, so a Llama-format
checkpoint loaded by :meth:`dmcp.models.llm.LocalLM.load_safetensors` runs
the same engine with its own vocabulary (:func:`load_local_model`).
"""
from __future__ import annotations

import json
import os
from typing import List, Optional, Sequence, Tuple

BYTE_BOS = 256

_FREE_BYTES = frozenset(b for b in range(0x20, 0x7F) if b not in (ord('"'), ord("\\")))


def _pack_bits(ids: Sequence[int], vocab: int) -> List[int]:
    """int32 words (two's complement view of the uint32 bit pattern) with bit
    ``id`` set for every id of ``ids``."""
    words = [0] * ((vocab + 31) // 32)
    for i in ids:
        words[i >> 5] |= 1 << (i & 31)
    return [w - (1 << 32) if w >= (1 << 31) else w for w in words]


class _Base:
    bos: Optional[int]
    quote: int
    token_bytes: List[bytes]

    def encode(self, text: str) -> List[int]:
        raise NotImplementedError

    def encode_fragment(self, text: str) -> List[int]:
        """Ids that decode to exactly ``text`` wherever they are spliced in
        (forced reply skeleton).  A tokenizer whose pre-tokenizer rewrites the
        start of a text (SentencePiece's dummy-prefix space) falls back to one
        single-byte token per byte."""
        ids = self.encode(text)
        raw = text.encode("utf-8")
        tb = self.token_bytes
        if b"".join(map(tb.__getitem__, ids)) == raw:
            return ids
        bid = self.byte_ids()
        if any(bid[b] < 0 for b in raw):
            raise ValueError(f"tokenizer cannot spell {text!r} exactly")
        return [bid[b] for b in raw]

    def byte_ids(self) -> List[int]:
        """For every byte value the id of a token spelling exactly that byte
        (-1 if none): plain vocabulary pieces before byte-fallback tokens."""
        if getattr(self, "_byte_ids", None) is None:
            out = [-1] * 256
            for i in sorted(range(len(self.token_bytes)), key=lambda i: (i in self._fallback_ids, i)):
                b = self.token_bytes[i]
                if len(b) == 1 and out[b[0]] < 0:
                    out[b[0]] = i
            self._byte_ids = out
        return self._byte_ids

    _fallback_ids: frozenset = frozenset()

    def decode(self, ids: Sequence[int]) -> str:
        tb = self.token_bytes
        return b"".join(tb[i] for i in ids if 0 <= i < len(tb)).decode("utf-8", "replace")

    def json_masks(self, vocab: int) -> Tuple[List[int], List[int]]:
        """(no-quote mask, quote mask) over ``vocab`` ids: tokens whose bytes
        are all JSON-string-safe printable ASCII; the second adds the quote."""
        free = [i for i, b in enumerate(self.token_bytes[:vocab])
                if b and i != self.quote and all(c in _FREE_BYTES for c in b)]
        return _pack_bits(free, vocab), _pack_bits(free + [self.quote], vocab)

    def encode_split(self, text: str, marker: str) -> Tuple[List[int], int]:
        """``[bos] + ids`` of ``text`` and the number of leading ids (BOS
        included) encoding the text before ``marker`` (0 when absent).  The
        two sides are encoded separately, so every prompt that shares the
        text before the marker shares those ids exactly."""
        head = [self.bos] if self.bos is not None else []
        i = text.find(marker)
        if i <= 0:
            return head + self.encode(text), 0
        pre = head + self.encode(text[:i])
        return pre + self.encode_continuation(text[i:]), len(pre)

    def encode_continuation(self, text: str) -> List[int]:
        """Ids of ``text`` spliced after other text: exactly its bytes.  A
        SentencePiece-style pre-tokenizer prepends a dummy-prefix space to
        every encode -- a leading lone space token is dropped; a piece that
        merged that space into the first word falls back to
        :meth:`encode_fragment` for that word only."""
        return self._continuation(text, self.encode(text))

    def encode_continuation_batch(self, texts: Sequence[str]) -> List[List[int]]:
        """:meth:`encode_continuation` of several texts (one call: a native
        tokenizer encodes them in parallel)."""
        return [self.encode_continuation(t) for t in texts]

    def _continuation(self, text: str, ids: List[int]) -> List[int]:
        raw = text.encode("utf-8")
        tb = self.token_bytes
        got = b"".join(map(tb.__getitem__, ids))
        if got == raw:
            return ids
        if got == b" " + raw:
            if ids and tb[ids[0]] == b" ":
                return ids[1:]
            # "▁Source" as one piece: re-spell the first piece's text without the space
            first = tb[ids[0]]
            if first.startswith(b" ") and b"".join(tb[i] for i in ids[1:]) == raw[len(first) - 1:]:
                return self.encode_fragment(first[1:].decode("utf-8", "replace")) + ids[1:]
        return self.encode_fragment(text)


class ByteTokenizer(_Base):
    """One id per byte plus BOS (256); EOS / PAD (257 / 258) are never
    sampled.  ``vocab`` is the model's (padded) vocabulary size."""

    def __init__(self, vocab: int = 320) -> None:
        self.bos = BYTE_BOS
        self.quote = ord('"')
        self.token_bytes = [bytes([i]) if i < 256 else b"" for i in range(max(vocab, 259))]

    def encode(self, text: str) -> List[int]:
        return list(text.encode("utf-8", "replace"))

    def encode_continuation(self, text: str) -> List[int]:
        return self.encode(text)  # one id per byte: always exact

    def encode_fragment(self, text: str) -> List[int]:
        return self.encode(text)


def _byte_level_decoder_map() -> dict:
    """Inverse of GPT-2's bytes_to_unicode: printable bytes map to
    themselves, the other 68 to U+0100 onwards."""
    keep = list(range(ord("!"), ord("~") + 1)) + list(range(0xA1, 0xAD)) + list(range(0xAE, 0x100))
    chars = list(keep)
    n = 0
    for b in range(256):
        if b not in keep:
            keep.append(b)
            chars.append(256 + n)
            n += 1
    return {chr(c): b for b, c in zip(keep, chars)}


class HFTokenizer(_Base):
    """A Hugging Face ``tokenizer.json`` (``tokenizers`` library): a file, a
    checkpoint directory holding one, or (``text``) its JSON text."""

    def __init__(self, path: str = "", bos: Optional[int] = None, text: Optional[str] = None) -> None:
        from tokenizers import Tokenizer
        if text is None:
            file = os.path.join(path, "tokenizer.json") if os.path.isdir(path) else path
            with open(file, encoding="utf-8") as f:
                text = f.read()
        else:
            file = path or "<text>"
        self.tk = Tokenizer.from_str(text)
        spec = json.loads(text)
        special = {t["id"] for t in spec.get("added_tokens") or [] if t.get("special")}
        dec = spec.get("decoder") or {}
        kinds = {dec.get("type")} | {d.get("type") for d in dec.get("decoders") or []}
        byte_level = "ByteLevel" in kinds
        bmap = _byte_level_decoder_map() if byte_level else None
        n = self.tk.get_vocab_size(with_added_tokens=True)
        fallback = set()
        self.token_bytes: List[bytes] = []
        for i in range(n):
            s = self.tk.id_to_token(i)
            if s is not None and not byte_level and len(s) == 6 and s.startswith("<0x") and s.endswith(">"):
                # byte-fallback piece (a byte, even where the file flags it special)
                self.token_bytes.append(bytes([int(s[3:5], 16)]))
                fallback.add(i)
            elif s is None or i in special:
                self.token_bytes.append(b"")
            elif byte_level:
                try:
                    self.token_bytes.append(bytes(bmap[c] for c in s))
                except KeyError:  # an added (non byte-level) token: its literal text
                    self.token_bytes.append(s.encode("utf-8"))
            elif len(s) == 6 and s.startswith("<0x") and s.endswith(">"):
                self.token_bytes.append(bytes([int(s[3:5], 16)]))
                fallback.add(i)
            else:
                self.token_bytes.append(s.replace("▁", " ").encode("utf-8"))
        self._fallback_ids = frozenset(fallback)
        self.quote = self.byte_ids()[ord('"')]
        if self.quote < 0:
            raise ValueError(f"tokenizer {file}: no token spells '\"' alone")
        self.bos = bos

    def encode(self, text: str) -> List[int]:
        return self.tk.encode(text, add_special_tokens=False).ids

    def encode_continuation_batch(self, texts: Sequence[str]) -> List[List[int]]:
        # encode_batch runs the texts on the library's thread pool with the
        # GIL released: 64 prompts of ~500 tokens in ~11 ms instead of ~60 ms
        encs = self.tk.encode_batch(list(texts), add_special_tokens=False)
        return [self._continuation(t, e.ids) for t, e in zip(texts, encs)]


def load_tokenizer(path: str) -> HFTokenizer:
    """The tokenizer of a checkpoint directory: ``tokenizer.json`` plus the
    BOS id of ``config.json`` (``bos_token_id``) when the model uses one."""
    bos = None
    cfg = os.path.join(path, "config.json")
    if os.path.isdir(path) and os.path.exists(cfg):
        with open(cfg) as f:
            bos = json.load(f).get("bos_token_id")
        tc = os.path.join(path, "tokenizer_config.json")
        if os.path.exists(tc):
            with open(tc) as f:
                if json.load(f).get("add_bos_token") is False:
                    bos = None
    return HFTokenizer(path, bos=bos if isinstance(bos, int) else None)


ASSETS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "models", "assets")
_PRESET_TOKENIZERS: dict = {}


def load_asset_tokenizer(name: str) -> HFTokenizer:
    """A tokenizer shipped in ``dmcp/models/assets/<name>`` (gzipped
    ``tokenizer.json`` + ``tokenizer_meta.json`` with the BOS id); cached
    per process (building the 128k-id byte tables takes ~1 s)."""
    tok = _PRESET_TOKENIZERS.get(name)
    if tok is None:
        import gzip
        d = os.path.join(ASSETS, name)
        with gzip.open(os.path.join(d, "tokenizer.json.gz"), "rt", encoding="utf-8") as f:
            text = f.read()
        with open(os.path.join(d, "tokenizer_meta.json")) as f:
            meta = json.load(f)
        tok = _PRESET_TOKENIZERS[name] = HFTokenizer(os.path.join(d, "tokenizer.json.gz"),
                                                     bos=meta.get("bos_token_id"), text=text)
    return tok


def load_local_model(path: str, device: str = "cuda", **cfg_overrides):
    """(LocalLM, tokenizer) of a Llama-format checkpoint directory
    (``config.json`` + ``*.safetensors`` + ``tokenizer.json``)."""
    from ..models.llm import LocalLM
    model = LocalLM.load_safetensors(path, device=device, **cfg_overrides)
    tok = load_tokenizer(path)
    if len(tok.token_bytes) > model.cfg.vocab_size:
        # ids past the embedding table (added tokens of the tokenizer) are
        # never produced by the model and never forced (the skeleton is ASCII)
        tok.token_bytes = tok.token_bytes[:model.cfg.vocab_size]
    return model, tok
