#!/usr/bin/env python3
"""Trains the byte-level BPE code tokenizer of the ``llama3.2-1b-code``
preset (dmcp/models/llm.py) -- offline, from source code already on this host.

There is no checkpoint and no network here, so the real-checkpoint operating
point (VERDICT r3 "next" #2) is reproduced by geometry: Llama-3.2-1B shapes
with a 128,256-id vocabulary (128,000 learned BPE pieces + 256 special ids,
the Llama 3 layout) and a tokenizer that compresses source code the way a
production code tokenizer does (~3-4 bytes / token), so prompt and reply
token counts, the LM-head width and the grammar masks all sit where a real
1B code model puts them.

Corpus (all local, deterministic file order): CPython's standard library,
a slice of site-packages Python, C/C++ headers (/usr/include, ROCm), and
synthetic Java / TypeScript / Go projects from :mod:`dmcp.utils.synth`
(the languages this service indexes).  Usage::

    python scripts/train_code_bpe.py [--out dmcp/models/assets/code-bpe-128k]
"""
from __future__ import annotations

import argparse
import glob
import gzip
import json
import os
import random
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N_LEARNED = 128_000
N_SPECIAL = 256


def corpus_files(max_mb: float) -> list:
    pats = [("/usr/lib/python3.10/**/*.py", 12), ("/usr/local/lib/python3.10/dist-packages/**/*.py", 45),
            ("/usr/include/**/*.h", 25), ("/opt/rocm/include/**/*.hpp", 20)]
    out = []
    for pat, mb in pats:
        files = sorted(glob.glob(pat, recursive=True))
        random.Random(0).shuffle(files)
        budget = min(mb, max_mb) * 1e6
        for f in files:
            try:
                n = os.path.getsize(f)
            except OSError:
                continue
            if n > 2_000_000 or n == 0:
                continue
            out.append(f)
            budget -= n
            if budget <= 0:
                break
    return out


def synthetic_sources(work: str) -> list:
    from dmcp.utils import synth
    files = []
    for i in range(6):
        root = os.path.join(work, f"java{i}")
        synth.java_spring_repo(root, n_classes=400, base_package=f"co.acme.p{i}", seed=100 + i)
        root_ts = os.path.join(work, f"ts{i}")
        synth.nestjs_repo(root_ts, n_modules=40, seed=200 + i, commit=False)
        root_go = os.path.join(work, f"go{i}")
        synth.go_gin_repo(root_go, n_packages=30, module=f"github.com/acme/svc{i}", commit=False)
    for ext in ("java", "ts", "go", "md"):
        files += sorted(glob.glob(os.path.join(work, f"**/*.{ext}"), recursive=True))
    return files


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "dmcp", "models", "assets", "code-bpe-128k"))
    ap.add_argument("--max-mb", type=float, default=45.0)
    args = ap.parse_args()
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    from tokenizers import AddedToken
    with tempfile.TemporaryDirectory() as work:
        files = corpus_files(args.max_mb) + synthetic_sources(work)
        size = sum(os.path.getsize(f) for f in files)
        print(f"corpus: {len(files)} files, {size / 1e6:.1f} MB", flush=True)
        tok = Tokenizer(models.BPE())
        tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=True)
        tok.decoder = decoders.ByteLevel()
        trainer = trainers.BpeTrainer(vocab_size=N_LEARNED, min_frequency=2, show_progress=False,
                                      initial_alphabet=pre_tokenizers.ByteLevel.alphabet(), special_tokens=[])

        def lines():
            for f in files:
                try:
                    with open(f, encoding="utf-8", errors="replace") as fh:
                        yield fh.read()
                except OSError:
                    continue
        tok.train_from_iterator(lines(), trainer=trainer, length=len(files))
    learned = tok.get_vocab_size()
    # pad to exactly N_LEARNED ids when the corpus ran out of merges, then
    # the Llama 3 special block: begin/end of text + reserved ids
    specials = ["<|begin_of_text|>", "<|end_of_text|>"] + [f"<|reserved_special_token_{i}|>"
                                                          for i in range(N_SPECIAL - 2)]
    if learned < N_LEARNED:
        specials = [f"<|unused_{i}|>" for i in range(N_LEARNED - learned)] + specials
    tok.add_special_tokens([AddedToken(s, special=True, normalized=False) for s in specials])
    assert tok.get_vocab_size() == N_LEARNED + N_SPECIAL, tok.get_vocab_size()
    os.makedirs(args.out, exist_ok=True)
    raw = tok.to_str().encode("utf-8")
    with gzip.open(os.path.join(args.out, "tokenizer.json.gz"), "wb", compresslevel=9) as f:
        f.write(raw)
    bos = tok.token_to_id("<|begin_of_text|>")
    with open(os.path.join(args.out, "tokenizer_meta.json"), "w") as f:
        json.dump({"bos_token_id": bos, "eos_token_id": tok.token_to_id("<|end_of_text|>"),
                   "learned": learned, "vocab_size": tok.get_vocab_size(), "corpus_files": len(files),
                   "corpus_mb": round(size / 1e6, 1)}, f, indent=1)
    # compression on a held-out synthetic Java project
    with tempfile.TemporaryDirectory() as work:
        from dmcp.utils import synth
        synth.java_spring_repo(os.path.join(work, "h"), n_classes=100, base_package="org.held.out", seed=999)
        text = "".join(open(p, encoding="utf-8").read() for p in glob.glob(os.path.join(work, "h/**/*.java"),
                                                                           recursive=True))
    n = len(tok.encode(text, add_special_tokens=False).ids)
    py = open("/usr/lib/python3.10/json/decoder.py", encoding="utf-8").read()
    npy = len(tok.encode(py, add_special_tokens=False).ids)
    print(json.dumps({"learned": learned, "vocab": tok.get_vocab_size(), "bos": bos,
                      "java_bytes_per_token": round(len(text.encode()) / n, 2),
                      "python_bytes_per_token": round(len(py.encode()) / npy, 2),
                      "size_mb": round(len(raw) / 1e6, 2)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
