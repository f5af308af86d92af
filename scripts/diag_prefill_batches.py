#!/usr/bin/env python3
"""Per-batch device time of the engine's batched prefills during a
bench_enrich run (sequences, tokens, ms per class): wraps
LocalLM.prefill_batch with timing events, then runs bench_enrich.main with the
given arguments.

    python scripts/diag_prefill_batches.py --kv-dtype fp8
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dmcp.models.llm import LocalLM  # noqa: E402

REC = []
_orig = LocalLM.prefill_batch


def timed(self, reqs):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    out = _orig(self, reqs)
    b.record()
    REC.append((len(reqs), sum(len(t) for t, _, _ in reqs), a, b))
    return out


LocalLM.prefill_batch = timed

if __name__ == "__main__":
    import bench_enrich
    rc = bench_enrich.main(sys.argv[1:])
    torch.cuda.synchronize()
    rows = [(n, tok, a.elapsed_time(b)) for n, tok, a, b in REC]
    print("batches", len(rows), "classes", sum(r[0] for r in rows), "gpu_s", round(sum(r[2] for r in rows) / 1e3, 3))
    for lo, hi in ((1, 1), (2, 4), (5, 8), (9, 12), (13, 16), (17, 64)):
        sel = [r for r in rows if lo <= r[0] <= hi]
        if sel:
            ms = sum(r[2] for r in sel)
            cls = sum(r[0] for r in sel)
            tok = sum(r[1] for r in sel)
            print(f"seqs {lo:2d}-{hi:2d}: {len(sel):4d} batches {cls:5d} classes {ms / cls:7.2f} ms/class "
                  f"{tok / ms * 1e3 / 1e3:8.1f} k tok/s")
    raise SystemExit(rc)
