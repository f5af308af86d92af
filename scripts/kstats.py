#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv by op category (per decode step).

    python scripts/kstats.py gpurun_out/prof_prefix/enrich_kernel_stats.csv [decode_attn_calls_per_step]
"""
import collections
import csv
import re
import sys

CATS = [("tgemm_head", re.compile(r"tgemm_kernel<\d+, 3|tgemm_argmax_reduce")),  # reduce: before round 6
        ("tgemm_swiglu", re.compile(r"tgemm_kernel<\d+, 2")), ("tgemm", "tgemm_kernel"),
        ("lm_head_argmax", re.compile(r"wgemm_kernel<\d+, \d+, \d+, 3|lm_head_reduce|argmax_pairs")),
        ("wgemm_swiglu", re.compile(r"wgemm_kernel<\d+, \d+, \d+, 2")), ("wgemm", "wgemm_kernel"),
        ("wmx_swiglu(fp8)", re.compile(r"wmx_kernel<\d+, \d+, 2")), ("wmx(fp8)", "wmx_kernel"),
        ("pgemm(fp8)", "pgemm_kernel"), ("mx_quant", re.compile(r"mx_quant|rmsnorm_mx|resid_norm_mx")),
        ("wgemm_reduce", "reduce_"),
        ("attn_prefix(mfma)", "prefill_attn_kernel"), ("prefill_varlen", "prefill_varlen"),
        ("gemm(hipblaslt)", "Cijk"), ("fused_gemm", "fused_gemm"), ("attn_combine", "combine"),
        ("attn_per_row", "decode_attn_"), ("rmsnorm", "rmsnorm"), ("silu", "silu"),
        ("rope", "rope"), ("embedding", "embedding"), ("argmax", "argmax")]


def _match(key, name: str) -> bool:
    return key.search(name) is not None if hasattr(key, "search") else key in name


def main() -> int:
    rows = list(csv.DictReader(open(sys.argv[1])))
    layers = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    cat = collections.Counter()
    steps = 0
    for r in rows:
        name = r["Name"]
        if "decode_attn_" in name and "combine" not in name:
            steps = int(r["Calls"]) // layers
    for r in rows:
        name, t = r["Name"], int(r["TotalDurationNs"])
        for c, key in CATS:
            if _match(key, name):
                cat[c] += t
                break
        else:
            # kernels of no category launched less than once per two steps
            # are the process's one-time work (weight init / quantisation, KV
            # cache zero-fill), not the step path's
            cat["other" if int(r["Calls"]) * 2 >= max(1, steps) else "other(one-time)"] += t
    total = sum(cat.values())
    print(f"total {total / 1e6:.1f} ms over {steps} decode steps")
    for k, v in cat.most_common():
        print(f"  {k:14s} {v / 1e6:9.1f} ms  {100 * v / total:5.1f}%  per-step {v / 1e3 / max(1, steps):8.1f} us")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
