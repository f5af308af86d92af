#!/usr/bin/env python3
"""Block timeline of the MX prefill GEMM (GPU box), from a library built with
PG_PROBE=4 (scripts/pgemm_probe.py 4): per block s_memtime at start, after the
K loop and after the epilogue.  Prints the mean K-loop and epilogue spans per
block and the idle gaps between consecutive blocks on a CU, per shape.

    DMCP_HIPOPS_SO=dmcp/ops/variants/probe4.so python scripts/pgemm_stamps.py
"""
import collections
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main() -> int:
    from dmcp import ops
    from dmcp.ops import hip
    lib = hip.lib()
    M = 24576
    for name, N, K in (("gate_up", 16384, 2048), ("down", 2048, 8192), ("qkv", 3072, 2048)):
        g = torch.Generator(device="cuda").manual_seed(0)
        x = (torch.randn(M, K, generator=g, device="cuda") * 2).to(torch.bfloat16)
        w = (torch.randn(N, K, generator=g, device="cuda") * 0.03).to(torch.bfloat16)
        aq, as_ = hip.mx_quant(x)
        wq, ws = ops.quantize_weight(w)
        for _ in range(3):
            hip.pgemm(aq, as_, wq, ws)
        torch.cuda.synchronize()
        nblk = (M // 256) * (N // 256)
        buf = (ctypes.c_longlong * (nblk * 4))()
        assert lib.dmcp_pg_stamps(ctypes.cast(buf, ctypes.c_void_p), nblk) == 0
        # hw id bits 8-15: CU / SH / SE inside an XCD; blockIdx % 8: the XCD (round-robin dispatch)
        st = [(buf[4 * b], buf[4 * b + 1], buf[4 * b + 2], ((buf[4 * b + 3] >> 8) & 0xFF) * 8 + b % 8)
              for b in range(nblk)]
        t0 = min(s[0] for s in st)
        loop = sum(s[1] - s[0] for s in st) / nblk
        epi = sum(s[2] - s[1] for s in st) / nblk
        # per CU (hw id without the wave / simd bits): gaps between a block's end and the next start
        bycu = collections.defaultdict(list)
        for s in st:
            bycu[s[3]].append(s)
        gaps = []
        for v in bycu.values():
            v.sort()
            gaps += [b[0] - a[2] for a, b in zip(v, v[1:])]
        span = max(s[2] for s in st) - t0
        first = sorted(s[0] - t0 for s in st)
        print(json.dumps({"proj": name, "blocks": nblk, "cus_seen": len(bycu), "span_cycles": span,
                          "loop_cycles": round(loop), "epilogue_cycles": round(epi),
                          "gap_cycles_mean": round(sum(gaps) / max(1, len(gaps))),
                          "blocks_per_cu": round(nblk / max(1, len(bycu)), 2),
                          "first_wave_start_spread": first[min(255, nblk - 1)]}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
