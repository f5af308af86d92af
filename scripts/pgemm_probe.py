#!/usr/bin/env python3
"""Builds ablation variants of the HIP library (CPU host) for a same-box A/B
of the MX prefill GEMM's main loop: PG_PROBE=1 (no refill DMAs), 2 (no
per-stage barrier), 3 (neither).  The variants land in dmcp/ops/variants/;
run scripts/bench_pgemm.py with DMCP_HIPOPS_SO pointing at each.

    python scripts/pgemm_probe.py            # builds probe1..3
"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dmcp.ops import build as B  # noqa: E402

OUT = os.path.join(os.path.dirname(B.TARGET), "variants")


def build(name: str, defines: list) -> str:
    os.makedirs(OUT, exist_ok=True)
    objs = []
    for src in B.SRCS:
        obj = os.path.join(OUT, f"{name}_{os.path.basename(src)}.o")
        subprocess.run([B.hipcc(), *B._flags(src), *defines, f"-I{B.CSRC}", "-c", "-o", obj, src], check=True)
        objs.append(obj)
    so = os.path.join(OUT, f"{name}.so")
    subprocess.run([B.hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", so, *objs], check=True)
    for o in objs:
        os.remove(o)
    return so


if __name__ == "__main__":
    for v in (sys.argv[1:] or ["1", "2", "3"]):
        print(build(f"probe{v}", [f"-DPG_PROBE={v}"]))
