"""Builds the gfx950 HIP kernel library ``dmcp/ops/_hipops.so`` in-tree.

``hipcc --offload-arch=gfx950`` cross-compiles on a GPU-less host, so the
artefact is produced here and travels with the repository snapshot to the
MI355X box.  No torch headers are involved (plain HIP + ctypes ABI), which
keeps the build to a few seconds.
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
SRCS = [os.path.join(CSRC, "dmcp_kernels.hip"), os.path.join(CSRC, "fused_gemm.hip"),
        os.path.join(CSRC, "prefill_attn.hip"), os.path.join(CSRC, "wgemm.hip"), os.path.join(CSRC, "pgemm.hip"),
        os.path.join(CSRC, "tgemm.hip")]
HEADERS = [os.path.join(CSRC, "dmcp_common.hpp")]
SRC = SRCS[0]  # kept for callers that name the main source
TARGET = os.path.join(HERE, "_hipops.so")
STAMP = TARGET + ".stamp"
ARCH = os.environ.get("DMCP_HIP_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-Wall", "-Wno-unused-function",
         "-munsafe-fp-atomics"]
# MFMA accumulators in VGPRs: the prefix-attention softmax works on the score
# tile in place (AGPR form cost ~90 v_accvgpr moves per 32-key tile).  Not for
# pgemm.hip / tgemm.hip: their 256 accumulator registers per lane must live in
# the AGPR half.
VGPR_FORM = ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]
# The flash-attention source without SLP vectorisation: packed f32 VALU
# (v_pk_add / v_pk_mul) issued beside MFMAs costs more than the scalar pair
# it replaces (cdna_hip_programming.md, MI355X_MICROARCH.md 'Per-instruction
# cycle constants'); the compiler had packed the softmax row sums and the O
# rescale.  Prefill attention 128 VGPRs / 4 waves per SIMD (130 / 3 packed),
# prefill GPU time -1 to -2 %, engine +0.3-1 % (profiles/attn_noslp_ab_r6.txt).
# Elsewhere the packed math stays: the GEMMs' epilogues lose 0.3-4 % per
# decode step without it, the per-row decode attention measured even
# (profiles/gemm_noslp_step_ab_r6.txt).
NO_SLP = ["-fno-slp-vectorize"]
PER_FILE = {"pgemm.hip": [], "tgemm.hip": [], "prefill_attn.hip": VGPR_FORM + NO_SLP}


def _flags(src: str) -> list:
    return FLAGS + PER_FILE.get(os.path.basename(src), VGPR_FORM)


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm is required to build dmcp HIP kernels)")


def _key() -> str:
    h = hashlib.sha256(" ".join(FLAGS + VGPR_FORM + sorted(f"{k}={v}" for k, v in PER_FILE.items())).encode())
    for path in SRCS + HEADERS:
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def build(force: bool = False, jobs: int = 0) -> str:
    """One object per source (own flags), compiled in parallel, then linked."""
    key = _key()
    if not force and os.path.exists(TARGET) and os.path.exists(STAMP) and open(STAMP).read().strip() == key:
        return TARGET
    import concurrent.futures
    import tempfile
    with tempfile.TemporaryDirectory(prefix="dmcp_hip_") as tmpdir:
        def compile_one(src):
            obj = os.path.join(tmpdir, os.path.basename(src) + ".o")
            r = subprocess.run([hipcc(), *_flags(src), f"-I{CSRC}", "-c", "-o", obj, src],
                               stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"hipcc failed on {os.path.basename(src)} ({r.returncode}):\n{r.stdout}")
            return obj
        n = jobs or min(len(SRCS), os.cpu_count() or 1, 8)
        with concurrent.futures.ThreadPoolExecutor(max_workers=n) as ex:
            objs = list(ex.map(compile_one, SRCS))
        tmp = TARGET + ".tmp"
        r = subprocess.run([hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs],
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc link failed ({r.returncode}):\n{r.stdout}")
    os.replace(tmp, TARGET)
    with open(STAMP, "w") as f:
        f.write(key)
    return TARGET


if __name__ == "__main__":
    print(build(force=True))
