#!/usr/bin/env bash
# Swizzled V tile of the per-row decode attention: kernel tests, step time at
# 320 / 78 rows, LDS conflict counters at 320 rows.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/swz
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_fp8kv.py \
    > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
for a in "256 64" "64 14"; do
    set -- $a
    timeout -k 10 200 python3 scripts/bench_step.py --batch $1 --extra $2 --kv-dtype fp8 --iters 100 > "$OUT/step$1.log" 2>&1 \
        || { tail -20 "$OUT/step$1.log"; exit 1; }
    grep bench "$OUT/step$1.log"
done
PMC_SETS="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA" bash scripts/pmc_decode_step.sh --batch 256 --extra 64 --kv-dtype fp8 \
    > "$OUT/pmc.txt" 2>&1 || { tail -5 "$OUT/pmc.txt"; exit 1; }
cat "$OUT/pmc.txt"
