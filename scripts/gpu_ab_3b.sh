#!/usr/bin/env bash
# 3B preset (head_dim 128) decode step: working tree vs dmcp/ops/ab/_hipops_$AB.so, alternated, plus the
# per-row kernel's LDS conflict counters on the working tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab3
mkdir -p "$OUT"
AB=${AB:-HEAD}
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
    tests/test_gpu_fp8kv.py > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for rep in 1 2; do
    for v in new old; do
        if [ $v = old ]; then export DMCP_HIPOPS_SO=dmcp/ops/ab/_hipops_$AB.so; else unset DMCP_HIPOPS_SO; fi
        timeout -k 10 200 python3 scripts/bench_step.py --preset dmcp-coder-3b --batch 256 --extra 64 --kv-dtype fp8 \
            --iters 40 > "$OUT/$v.log" 2>&1 || { tail -20 "$OUT/$v.log"; exit 1; }
        echo "$v $(grep -o '"device_ms": [0-9.]*' "$OUT/$v.log")"
    done
done
unset DMCP_HIPOPS_SO
PMC_SETS="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" bash scripts/pmc_decode_step.sh --preset dmcp-coder-3b \
    --batch 256 --extra 64 --kv-dtype fp8 > "$OUT/pmc.txt" 2>&1 || { tail -5 "$OUT/pmc.txt"; exit 1; }
grep decode_mfma "$OUT/pmc.txt"
