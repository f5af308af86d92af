#!/usr/bin/env bash
# Decode-step A/B: working-tree kernels vs dmcp/ops/ab/_hipops_$AB.so (built by
# scripts/hipops_ab.sh), alternated twice at 320 and 78 rows (fp8 KV).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab
mkdir -p "$OUT"
AB=${AB:-HEAD}
for rep in 1 2; do
    for v in new old; do
        for a in "256 64" "64 14" "448 64"; do
            set -- $a
            if [ $v = old ]; then export DMCP_HIPOPS_SO=dmcp/ops/ab/_hipops_$AB.so; else unset DMCP_HIPOPS_SO; fi
            timeout -k 10 200 python3 scripts/bench_step.py --batch $1 --extra $2 --kv-dtype fp8 --iters 100 \
                > "$OUT/$v$1.log" 2>&1 || { tail -20 "$OUT/$v$1.log"; exit 1; }
            echo "$v $(grep -o '"rows": [0-9]*' "$OUT/$v$1.log") $(grep -o '"device_ms": [0-9.]*' "$OUT/$v$1.log")"
        done
    done
done
