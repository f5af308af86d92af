#!/usr/bin/env bash
# bench_enrich.py fp8 at three admission thresholds (KV slots that must be free
# before a running batch admits a new batched prefill), alternated twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/admit
mkdir -p "$OUT"
for rep in 1 2; do
    for a in 16 32 64; do
        timeout -k 10 300 python3 bench_enrich.py --kv-dtype fp8 --admit-min $a > "$OUT/a$a-$rep.log" 2>&1 \
            || { tail -20 "$OUT/a$a-$rep.log"; exit 1; }
        echo "admit_min=$a $(grep -o '"value": [0-9.]*' "$OUT/a$a-$rep.log") $(grep -o '"prefill_gpu_s": [0-9.]*' "$OUT/a$a-$rep.log") $(grep -o '"decode_steps": [0-9]*' "$OUT/a$a-$rep.log")"
    done
done
