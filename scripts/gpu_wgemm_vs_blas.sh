#!/usr/bin/env bash
# Decode step with the weight-streaming GEMMs vs hipBLASLt (F.linear) for the
# projections, at several row counts (fp8 KV), alternated twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/wvb
mkdir -p "$OUT"
for rep in 1 2; do
    for a in "256 64" "384 64" "448 64" "512 128" "640 128"; do
        set -- $a
        for w in 1 0; do
            timeout -k 10 200 python3 scripts/bench_step.py --batch $1 --extra $2 --kv-dtype fp8 --iters 60 --wgemm $w \
                > "$OUT/s.log" 2>&1 || { tail -20 "$OUT/s.log"; exit 1; }
            echo "wgemm=$w $(grep -o '"rows": [0-9]*' $OUT/s.log) $(grep -o '"device_ms": [0-9.]*' $OUT/s.log)"
        done
    done
done
