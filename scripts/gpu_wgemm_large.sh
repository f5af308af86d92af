#!/usr/bin/env bash
# Weight-streaming GEMM tests, then decode step with wgemm vs hipBLASLt at
# 448-1024 rows (fp8 KV), then bench_enrich fp8 (512 slots, 768 rows).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/wl
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wgemm.py \
    tests/test_gpu_model.py > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for a in "448 64" "512 128" "640 128" "768 256"; do
    set -- $a
    for w in 1 0; do
        timeout -k 10 200 python3 scripts/bench_step.py --batch $1 --extra $2 --kv-dtype fp8 --iters 60 --wgemm $w --adjacent \
            > "$OUT/s.log" 2>&1 || { tail -20 "$OUT/s.log"; exit 1; }
        echo "wgemm=$w $(grep -o '"rows": [0-9]*' $OUT/s.log) $(grep -o '"device_ms": [0-9.]*' $OUT/s.log)"
    done
done
timeout -k 10 400 python3 bench_enrich.py --kv-dtype fp8 > "$OUT/e.log" 2>&1 || { tail -20 "$OUT/e.log"; exit 1; }
grep '^{' "$OUT/e.log"
