#!/usr/bin/env bash
# Decode step with equal vs varied own lengths and jump-row placement
# (fp8 KV, 448 sequences + 64 jump rows and 256 + 64).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/jit
mkdir -p "$OUT"
for a in "448 64" "256 64"; do
    set -- $a
    for opt in "--jitter 0" "--jitter 0.25" "--jitter 0 --adjacent" "--jitter 0.25 --adjacent"; do
        timeout -k 10 200 python3 scripts/bench_step.py --batch $1 --extra $2 --kv-dtype fp8 --iters 60 $opt > "$OUT/s.log" 2>&1 \
            || { tail -20 "$OUT/s.log"; exit 1; }
        echo "$opt $(grep -o '"rows": [0-9]*' $OUT/s.log) $(grep -o '"device_ms": [0-9.]*' $OUT/s.log) $(grep -o '"kv_MB": [0-9.]*' $OUT/s.log)"
    done
done
bash scripts/gpu_wgemm_vs_blas.sh
