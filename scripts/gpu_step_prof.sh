#!/usr/bin/env bash
# Decode step device time + rocprofv3 kernel-stats breakdown at one operating
# point: scripts/gpu_step_prof.sh <sequences> <jump rows> (fp8 KV).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
B=${1:-448}; X=${2:-64}
OUT=gpurun_out/sp$B
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/bench_step.py --batch $B --extra $X --kv-dtype fp8 --iters 100 ${STEP_ARGS:-} > "$OUT/step.log" 2>&1 \
    || { tail -20 "$OUT/step.log"; exit 1; }
grep '^{' "$OUT/step.log"
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o step \
    -- python3 "$ROOT/scripts/bench_step.py" --batch $B --extra $X --kv-dtype fp8 --iters 50 ${STEP_ARGS:-} > "$ROOT/$OUT/prof.log" 2>&1 ) \
    || { tail -5 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -type f ! -name '*kernel_stats*' -delete
python3 scripts/kstats.py $(find "$OUT/prof" -name '*kernel_stats.csv' | head -1) | tee "$OUT/kstats.txt"
