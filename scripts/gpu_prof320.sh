#!/usr/bin/env bash
# Decode step at the enrichment operating point (256 sequences + 64 jump rows,
# fp8 KV): bench_step device time, rocprofv3 kernel stats, PMC of the kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/p320
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--batch 256 --extra 64 --kv-dtype fp8 ${STEP_ARGS:-}"
timeout -k 10 300 python3 scripts/bench_step.py $ARGS > "$OUT/step.log" 2>&1 || { tail -20 "$OUT/step.log"; exit 1; }
grep bench "$OUT/step.log" || tail -3 "$OUT/step.log"
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o step \
    -- python3 "$ROOT/scripts/bench_step.py" --iters 50 $ARGS > "$ROOT/$OUT/prof.log" 2>&1 ) || exit 1
find "$OUT/prof" -type f ! -name '*kernel_stats*' -delete
python3 scripts/kstats.py $(find "$OUT/prof" -name '*kernel_stats.csv' | head -1) > "$OUT/kstats.txt" 2>&1 || true
cat "$OUT/kstats.txt" | head -40
if [ "${PMC:-1}" = 1 ]; then
    bash scripts/pmc_decode_step.sh $ARGS > "$OUT/pmc.txt" 2>&1 || { tail -5 "$OUT/pmc.txt"; exit 1; }
    tail -8 "$OUT/pmc.txt"
fi
