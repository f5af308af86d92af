#!/usr/bin/env bash
# Shared-prefix attention A/B at the enrichment operating point: the 256-key
# chunk kernel vs the MFMA prefill kernel in prefix mode at several split counts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pfx
mkdir -p "$OUT"
for rows in "256 64" "64 14"; do
  set -- $rows
  ARGS="--batch $1 --extra $2 --kv-dtype fp8 --iters 100"
  DMCP_PREFIX_IMPL=chunk timeout -k 10 200 python3 scripts/bench_step.py $ARGS > "$OUT/chunk_$1.log" 2>&1 || exit 1
  echo "chunk b$1 $(grep -o '"device_ms": [0-9.]*' "$OUT/chunk_$1.log")"
  for sp in 2 3 4 6 8 12; do
    DMCP_PREFIX_IMPL=prefill DMCP_PREFIX_SPLITS=$sp timeout -k 10 200 python3 scripts/bench_step.py $ARGS \
        > "$OUT/prefill_$1_$sp.log" 2>&1 || exit 1
    echo "prefill b$1 s$sp $(grep -o '"device_ms": [0-9.]*' "$OUT/prefill_$1_$sp.log")"
  done
done
