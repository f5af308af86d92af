#!/usr/bin/env bash
# Engine admission threshold A/B (bench_enrich, fp8 KV, batch 256).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/admit
mkdir -p "$OUT"
for am in ${ADMITS:-1 16 48}; do
  timeout -k 10 300 python3 bench_enrich.py --kv-dtype fp8 --admit-min $am > "$OUT/a$am.log" 2>&1 || { tail -5 "$OUT/a$am.log"; exit 1; }
  echo "admit $am: $(tail -1 "$OUT/a$am.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decode_step_ms"], d["prefill_s"], d["prefill_batches"], d["decode_s"], d["elapsed_s"])')"
done
