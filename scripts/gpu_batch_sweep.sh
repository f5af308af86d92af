#!/usr/bin/env bash
# Engine batch (KV slots) sweep: bench_enrich fp8, classes x batch x max_rows;
# weight-streaming GEMM tests first (rows up to 1024).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/bs
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wgemm.py \
    > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for cfg in ${CFGS:-"1024 256 384" "1024 512 768" "1024 640 960" "1024 768 1024" "2048 512 768" "2048 768 1024"}; do
    set -- $cfg
    timeout -k 10 400 python3 bench_enrich.py --kv-dtype fp8 --classes $1 --batch $2 --max-rows $3 > "$OUT/b.log" 2>&1 \
        || { tail -20 "$OUT/b.log"; exit 1; }
    python3 - "$OUT/b.log" "$cfg" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], {k: d[k] for k in ("value", "elapsed_s", "decode_step_ms", "rows_per_step", "decode_steps", "prefill_gpu_s", "decode_s")})
PY
done
