#!/usr/bin/env bash
# Batched prefill (12 classes) with a bf16 vs fp8 KV cache: ms per class and
# rocprofv3 kernel stats of each (varlen attention vs GEMMs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/pkv
mkdir -p "$OUT"
export TMPDIR=/tmp
for kv in bf16 fp8; do
    ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/$kv" -o p \
        -- python3 "$ROOT/scripts/bench_prefill.py" --seqs 12 --kv-dtype $kv > "$ROOT/$OUT/$kv.log" 2>&1 ) || { tail -5 "$OUT/$kv.log"; exit 1; }
    find "$OUT/$kv" -type f ! -name '*kernel_stats*' -delete
    grep '^{' "$OUT/$kv.log"
    python3 - "$OUT/$kv" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -int(r["TotalDurationNs"]))
for r in rows[:6]:
    print(f'{int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:9.1f} us {r["Name"][:100]}')
PY
done
