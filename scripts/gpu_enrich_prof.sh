#!/usr/bin/env bash
# bench_enrich (fp8 KV, 1,024 classes) with prefill device time, then the same
# run under rocprofv3 kernel stats (summaries only kept).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/ep
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 bench_enrich.py --kv-dtype fp8 > "$OUT/enrich.log" 2>&1 || { tail -20 "$OUT/enrich.log"; exit 1; }
tail -1 "$OUT/enrich.log"
( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o e \
    -- python3 "$ROOT/bench_enrich.py" --kv-dtype fp8 > "$ROOT/$OUT/prof.log" 2>&1 ) || { tail -5 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -type f ! -name '*kernel_stats*' -delete
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -int(r["TotalDurationNs"]))
tot = sum(int(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e9:.3f} s")
for r in rows[:30]:
    print(f'{int(r["Calls"]):8d} {int(r["TotalDurationNs"])/1e6:9.1f} ms {float(r["AverageNs"])/1e3:8.1f} us {r["Name"][:110]}')
PY
