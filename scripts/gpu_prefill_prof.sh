#!/usr/bin/env bash
# Batched prefill: time per class at 1 / 4 / 12 sequences, then a rocprofv3
# kernel-stats run of the 12-sequence batch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/pf
mkdir -p "$OUT"
export TMPDIR=/tmp
for n in 1 4 12; do
  timeout -k 10 200 python3 scripts/bench_prefill.py --seqs $n > "$OUT/s$n.log" 2>&1 || { tail -5 "$OUT/s$n.log"; exit 1; }
  tail -1 "$OUT/s$n.log"
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o pf \
    -- python3 "$ROOT/scripts/bench_prefill.py" --seqs 12 --iters 5 > "$ROOT/$OUT/prof.log" 2>&1 ) || exit 1
find "$OUT/prof" -type f ! -name '*kernel_stats*' -delete
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -int(r["TotalDurationNs"]))
tot = sum(int(r["TotalDurationNs"]) for r in rows)
for r in rows[:14]:
    print(f'{int(r["TotalDurationNs"])/1e6:8.2f} ms {100*int(r["TotalDurationNs"])/tot:5.1f}% {r["Calls"]:>6} {r["Name"][:110]}')
PY
