#!/usr/bin/env bash
# Kernel-trace profile of decode attention at a few shapes (GPU box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pd
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in "64 512" "64 2300" "1 4096"; do
    set -- $cfg
    ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o "b$1_l$2" \
        -- python3 "$ROOT/scripts/prof_decode.py" --B "$1" --L "$2" > "$OUT/b$1_l$2.log" 2>&1 ) || exit $?
done
find "$OUT" -type f ! -name '*stats*' ! -name '*.log' -delete
for f in "$OUT"/*kernel_stats.csv; do echo "== $f"; cut -c1-200 "$f"; done
