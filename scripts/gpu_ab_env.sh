#!/usr/bin/env bash
# Decode-step A/B of an environment switch on the same .so: VAR=$1, values
# "$2" (space separated), alternated twice at 320 / 78 / 512 rows (fp8 KV).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abenv
mkdir -p "$OUT"
VAR=$1
VALS=$2
ROWS=${ROWS:-"256 64|64 14|448 64"}
for rep in 1 2; do
    for v in $VALS; do
        IFS='|' read -ra RS <<< "$ROWS"
        for a in "${RS[@]}"; do
            set -- $a
            env "$VAR=$v" timeout -k 10 200 python3 scripts/bench_step.py --batch $1 --extra $2 --kv-dtype fp8 --iters 100 ${ARGS:-} \
                > "$OUT/$v-$1${TAG:-}.log" 2>&1 || { tail -20 "$OUT/$v-$1${TAG:-}.log"; exit 1; }
            echo "$VAR=$v $(grep -o '"rows": [0-9]*' "$OUT/$v-$1${TAG:-}.log") $(grep -o '"device_ms": [0-9.]*' "$OUT/$v-$1${TAG:-}.log")"
        done
    done
done
