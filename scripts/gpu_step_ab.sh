#!/usr/bin/env bash
# GPU box: every GPU test, then bench_step.py A/B runs (STEP_VARIANTS, ';'-
# separated argument lists) and a rocprofv3 kernel-stats run of the first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/ab
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > "$OUT/tests.log" 2>&1
    rc=$?; tail -4 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
fi
IFS=';' read -ra VARIANTS <<< "${STEP_VARIANTS:- ;--no-groups}"
i=0
for v in "${VARIANTS[@]}"; do
    timeout -k 10 300 python scripts/bench_step.py $v > "$OUT/step_$i.log" 2>&1 || { tail -20 "$OUT/step_$i.log"; exit 1; }
    grep bench "$OUT/step_$i.log"
    i=$((i + 1))
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o step \
    -- python3 "$ROOT/scripts/bench_step.py" --iters 50 ${VARIANTS[0]} > "$ROOT/$OUT/prof.log" 2>&1 ) || exit 1
find "$OUT/prof" -type f ! -name '*kernel_stats*' -delete
python3 scripts/kstats.py "$OUT/prof/step_kernel_stats.csv" || true
