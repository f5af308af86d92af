#!/usr/bin/env bash
# Decode-step A/B on the GPU box: kernel tests, bench_step per decode impl,
# then a rocprofv3 kernel-stats run of the default configuration.
set -u
STEP_ARGS=${STEP_ARGS:-}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/step
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
    timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 120 \
        --timeout-method thread > "$OUT/tests.log" 2>&1
    rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python scripts/bench_step.py $STEP_ARGS > "$OUT/step.log" 2>&1 || { tail -20 "$OUT/step.log"; exit 1; }
grep bench "$OUT/step.log"
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o step \
    -- python3 "$ROOT/scripts/bench_step.py" --iters 50 $STEP_ARGS > "$ROOT/$OUT/prof.log" 2>&1 ) || exit 1
find "$OUT/prof" -type f ! -name '*kernel_stats*' -delete
python3 scripts/kstats.py "$OUT/prof/step_kernel_stats.csv" 2>/dev/null | head -30 || true
