#!/usr/bin/env bash
# Fused-GEMM decode step on the GPU box: GPU numerics tests, bench_step.py
# with hipBLASLt (--fused 0) vs fused gfx950 GEMMs (--fused 1), and a
# rocprofv3 kernel-stats run of the fused step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/fused
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_model.py tests/test_gpu_kernels.py -x -q \
    --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -15 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
for f in 0 1; do
    timeout -k 10 300 python scripts/bench_step.py --fused $f > "$OUT/step_f$f.log" 2>&1 || { tail -20 "$OUT/step_f$f.log"; exit 1; }
    grep bench "$OUT/step_f$f.log"
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o step \
    -- python3 "$ROOT/scripts/bench_step.py" --iters 50 --fused 1 > "$ROOT/$OUT/prof.log" 2>&1 ) || exit 1
find "$OUT/prof" -type f ! -name '*kernel_stats*' -delete
python3 scripts/kstats.py "$OUT/prof/step_kernel_stats.csv" || true
