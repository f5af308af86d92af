#!/usr/bin/env bash
# Weight-streaming GEMM: its GPU tests, then the whole GPU suite, the decode
# step at 78 / 320 rows and the engine bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/wg
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgemm.py -x -q --timeout 120 --timeout-method thread > "$OUT/wgemm_tests.log" 2>&1 \
  && tail -2 "$OUT/wgemm_tests.log" \
  && timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gputest.log" 2>&1 \
  && tail -2 "$OUT/gputest.log" \
  && timeout -k 10 200 python3 scripts/bench_step.py --batch 256 --extra 64 --kv-dtype fp8 --iters 100 > "$OUT/step320.log" 2>&1 \
  && grep bench "$OUT/step320.log" \
  && timeout -k 10 200 python3 scripts/bench_step.py --batch 64 --extra 14 --kv-dtype fp8 --iters 100 > "$OUT/step78.log" 2>&1 \
  && grep bench "$OUT/step78.log" \
  && timeout -k 10 300 python3 bench_enrich.py --kv-dtype fp8 > "$OUT/enrich.log" 2>&1 \
  && tail -1 "$OUT/enrich.log"
