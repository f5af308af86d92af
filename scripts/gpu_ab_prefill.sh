#!/usr/bin/env bash
# Prefill attention change: prefill + kernel GPU tests, then batched prefill and decode step (prefix kernel)
# with the working tree vs dmcp/ops/ab/_hipops_$AB.so, alternated twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abp
mkdir -p "$OUT"
AB=${AB:-HEAD}
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_prefill.py \
    tests/test_gpu_kernels.py tests/test_gpu_fp8kv.py tests/test_gpu_model.py > "$OUT/tests.log" 2>&1 \
    || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for rep in 1 2; do
    for v in new old; do
        if [ $v = old ]; then export DMCP_HIPOPS_SO=dmcp/ops/ab/_hipops_$AB.so; else unset DMCP_HIPOPS_SO; fi
        timeout -k 10 200 python3 scripts/bench_prefill.py --seqs 12 > "$OUT/p.log" 2>&1 || { tail -20 "$OUT/p.log"; exit 1; }
        timeout -k 10 200 python3 scripts/bench_step.py --batch 256 --extra 64 --kv-dtype fp8 --iters 60 > "$OUT/s.log" 2>&1 \
            || { tail -20 "$OUT/s.log"; exit 1; }
        echo "$v prefill $(grep -o '"ms_per_class": [0-9.]*' $OUT/p.log) step320 $(grep -o '"device_ms": [0-9.]*' $OUT/s.log)"
    done
done
