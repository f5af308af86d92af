#!/usr/bin/env bash
# FP8 KV cache on the MI355X box: kernel numerics, decode-step A/B (bf16 vs
# fp8 cache), end-to-end enrichment with the fp8 cache.  Stops at the first
# crash, abort or timeout (test failures are reported, not fatal).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS="${STEPS:-tests step enrich}"
step() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 8 "$OUT/$name.log"
    case $rc in 0|1) return 0 ;; *) echo "fatal rc=$rc in $name"; exit $rc ;; esac
}
for s in $STEPS; do
    case $s in
        tests) step fp8_tests 400 python -u -m pytest tests/test_gpu_fp8kv.py tests/test_gpu_prefill.py \
                   tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_fused.py -x -q --timeout 120 \
                   --timeout-method thread ;;
        step) step step_bf16 300 python scripts/bench_step.py
              step step_fp8 300 python scripts/bench_step.py --kv-dtype fp8
              DMCP_PREFIX_IMPL=v1 step step_bf16_prefix_v1 300 python scripts/bench_step.py
              DMCP_PREFIX_IMPL=v1 step step_fp8_prefix_v1 300 python scripts/bench_step.py --kv-dtype fp8 ;;
        overlap) DMCP_PREFIX_OVERLAP=0 step step_fp8_no_overlap 300 python scripts/bench_step.py --kv-dtype fp8
                 DMCP_PREFIX_OVERLAP=0 DMCP_PREFIX_IMPL=v1 step step_fp8_v1_no_overlap 300 python scripts/bench_step.py --kv-dtype fp8 ;;
        splits) for n in 4 8 12 16; do
                    DMCP_PREFIX_SPLITS=$n step step_fp8_psplit$n 300 python scripts/bench_step.py --kv-dtype fp8
                done ;;
        enrich) step enrich_fp8 600 python bench_enrich.py --classes 256 --batch 64 --kv-dtype fp8
                step enrich_bf16 600 python bench_enrich.py --classes 256 --batch 64 ;;
    esac
done
echo "=== done"
