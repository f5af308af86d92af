#!/usr/bin/env bash
# Prefill-attention kernel on the MI355X box: numerics tests, kernel A/B,
# per-class prefill with and without the kernel, end-to-end enrichment, and a
# kernel-trace profile of the per-class prefill.  Stops at the first crash,
# abort or timeout (test failures are reported, not fatal).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS="${STEPS:-tests attn class enrich prof}"
step() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 14 "$OUT/$name.log"
    case $rc in 0|1) return 0 ;; *) echo "fatal rc=$rc in $name"; exit $rc ;; esac
}
for s in $STEPS; do
    case $s in
        tests) step pf_tests 300 python -u -m pytest tests/test_gpu_prefill.py tests/test_gpu_model.py \
                   tests/test_local_engine.py -x -q --timeout 120 --timeout-method thread ;;
        attn) step pf_attn 300 python scripts/bench_prefill_attn.py ;;
        class) step pf_class_kernel 300 python scripts/bench_prefill.py
               DMCP_PREFILL_KERNEL=0 step pf_class_sdpa 300 python scripts/bench_prefill.py ;;
        enrich) step pf_enrich 600 python bench_enrich.py --classes 256 --batch 64 ;;
        prof)
            ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
                -d "$ROOT/$OUT/pfprof" -o pf -- python3 "$ROOT/scripts/bench_prefill.py" > "$ROOT/$OUT/pfprof.log" 2>&1 )
            rc=$?
            echo "=== pfprof rc=$rc"
            find "$OUT/pfprof" -type f ! -name '*stats*' -delete 2>/dev/null
            f=$(find "$OUT/pfprof" -name '*kernel_stats.csv' | head -n 1)
            [ -n "$f" ] && cut -d, -f1-5 "$f" | head -n 16
            [ $rc -eq 0 ] || exit $rc ;;
    esac
done
echo "=== done"
