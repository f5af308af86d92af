#!/usr/bin/env bash
# One GPU session on the MI355X box: tests, smoke, benches, rocprofv3 profile.
# Every GPU step has its own time limit; a crash / abort / timeout ends the
# script (ordinary test failures do not).  Output goes to gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS="${STEPS:-pytest smoke bench enrich prof}"

run() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 5 "$OUT/$name.log"
    case $rc in
        0|1|5) return 0 ;;                 # ok / test failures / no tests collected
        *) echo "fatal rc=$rc in $name: stopping"; exit $rc ;;
    esac
}

for s in $STEPS; do
    case $s in
        pytest) run pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:randomly ;;
        smoke) run smoke 600 python __graft_entry__.py smoke ;;
        bench) run bench 600 python bench.py --steps 5 --warmup 2 ;;
        enrich) run bench_enrich 900 python bench_enrich.py --classes 256 --batch 64 ;;
        enrich_nojump) run bench_enrich_nojump 900 python bench_enrich.py --classes 256 --batch 64 --no-jump ;;
        enrich_noprefix) run bench_enrich_noprefix 900 python bench_enrich.py --classes 256 --batch 64 --no-shared-prefix ;;
        kernels) run kernels 600 python scripts/bench_kernels.py ;;
        prof)
            ROOT=$(pwd)
            ( cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv \
                -d "$ROOT/$OUT/prof" -o enrich \
                -- python3 "$ROOT/bench_enrich.py" --classes 64 --batch 64 > "$ROOT/$OUT/prof.log" 2>&1 )
            rc=$?
            echo "=== prof rc=$rc"; tail -n 5 "$OUT/prof.log"
            # keep only the summaries (the raw trace can exceed the 64 MiB copy-back limit)
            find "$OUT/prof" -type f ! -name '*stats*' -delete 2>/dev/null
            find "$OUT/prof" -name '*kernel_stats.csv' -exec head -n 40 {} \; 2>/dev/null
            [ $rc -eq 0 ] || exit $rc ;;
    esac
done
echo "=== done"
