#!/usr/bin/env bash
# rocprofv3 kernel stats of bench_enrich.py (shared prefix on, and off with
# TAGS="prefix noprefix").  Keeps only the *_stats.csv summaries under
# gpurun_out/prof_<tag>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
export TMPDIR=/tmp
for tag in ${TAGS:-prefix}; do
    extra=""
    [ "$tag" = noprefix ] && extra="--no-shared-prefix"
    ( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$ROOT/gpurun_out/prof_$tag" -o enrich \
        -- python3 "$ROOT/bench_enrich.py" --classes 64 --batch 64 $extra > "$ROOT/gpurun_out/prof_$tag.log" 2>&1 )
    rc=$?
    find "$ROOT/gpurun_out/prof_$tag" -type f ! -name '*stats*' -delete 2>/dev/null
    echo "=== prof_$tag rc=$rc"
    grep metric "$ROOT/gpurun_out/prof_$tag.log" | cut -c1-200
    [ $rc -eq 0 ] || exit $rc
done
