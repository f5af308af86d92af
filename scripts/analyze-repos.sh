#!/usr/bin/env bash
# Bulk-analyze repositories through a running dmcp REST server.
#
#   scripts/analyze-repos.sh [repos.txt] [base-url]
#
# repos.txt: one "url [branch]" per line; blank lines and '#' comments are
# skipped.  Repositories are POSTed to /api/projects/analyze one at a time
# with fixMissed=true; the exit code is the number of failures (parity with
# the reference's scripts/analyze-repos.sh).  For in-process (optionally
# multi-process) indexing without a server use:
#   python -m dmcp analyze-batch repos.txt --workers 4
set -u
FILE="${1:-repos.txt}"
BASE="${2:-${DMCP_URL:-http://localhost:8080}}"
if [ ! -f "$FILE" ]; then
    echo "repository list not found: $FILE" >&2
    exit 1
fi
failed=0
total=0
while read -r url branch _; do
    case "$url" in ''|'#'*) continue ;; esac
    total=$((total + 1))
    if [ -n "${branch:-}" ]; then
        body=$(printf '{"repositoryUrl":"%s","branch":"%s","fixMissed":true}' "$url" "$branch")
    else
        body=$(printf '{"repositoryUrl":"%s","fixMissed":true}' "$url")
    fi
    echo "[$total] analyzing $url ${branch:-}"
    if resp=$(curl -sS -f -X POST -H 'Content-Type: application/json' -d "$body" "$BASE/api/projects/analyze"); then
        echo "    $resp"
    else
        echo "    FAILED: $resp" >&2
        failed=$((failed + 1))
    fi
done < "$FILE"
echo "done: $total repositories, $failed failed"
exit "$failed"
