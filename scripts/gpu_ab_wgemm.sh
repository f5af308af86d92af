#!/usr/bin/env bash
# Weight-streaming GEMM alone (scripts/bench_wgemm.py at 78 / 320 / 512 rows):
# working tree vs dmcp/ops/ab/_hipops_$AB.so
# (scripts/hipops_ab.sh), alternated twice; one line per variant: gemm M us TFLOP/s.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
AB=${AB:-HEAD}
for rep in 1 2; do
  for v in new old; do
    unset DMCP_HIPOPS_SO
    [ $v = old ] && export DMCP_HIPOPS_SO=dmcp/ops/ab/_hipops_$AB.so
    timeout -k 10 120 python scripts/bench_wgemm.py 78 320 512 > gpurun_out/wg_$v.jsonl 2>gpurun_out/wg_$v.err \
        || { tail -5 gpurun_out/wg_$v.err; exit 1; }
    python3 -c "
import json
print('$v', ' '.join(f\"{d['gemm']}/{d['M']}:{d['us']}\" for d in map(json.loads, open('gpurun_out/wg_$v.jsonl'))))"
  done
done
