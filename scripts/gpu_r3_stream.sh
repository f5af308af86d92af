#!/usr/bin/env bash
# GPU tests, smoke, the default bench (headline + extra.enrichLocal through the
# worker process) and the engine bench, each under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s_gputest.log 2>&1 \
  && tail -2 gpurun_out/s_gputest.log \
  && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s_smoke.log 2>&1 \
  && tail -1 gpurun_out/s_smoke.log \
  && timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s_bench.log 2> gpurun_out/s_bench.err \
  && tail -1 gpurun_out/s_bench.log \
  && timeout -k 10 600 python -u bench_enrich.py --kv-dtype fp8 > gpurun_out/s_enrich.log 2>&1 \
  && tail -1 gpurun_out/s_enrich.log
