#!/usr/bin/env bash
# The native core under AddressSanitizer + UBSan (host code only; CPU):
# builds build/asan/_srcscan<ext>, then runs the parser, source, pipeline,
# sync and fuzz tests with that module loaded into an ASan-preloaded Python.
# Any memory error or undefined behaviour aborts the run (non-zero exit).
set -euo pipefail
cd "$(dirname "$0")/.."
SO=$(python -c "from dmcp import buildtools; print(buildtools.build_srcscan_asan())")
LIBASAN=$(gcc -print-file-name=libasan.so)
export DMCP_SRCSCAN_SO="$SO"
export ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1:detect_stack_use_after_return=0"
export UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1"
export DMCP_FUZZ_ITERS="${DMCP_FUZZ_ITERS:-6000}"
LD_PRELOAD="$LIBASAN" python -m pytest -q -p no:cacheprovider -m "not gpu" \
    tests/test_fuzz.py tests/test_parser_java.py tests/test_parser_ts.py tests/test_parser_go.py \
    tests/test_ref_java_parser.py tests/test_ref_ts_parser.py tests/test_ref_ts_engine.py tests/test_ref_go.py \
    tests/test_source.py tests/test_pipeline.py tests/test_sync.py "$@"
