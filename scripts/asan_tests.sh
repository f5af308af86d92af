#!/usr/bin/env bash
# The native host code under AddressSanitizer + UBSan (CPU):
#  * build/asan/_srcscan<ext> (lexers, front-ends, loose-object inflater, row
#    writer): the parser, source, pipeline, sync and fuzz tests;
#  * build/asan/_grammar<ext> (native/grammar/engine.cpp, the local engine's
#    grammar state machine / step builder): the grammar fuzz (native vs the
#    Python state machine, DMCP_GRAMMAR_FUZZ_ITERS iterations, the same
#    comparison test_local_engine.py makes on the real tiny model -- which
#    under ASan's allocator runs past any sane time limit) and the capped-
#    string engine test.
# Both modules load into one ASan-preloaded Python; any memory error or
# undefined behaviour aborts the run (non-zero exit).
set -euo pipefail
cd "$(dirname "$0")/.."
SO=$(python -c "from dmcp import buildtools; print(buildtools.build_srcscan_asan())")
GSO=$(python -c "from dmcp import buildtools; print(buildtools.build_grammar_asan())")
LIBASAN=$(gcc -print-file-name=libasan.so)
# libstdc++ preloaded too: python itself does not link it, and without it
# ASan's __cxa_throw interceptor finds no real symbol -- a C++ exception
# thrown by a module (the grammar engine's argument checks) aborts
LIBSTDCXX=$(gcc -print-file-name=libstdc++.so)
export DMCP_SRCSCAN_SO="$SO"
export DMCP_GRAMMAR_SO="$GSO"
export ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1:detect_stack_use_after_return=0"
export UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1"
export DMCP_FUZZ_ITERS="${DMCP_FUZZ_ITERS:-6000}"
export DMCP_GRAMMAR_FUZZ_ITERS="${DMCP_GRAMMAR_FUZZ_ITERS:-6000}"
LD_PRELOAD="$LIBASAN $LIBSTDCXX" python -m pytest -q -p no:cacheprovider -m "not gpu" --timeout 3600 \
    tests/test_grammar_fuzz.py tests/test_fuzz.py tests/test_parser_java.py tests/test_parser_ts.py \
    tests/test_parser_go.py tests/test_ref_java_parser.py tests/test_ref_ts_parser.py tests/test_ref_ts_engine.py \
    tests/test_ref_go.py tests/test_source.py tests/test_pipeline.py tests/test_sync.py tests/test_scan_child.py \
    "tests/test_local_engine.py::test_capped_string_closes_at_a_word_boundary" "$@"
