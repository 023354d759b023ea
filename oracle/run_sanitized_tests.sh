#!/bin/sh
# CPU test suite against the ASan/UBSan build of the oracle (test
# infrastructure).  Python itself is not instrumented, so the
# sanitizer runtime is preloaded ahead of anything already preloaded, and leak
# checking is off (the interpreter's own allocations are not ours).
set -eu
HERE=$(cd "$(dirname "$0")" && pwd)
make -s -C "$HERE" sanitize
ASAN_RT=$(gcc -print-file-name=libasan.so)
UBSAN_RT=$(gcc -print-file-name=libubsan.so)
export ELP_ORACLE_SO="$HERE/_build/libelp_oracle_san.so"
export ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"
cd "$HERE/.."
LD_PRELOAD="$ASAN_RT $UBSAN_RT${LD_PRELOAD:+ $LD_PRELOAD}" \
    python -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@"
