#!/bin/bash
# Host-side ASan/UBSan run (SURVEY.md section 5 "Race detection / sanitizers"): the CPU tests that
# drive libsvgpu's C ABI (argument checks, error paths, host fold, host gather pool) and the C++
# restatement, loaded from their sanitizer builds (make -C snark-verifier-axiom_amd sanitize).
# CPU only: no GPU ASan (not available on this pool) -- compute entry points report SV_ERR_DEVICE here.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
RT="$(/opt/rocm/llvm/bin/clang++ -print-file-name=libclang_rt.asan-x86_64.so)"
[ -f "$RT" ] || RT="$(ls /opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)"
export SVGPU_LIB="$ROOT/snark-verifier-axiom_amd/build/asan/libsvgpu.so"
export ORACLE_LIB="$ROOT/oracle/build/asan/liboracle_bn254.so"
export ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"
cd "$ROOT"
LD_PRELOAD="$RT" python3 -m pytest -x -q -p no:cacheprovider tests/test_abi.py tests/test_oracle_cpp.py tests/test_host_mirror.py "$@"
