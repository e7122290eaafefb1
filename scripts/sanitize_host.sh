#!/bin/bash
# Sanitizer runs of the host C++ (the multi-threaded graph builder that replaces the
# reference's scipy / Python construction, utils.py:42-50, model.py:4162-4170).
#   1. tests/host_sanitize/driver.cpp + csrc/graph_host.cpp + csrc/capi.cpp built with g++
#      -fsanitize=address,undefined, and again with -fsanitize=thread; both run here (no GPU).
#   2. the whole library built by hipcc with the same host-side sanitizers (device code
#      unchanged), and the Python host tests run against it (IGR_LIB points at it).
# Writes the transcripts to the directory given as $1 (default profiles/).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-$ROOT/profiles}
B=$ROOT/inductive-recommendation_amd/build/sanitize
CSRC=$ROOT/inductive-recommendation_amd/csrc
mkdir -p "$B" "$OUT"
INC="-I$ROOT/include -I$CSRC -I/opt/rocm/include -D__HIP_PLATFORM_AMD__"
LOG=$OUT/${SAN_TAG:-r03}_sanitize_host.txt
: > "$LOG"
for san in address,undefined thread; do
  tag=${san//,/_}
  echo "== g++ -fsanitize=$san: driver + graph_host.cpp + capi.cpp" | tee -a "$LOG"
  g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=$san -fno-sanitize-recover=all $INC \
      "$ROOT/tests/host_sanitize/driver.cpp" "$CSRC/graph_host.cpp" "$CSRC/capi.cpp" \
      -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib -pthread -o "$B/driver_$tag"
  ( cd "$B" && ASAN_OPTIONS=detect_leaks=1 UBSAN_OPTIONS=print_stacktrace=1 TSAN_OPTIONS=halt_on_error=1 \
      "./driver_$tag" ) 2>&1 | tee -a "$LOG"
done
echo "== hipcc, host pass with -fsanitize=address,undefined: whole library + Python host tests" | tee -a "$LOG"
SRCS="spmm.hip spmm_rows.hip topk.hip edge_ops.hip att_shared.hip bpr.hip rowsort.hip gemm.hip linear_wgrad.hip train_ops.hip graph_host.cpp capi.cpp"
OBJS=""
for s in $SRCS; do
  o=$B/${s%.*}.o
  /opt/rocm/bin/hipcc -O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -I "$ROOT/include" -I "$CSRC" \
      -Xclang -target-feature -Xclang -packed-fp32-ops \
      -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer \
      -x hip -c "$CSRC/$s" -o "$o" 2> >(grep -v "packed-fp32-ops" >&2) &
  OBJS="$OBJS $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fsanitize=address -fsanitize=undefined -fno-gpu-sanitize \
    -shared-libsan -o "$B/libigr_asan.so" $OBJS -lpthread
RT=$(/opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
( cd "$ROOT" && IGR_LIB=$B/libigr_asan.so LD_PRELOAD="${LD_PRELOAD:+$LD_PRELOAD:}$RT" \
    ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
    python -m pytest tests/test_capi_host.py tests/test_host_logic.py -q -p no:cacheprovider ) 2>&1 | tail -5 | tee -a "$LOG"
echo "sanitize_host: done" | tee -a "$LOG"
