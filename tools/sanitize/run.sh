#!/bin/bash
# CPU sanitizer run: builds the host sources and the oracle with
# -fsanitize=address,undefined (tools/sanitize/Makefile), runs the BVH-builder driver, then the CPU tests
# of the OBJ/MTL loader, the Assimp cross-check, the PNG/texture decoder, the oracle and its golden
# vectors, the render.bmp pin and the post-processing oracle with both instrumented libraries loaded into
# the test process (LD_PRELOAD of the sanitizer runtimes; leak checking off for the Python interpreter's
# own allocations).  Exit status 0 = no sanitizer report and every test green.
#   tools/sanitize/run.sh [log]
set -euo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
REPO=$(cd "$HERE/../.." && pwd)
LOG=${1:-/dev/stdout}
make -s -C "$HERE" -j8
DATA=$(cd "$REPO" && python -c "import sys; sys.path.insert(0, 'raytracer-group27_amd'); import rt_amd; print(rt_amd.data_dir())")
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
{
  echo "== bvh_driver (host BVH builders, ASan+UBSan, leak check on)"
  ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
    "$HERE/build/bvh_driver" "$DATA" "$TMP"
  echo "== pytest with librt_amd_san.so + liboracle_san.so"
  ASAN_LIB=$(gcc -print-file-name=libasan.so)
  UBSAN_LIB=$(gcc -print-file-name=libubsan.so)
  cd "$REPO"
  LD_PRELOAD="$ASAN_LIB $UBSAN_LIB" \
  ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:verify_asan_link_order=0 \
  UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  RT_AMD_SANITIZER_LIB="$HERE/build/librt_amd_san.so" ORACLE_SANITIZER_LIB="$HERE/build/liboracle_san.so" \
  RT_SANITIZER_RUN=1 OMP_NUM_THREADS=4 \
    python -m pytest -q -p no:cacheprovider -m "not gpu" \
      tests/test_loader.py tests/test_assimp_crosscheck.py tests/test_texture.py tests/test_mip_chain.py \
      tests/test_oracle.py tests/test_render_bmp_pin.py tests/test_post.py tests/test_view_batch_layout.py
  echo "== sanitizer run: OK"
} 2>&1 | tee "$LOG"
