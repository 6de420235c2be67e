#!/bin/bash
# Sanitizer builds of libstormck's HOST code (tests/sanitize/host_paths.cpp drives it).
#   bash tests/sanitize/build.sh asan   -> tests/sanitize/build/host_paths_asan  (ASan + UBSan)
#   bash tests/sanitize/build.sh tsan   -> tests/sanitize/build/host_paths_tsan  (TSan)
# Each -fsanitize= sits right after -Xarch_host, so only the host pass is instrumented
# (no GPU sanitizer: device code is built exactly as in the product library). The
# library is compiled into the driver executable (one image, the sanitizer runtime
# linked statically by clang), with the oracle's C restatement as the checker.
set -euo pipefail
kind=${1:-asan}
R=$(cd "$(dirname "$0")/../.." && pwd)
out=$R/tests/sanitize/build
mkdir -p "$out"
case $kind in
  asan) host=(-fsanitize=address -fsanitize=undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer) ;;
  tsan) host=(-fsanitize=thread) ;;
  *) echo "usage: $0 asan|tsan" >&2; exit 2 ;;
esac
san=()
for f in "${host[@]}"; do san+=(-Xarch_host "$f"); done
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
CLANG=${CLANG:-/opt/rocm/llvm/bin/clang}
# the library (device code for gfx950 untouched, host pass instrumented)
"$HIPCC" --offload-arch=gfx950 -O1 -gline-tables-only -std=c++17 -fPIC "${san[@]}" -c -o "$out/stormck_$kind.o" \
    "$R/storm_amd/csrc/stormck.hip"
# the driver and the oracle (host only)
"$CLANG" -x c++ -std=c++17 -O1 -gline-tables-only "${host[@]}" -D__HIP_PLATFORM_AMD__ -I /opt/rocm/include -I "$R/include" \
    -c -o "$out/host_paths_$kind.o" "$R/tests/sanitize/host_paths.cpp"
"$CLANG" -x c -O1 -gline-tables-only "${host[@]}" -c -o "$out/oracle_$kind.o" "$R/oracle/xxh64_oracle.c"
"$HIPCC" --hip-link --offload-arch=gfx950 "${san[@]}" -o "$out/host_paths_$kind" \
    "$out/stormck_$kind.o" "$out/host_paths_$kind.o" "$out/oracle_$kind.o" -lpthread
echo "$out/host_paths_$kind"
