#!/bin/bash
# Build an A/B variant of libpcp.so with extra compile flags (profiling aid):
#   tools/build_variant.sh NAME [-DFOO=1 ...]  ->  variants/NAME/libpcp.so (load with PCP_LIB=...)
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/variants/$name
mkdir -p "$out/obj"
cd "${SRC:-$root/pointcloudprocess_amd/csrc}"  # SRC: another checkout, e.g. a git worktree of HEAD
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-result -Wno-unused-value -munsafe-fp-atomics"
objs=()
for f in *.hip *.cpp; do
  /opt/rocm/bin/hipcc $FLAGS -DPCP_SRC_SHA='"variant"' "$@" -x hip -c "$f" -o "$out/obj/$f.o" &
  objs+=("$out/obj/$f.o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/libpcp.so" "${objs[@]}"
rm -rf "$out/obj"
echo "$out/libpcp.so"
