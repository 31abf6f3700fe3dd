#!/bin/bash
# Build tools/sort_bench (measurement tool) against this tree's fm_sort.hip and the library's other
# objects.  Extra -D flags for the sort go in $@.  Output: ${OUT:-tools/sort_bench}.
set -eu
cd "$(dirname "$0")/.."
out=${OUT:-tools/sort_bench}
tmp=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -c fm_spark_amd/csrc/fm_sort.hip -o "$tmp/fm_sort.o"
objs=$(ls fm_spark_amd/lib/obj/*.o | grep -v fm_sort.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I. -c tools/sort_bench.hip -o "$tmp/sort_bench.o"
mkdir -p "$(dirname "$out")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 "$tmp/sort_bench.o" "$tmp/fm_sort.o" $objs \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -o "$out"
rm -rf "$tmp"
echo "built $out $*"
