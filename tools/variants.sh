#!/bin/bash
# Build experiment variants of libfm_hip.so (extra -D flags) into fm_spark_amd/lib/variants/.
#   tools/variants.sh name "FLAG=1 FLAG2=2" [name2 "flags2" ...]
set -eu
cd "$(dirname "$0")/.."
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  args=()
  for f in $flags; do args+=(-D "$f"); done
  python -m fm_spark_amd.build --out "fm_spark_amd/lib/variants/$name/libfm_hip.so" "${args[@]}" > /dev/null
  echo "built fm_spark_amd/lib/variants/$name/libfm_hip.so ($flags)"
done
