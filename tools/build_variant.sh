#!/usr/bin/env bash
# Build libicp_hip.so of the working tree with a sed edit applied to one source, for same-box
# A/B timing (load it with ICP_AMD_LIB=iterative-closest-point_amd/build_ab/NAME/libicp_hip.so):
#   tools/build_variant.sh NAME csrc/FILE 'sed-expression'
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=${1:?name}; FILE=${2:?file}; EXPR=${3:?sed expression}
TMP=$(mktemp -d)
cp -r "$ROOT/iterative-closest-point_amd" "$ROOT/include" "$TMP/"
rm -rf "$TMP/iterative-closest-point_amd/build" "$TMP/iterative-closest-point_amd/build_ab"
sed -i "$EXPR" "$TMP/iterative-closest-point_amd/$FILE"
if cmp -s "$ROOT/iterative-closest-point_amd/$FILE" "$TMP/iterative-closest-point_amd/$FILE"; then
    echo "sed changed nothing" >&2; exit 1
fi
make -s -j8 -C "$TMP/iterative-closest-point_amd" build/libicp_hip.so
mkdir -p "$ROOT/iterative-closest-point_amd/build_ab/$NAME"
cp "$TMP/iterative-closest-point_amd/build/libicp_hip.so" "$ROOT/iterative-closest-point_amd/build_ab/$NAME/"
rm -rf "$TMP"
echo "$ROOT/iterative-closest-point_amd/build_ab/$NAME/libicp_hip.so"
