#!/usr/bin/env bash
# Build libicp_hip.so of another git revision for same-box A/B timing:
#   tools/build_ab.sh REV   ->  iterative-closest-point_amd/build_ab/REV/libicp_hip.so
# (load it with ICP_AMD_LIB=<that path>; boxes differ by up to ~8%, so compare in one call)
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REV=${1:?revision}
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" iterative-closest-point_amd include | tar -x -C "$TMP"
make -s -j8 -C "$TMP/iterative-closest-point_amd" build/libicp_hip.so
mkdir -p "$ROOT/iterative-closest-point_amd/build_ab/$REV"
cp "$TMP/iterative-closest-point_amd/build/libicp_hip.so" "$ROOT/iterative-closest-point_amd/build_ab/$REV/"
rm -rf "$TMP"
echo "$ROOT/iterative-closest-point_amd/build_ab/$REV/libicp_hip.so"
