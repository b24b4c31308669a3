#!/bin/bash
# Strip kernel against the separable path over radii (1080p D=128, 8 frames per call): tools/r6_strip_sweep.sh LIB RADII
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIB=$1; shift
for r in "$@"; do tools/r6_strip_ab.sh r6sw_$r "tools/abv/nostrip.so $LIB" $r || exit 1; done
