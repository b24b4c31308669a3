#!/bin/bash
# Build libsm_hip.so from the sources of git revision REV into tools/abv/NAME.so (same-box A/B against
# the working tree's build).  usage: tools/build_rev_variant.sh NAME REV [extra hipcc flags]
set -e
cd "$(dirname "$0")/.."
NAME=$1; REV=$2; shift 2
EXTRA="$*"
TMP=$(mktemp -d)
git archive "$REV" gpu_stereo_matching_amd/csrc include | tar -x -C "$TMP"
OUT=tools/abv/$NAME
mkdir -p $OUT
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -fvisibility=hidden -Wall -Wno-unused-result $EXTRA"
pids=()
for f in $TMP/gpu_stereo_matching_amd/csrc/*.hip; do
  b=$(basename $f .hip)
  /opt/rocm/bin/hipcc $FLAGS -c $f -o $OUT/$b.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o tools/abv/$NAME.so $OUT/*.o
rm -rf "$TMP"
echo built tools/abv/$NAME.so
