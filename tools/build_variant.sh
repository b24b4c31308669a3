#!/bin/bash
# Build a libsm_hip.so variant for same-box A/B timing: tools/build_variant.sh NAME "-DFOO=1 ..."
# -> tools/abv/NAME.so (objects under tools/abv/NAME/).  Not part of the product build.
# SM_VARIANT_ONLY="bm_volume bm_staged": recompile only those sources with the extra flags and link
# them with the product's objects (gpu_stereo_matching_amd/csrc/build/, which must be current).
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
EXTRA="$*"
SRC=${SM_VARIANT_SRC:-gpu_stereo_matching_amd/csrc}
OUT=tools/abv/$NAME
mkdir -p $OUT
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -fvisibility=hidden -Wall -Wno-unused-result $EXTRA"
ALL="sm_capi bm_box bm_aux bm_guided bm_segtree bm_pre bm_post bm_volume bm_staged bm_rectify bm_literal bm_wide bm_strip bm_strip_lr"
if [ -n "$SM_VARIANT_ONLY" ]; then
  for f in $ALL; do cp gpu_stereo_matching_amd/csrc/build/$f.o $OUT/$f.o; done
  ALL="$SM_VARIANT_ONLY"
fi
pids=()
for f in $ALL; do
  /opt/rocm/bin/hipcc $FLAGS -c $SRC/$f.hip -o $OUT/$f.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o tools/abv/$NAME.so $OUT/*.o
echo built tools/abv/$NAME.so
