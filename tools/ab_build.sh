#!/bin/bash
# Builds variant copies of libzfec_hip.so for kernel A/Bs, each in
# abuild/<name>/ (git-ignored; travels to the GPU box with the tree).
# kernels.hip and bitslice.cpp (the JIT generator) are rebuilt per variant;
# the other objects are the in-tree build's (run `make` first).  A variant is
#
#   name=FLAGS        kernels.hip of this tree with extra compiler flags, e.g.
#                     "base=-DZFEC_TR64=0 -DZFEC_BSR_EARLY_ADDR=0 legacy"
#                     (the word `legacy` swaps in round 5's routine forms:
#                     tools/gen_gf_routines.py --form legacy; `form=NAME` any
#                     other form, e.g. form=trunc64, a timing-only experiment)
#   name=git:REV      kernels.hip, kernels.hpp and gf_routines.inc of commit REV
#   "name=git:REV FLAGS"  the same with compiler flags (a knob of that commit)
#
# The library loads its variant with ZFEC_HIP_LIB=abuild/<name>/libzfec_hip.so
# (zfec_amd/capi.py); tools/ab_bsr.py runs the variants interleaved.
#
#   tools/ab_build.sh "r05=git:a1850ed" "base=-DZFEC_TR64=0 legacy" "new="
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FLAGS="--offload-arch=gfx950 -mcode-object-version=5 -O3 -std=c++17 -fPIC -fvisibility=hidden -Wall -Wno-unused-function"
SRC=$ROOT/zfec_amd/csrc
OBJS="$SRC/fec_abi.o $SRC/gf256.o $SRC/host_pool.o $SRC/config.o"
for o in $OBJS; do [ -f "$o" ] || { echo "ab_build: $o missing (run make)"; exit 1; }; done
pids=()
for spec in "$@"; do
  name=${spec%%=*}
  val=${spec#*=}
  out=$ROOT/abuild/$name
  rm -rf "$out"
  mkdir -p "$out"
  (
    set -e
    if [[ $val == git:* ]]; then
      rev=${val#git:}
      gflags=""
      if [[ $rev == *" "* ]]; then gflags=${rev#* }; rev=${rev%% *}; fi
      mkdir -p "$out/src"
      for f in kernels.hip kernels.hpp gf_routines.inc; do
        git -C "$ROOT" show "$rev:zfec_amd/csrc/$f" > "$out/src/$f"
      done
      cp "$SRC"/*.hpp "$out/src/" 2>/dev/null || true
      git -C "$ROOT" show "$rev:zfec_amd/csrc/kernels.hpp" > "$out/src/kernels.hpp"
      $HIPCC $FLAGS -I"$ROOT/include" $gflags -c "$out/src/kernels.hip" -o "$out/kernels.o"
    else
      extra=()
      for w in $val; do
        if [ "$w" = legacy ] || [[ $w == form=* ]]; then
          form=${w#form=}
          python3 "$ROOT/tools/gen_gf_routines.py" --form "$form" --out "$out/gf_routines_$form.inc"
          extra+=("-DZFEC_GF_ROUTINES_INC=\"$out/gf_routines_$form.inc\"")
        else
          extra+=("$w")
        fi
      done
      $HIPCC $FLAGS -I"$ROOT/include" "${extra[@]}" -c "$SRC/kernels.hip" -o "$out/kernels.o"
      $HIPCC $FLAGS -I"$ROOT/include" "${extra[@]}" -c "$SRC/bitslice.cpp" -o "$out/bitslice.o"
    fi
    [ -f "$out/bitslice.o" ] || cp "$SRC/bitslice.o" "$out/bitslice.o"
    $HIPCC --offload-arch=gfx950 -shared -fPIC -o "$out/libzfec_hip.so" "$out/kernels.o" "$out/bitslice.o" $OBJS \
      -ldl -lpthread
    rm -f "$out/kernels.o" "$out/bitslice.o"
    echo "$spec" > "$out/SPEC"
    echo "built abuild/$name ($spec)"
  ) &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=1; done
exit $rc
