#!/bin/bash
# A/B variant of the library: some sources (default zk_msm.hip, the G1 MSM instantiations)
# recompiled with extra flags, linked with the in-tree build's other objects ->
# variants/NAME/libzkalgebra_gpu.so (selected at run time by ZK_LIB_PATH, tools/job_cmd.sh).
# Run after `make` in the package.
#   bash tools/build_variant.sh NAME "-DZK_KARA_MADD=0 -DZK_KARA_ADD=0" [zk_msm zk_ntt ...]
set -e
NAME=${1:?name}
FLAGS=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/zikkurat-algebra_amd
OUT=$ROOT/variants/$NAME
mkdir -p "$OUT"
shift 2 || true
UNITS=${@:-zk_msm}
OBJS=""
for u in $UNITS; do
  SRC=${VARIANT_SRC:-$PKG/csrc}  # VARIANT_SRC: an edited copy of csrc/ (experiments outside the tree)
  src="$SRC/$u.hip"; [ -f "$src" ] || src="$SRC/$u.cpp"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -Wall -Wno-unused-function \
    -Wno-unused-result $FLAGS -c "$src" -o "$OUT/$u.o"
  OBJS="$OBJS $OUT/$u.o"
done
for o in "$PKG"/build/*.o; do
  b=$(basename "$o" .o)
  case " $UNITS " in *" $b "*) ;; *) OBJS="$OBJS $o" ;; esac
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-Bsymbolic -Wl,--no-undefined $OBJS \
  -o "$OUT/libzkalgebra_gpu.so" -lpthread -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "$FLAGS" > "$OUT/FLAGS"
echo "built $OUT/libzkalgebra_gpu.so ($FLAGS)"
