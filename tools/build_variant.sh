#!/bin/bash
# A/B variant of the library: zk_msm.hip (the G1 MSM instantiations) recompiled with extra
# flags, linked with the in-tree build's other objects -> variants/NAME/libzkalgebra_gpu.so
# (selected at run time by ZK_LIB_PATH, tools/job_cmd.sh).  Run after `make` in the package.
#   bash tools/build_variant.sh NAME "-DZK_KARA_MADD=0 -DZK_KARA_ADD=0"
set -e
NAME=${1:?name}
FLAGS=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/zikkurat-algebra_amd
OUT=$ROOT/variants/$NAME
mkdir -p "$OUT"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -Wall -Wno-unused-function \
  -Wno-unused-result $FLAGS -c "$PKG/csrc/zk_msm.hip" -o "$OUT/zk_msm.o"
OBJS=$(ls "$PKG"/build/*.o | grep -v '/zk_msm.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-Bsymbolic -Wl,--no-undefined "$OUT/zk_msm.o" $OBJS \
  -o "$OUT/libzkalgebra_gpu.so" -lpthread
echo "$FLAGS" > "$OUT/FLAGS"
echo "built $OUT/libzkalgebra_gpu.so ($FLAGS)"
