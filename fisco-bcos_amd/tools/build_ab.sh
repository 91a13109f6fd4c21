# Build an A/B variant of libbcosgpu.so: one kernel TU recompiled with extra flags, linked with the
# other objects of the current build, into fisco-bcos_amd/lib_ab/<name>/libbcosgpu.so.
#   bash fisco-bcos_amd/tools/build_ab.sh <name> <tu, e.g. ecc_coop> [extra hipcc flags...]
# (tools/gpu_run.sh step `ab=<name>,<bench args>` swaps it in on the GPU box for one bench run)
set -e
HERE=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; TU=$2; shift 2
OUT=$HERE/lib_ab/$NAME      # the .so only (travels to the GPU box)
OBJ=$HERE/build_ab/$NAME    # the object (gpurun-ignored)
mkdir -p $OUT $OBJ
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -mllvm -amdgpu-dpp-combine=false \
  "$@" -c $HERE/csrc/$TU.hip -o $OBJ/$TU.o 2> $OBJ/build.log
OBJS=""
for o in $HERE/build/*.o; do
  b=$(basename $o)
  if [ "$b" = "$TU.o" ]; then OBJS="$OBJS $OBJ/$TU.o"; else OBJS="$OBJS $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $OUT/libbcosgpu.so $OBJS -lpthread
echo "$NAME: $TU $* -> $OUT/libbcosgpu.so"
