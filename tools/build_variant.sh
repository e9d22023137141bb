#!/bin/bash
# Experiment builds: libpmg_hip.so with ONE translation unit replaced / re-flagged.
#   tools/build_variant.sh NAME SRC.hip [extra hipcc flags...]
# -> exp/NAME/libpmg_hip.so (load it with PMG_LIB_PATH=exp/NAME/libpmg_hip.so)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/poor_man_gplvm_amd/csrc
NAME=$1; SRC=$2; shift 2
base=$(basename "$SRC" .hip)
mkdir -p "$R/exp/$NAME"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-pass-failed \
  -I"$C" -I"$R/include" "$@" -c "$SRC" -o "$R/exp/$NAME/$base.o"
objs=""
for o in "$C"/*.o; do
  b=$(basename "$o" .o)
  if [ "$b" = "${base%%_v[0-9]*}" ] || [ "$b" = "$base" ]; then continue; fi
  objs="$objs $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$R/exp/$NAME/libpmg_hip.so" $objs "$R/exp/$NAME/$base.o"
echo "built exp/$NAME/libpmg_hip.so"
