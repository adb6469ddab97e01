#!/bin/bash
# Build an A/B variant of the library: tools/build_ab.sh NAME "-DFOO=1 ..." [source]
# recompiles one source (default kernels_bf.hip) with the extra flags, links it with the default
# objects of ignnition_amd/build/, writes ignnition_amd/ab/lib_NAME.so (tools/ab_lib.sh runs it)
set -e
NAME=$1; DEFS=$2; SRC=${3:-kernels_bf.hip}
cd "$(dirname "$0")/.."
python -m ignnition_amd.build > /dev/null
mkdir -p ignnition_amd/ab/obj_$NAME
EXTRA=""
[ "$SRC" = kernels_bf.hip ] && EXTRA="-mllvm -amdgpu-mfma-vgpr-form"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -Wno-unused-value $EXTRA $DEFS \
  -c ignnition_amd/csrc/$SRC -o ignnition_amd/ab/obj_$NAME/$SRC.o
OBJS=""
for o in ignnition_amd/build/*.o; do
  b=$(basename $o)
  if [ "$b" = "$SRC.o" ]; then OBJS="$OBJS ignnition_amd/ab/obj_$NAME/$SRC.o"; else OBJS="$OBJS $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS -o ignnition_amd/ab/lib_$NAME.so -lz -lpthread
echo ignnition_amd/ab/lib_$NAME.so
