#!/bin/bash
# Build an A/B variant of the library: tools/build_ab.sh NAME "-DFOO=1 ..."
# recompiles the .hip sources with the extra flags, links them with the default host objects of
# ignnition_amd/build/, writes ignnition_amd/ab/lib_NAME.so (tools/ab_lib.sh runs it)
set -e
NAME=$1; DEFS=$2
cd "$(dirname "$0")/.."
python -m ignnition_amd.build > /dev/null
mkdir -p ignnition_amd/ab/obj_$NAME
pids=""
for SRC in kernels.hip kernels_bf.hip train_kernels.hip readout_kernels.hip resident.hip readout_h32.hip train_csr.hip; do
  EXTRA=""
  { [ "$SRC" = kernels_bf.hip ] || [ "$SRC" = resident.hip ] || [ "$SRC" = readout_h32.hip ]; } && EXTRA="-mllvm -amdgpu-mfma-vgpr-form"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -Wno-unused-value $EXTRA $DEFS \
    -c ignnition_amd/csrc/$SRC -o ignnition_amd/ab/obj_$NAME/$SRC.o &
  pids="$pids $!"
done
for p in $pids; do wait $p; done
OBJS=""
for o in ignnition_amd/build/*.o; do
  b=$(basename $o)
  if [ -f ignnition_amd/ab/obj_$NAME/$b ]; then OBJS="$OBJS ignnition_amd/ab/obj_$NAME/$b"; else OBJS="$OBJS $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS -o ignnition_amd/ab/lib_$NAME.so -lz -lpthread
echo ignnition_amd/ab/lib_$NAME.so
