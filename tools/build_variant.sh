#!/bin/bash
# Build an A/B variant of libcnngp: one translation unit (netfuse.hip by default, or
# VARIANT_SRC=cnngp) compiled with extra -D flags and linked with the regular object of the
# other into cnn-gp_amd/lib/ab/lib_<name>.so (tools/gpu.sh ab / tools/variants.sh time it).
#   bash tools/build_variant.sh NAME "-DFOO=1 -DBAR=0"
set -eu
cd "$(dirname "$0")/../cnn-gp_amd/csrc"
NAME=$1; DEFS=${2:-}; SRC=${VARIANT_SRC:-netfuse}
ROCM=/opt/rocm
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -I../../include -I$ROCM/include"
mkdir -p build/ab ../lib/ab
make -s build/cnngp.o build/netfuse.o
$ROCM/bin/hipcc $FL $DEFS -c $SRC.hip -o build/ab/${SRC}_$NAME.o
if [ "$SRC" = netfuse ]; then OBJS="build/cnngp.o build/ab/netfuse_$NAME.o"
else OBJS="build/ab/cnngp_$NAME.o build/netfuse.o"; fi
$ROCM/bin/hipcc $FL $OBJS -shared -L$ROCM/lib -lrocsolver -lrocblas -Wl,-rpath,$ROCM/lib -o ../lib/ab/lib_$NAME.so
echo "built lib/ab/lib_$NAME.so ($SRC.hip $DEFS)"
