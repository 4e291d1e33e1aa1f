#!/bin/bash
# Build an A/B variant of libcnngp: netfuse.hip (default), cnngp.hip (VARIANT_SRC=cnngp) or
# both (VARIANT_SRC=both) compiled with extra -D flags and linked with the regular object of
# the other into cnn-gp_amd/lib/ab/lib_<name>.so (tools/gpu.sh ab / tools/ab_variant.sh time it).
#   bash tools/build_variant.sh NAME "-DFOO=1 -DBAR=0"
set -eu
cd "$(dirname "$0")/../cnn-gp_amd/csrc"
NAME=$1; DEFS=${2:-}; SRC=${VARIANT_SRC:-netfuse}
ROCM=/opt/rocm
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -I../../include -I$ROCM/include"
mkdir -p build/ab ../lib/ab
make -s build/cnngp.o build/netfuse.o
C=build/cnngp.o; F=build/netfuse.o
if [ "$SRC" = cnngp ] || [ "$SRC" = both ]; then
    $ROCM/bin/hipcc $FL $DEFS -c cnngp.hip -o build/ab/cnngp_$NAME.o; C=build/ab/cnngp_$NAME.o
fi
if [ "$SRC" = netfuse ] || [ "$SRC" = both ]; then
    $ROCM/bin/hipcc $FL $DEFS -c netfuse.hip -o build/ab/netfuse_$NAME.o; F=build/ab/netfuse_$NAME.o
fi
$ROCM/bin/hipcc $FL $C $F -shared -L$ROCM/lib -lrocsolver -lrocblas -Wl,-rpath,$ROCM/lib -o ../lib/ab/lib_$NAME.so
echo "built lib/ab/lib_$NAME.so ($SRC $DEFS)"
