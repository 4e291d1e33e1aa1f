#!/bin/bash
# Build an A/B variant of libcnngp: netfuse.hip compiled with extra -D flags, linked with
# the regular cnngp.o into cnn-gp_amd/lib/ab/lib_<name>.so (tools/variants.sh times it).
#   bash tools/build_variant.sh NAME "-DFOO=1 -DBAR=0"
set -eu
cd "$(dirname "$0")/../cnn-gp_amd/csrc"
NAME=$1; DEFS=${2:-}
ROCM=/opt/rocm
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -I../../include -I$ROCM/include"
mkdir -p build/ab ../lib/ab
make -s build/cnngp.o
$ROCM/bin/hipcc $FL $DEFS -c netfuse.hip -o build/ab/netfuse_$NAME.o
$ROCM/bin/hipcc $FL build/cnngp.o build/ab/netfuse_$NAME.o -shared -L$ROCM/lib -lrocsolver -lrocblas -Wl,-rpath,$ROCM/lib -o ../lib/ab/lib_$NAME.so
echo "built lib/ab/lib_$NAME.so ($DEFS)"
