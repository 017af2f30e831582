#!/bin/bash
# Library variant for same-box A/B (tools/ab_demod.sh): tools/build_variant.sh NAME "-DFLAG ..." [SRC]
# rebuilds csrc/SRC.hip (default etsi_rx) with the extra flags and links lib/variants/libNAME.so
# from the other objects of the current build.
set -e
cd "$(dirname "$0")/../tetraear-bladerf_amd"
make -s
SRC=${3:-etsi_rx}
mkdir -p build/var lib/variants
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function $2 \
    -c csrc/$SRC.hip -o build/var/${SRC}_$1.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o lib/variants/lib$1.so \
    $(ls build/*.o | grep -v "/$SRC.o") build/var/${SRC}_$1.o -L/opt/rocm/lib -lrocfft -Wl,-rpath,/opt/rocm/lib
echo lib/variants/lib$1.so
