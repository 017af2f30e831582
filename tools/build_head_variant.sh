#!/bin/bash
# lib/variants/libNAME.so with csrc/SRC.hip taken from git revision REV (default HEAD) and every other
# object from the current build -- the "before" side of a same-box A/B (tools/ab_demod.sh).
#   tools/build_head_variant.sh NAME [REV] [SRC]
set -e
cd "$(dirname "$0")/../tetraear-bladerf_amd"
make -s
REV=${2:-HEAD}
SRC=${3:-etsi_rx}
mkdir -p build/var lib/variants
git show $REV:tetraear-bladerf_amd/csrc/$SRC.hip > build/var/${SRC}_$1.hip
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function -Icsrc \
    -c build/var/${SRC}_$1.hip -o build/var/${SRC}_$1.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o lib/variants/lib$1.so \
    $(ls build/*.o | grep -v "/$SRC.o") build/var/${SRC}_$1.o -L/opt/rocm/lib -lrocfft -Wl,-rpath,/opt/rocm/lib
echo lib/variants/lib$1.so
