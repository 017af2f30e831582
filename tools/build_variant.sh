#!/bin/bash
# Library variant for same-box A/B (tools/ab_demod.sh): tools/build_variant.sh NAME "-DFLAG ..."
# rebuilds etsi_rx.hip with the extra flags and links lib/variants/libNAME.so from the other objects.
set -e
cd "$(dirname "$0")/../tetraear-bladerf_amd"
make -s
mkdir -p build/var lib/variants
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function $2 \
    -c csrc/etsi_rx.hip -o build/var/etsi_rx_$1.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o lib/variants/lib$1.so \
    $(ls build/*.o | grep -v etsi_rx.o) build/var/etsi_rx_$1.o -L/opt/rocm/lib -lrocfft -Wl,-rpath,/opt/rocm/lib
echo lib/variants/lib$1.so
