#!/bin/bash
# Library variant for same-box A/B (tools/ab_demod.sh):
#   tools/build_variant.sh NAME "-DFLAG ..." [SRC]       extra compiler flags, or
#   tools/build_variant.sh NAME tools/variants/X.sed [SRC]   a sed patch applied to a copy of the source
#   tools/build_variant.sh NAME tools/variants/X.py [SRC]    a python filter (stdin -> stdout) likewise
# rebuilds csrc/SRC.hip (default etsi_rx) and links lib/variants/libNAME.so from the other objects of
# the current build.  Timing-only variants (a phase skipped, outputs wrong) live as patches here, not
# as #ifdefs in the product kernels.
set -e
cd "$(dirname "$0")/../tetraear-bladerf_amd"
make -s
SRC=${3:-etsi_rx}
mkdir -p build/var lib/variants
FLAGS="$2"
IN=csrc/$SRC.hip
if [[ "$2" == *.sed || "$2" == *.py ]]; then
    IN=build/var/${SRC}_$1.hip
    if [[ "$2" == *.sed ]]; then sed -f "../$2" csrc/$SRC.hip > $IN; else python3 "../$2" < csrc/$SRC.hip > $IN; fi
    cmp -s csrc/$SRC.hip $IN && { echo "patch $2 changed nothing" >&2; exit 1; }
    FLAGS="-Icsrc"
fi
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function $FLAGS \
    -c $IN -o build/var/${SRC}_$1.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o lib/variants/lib$1.so \
    $(ls build/*.o | grep -v "/$SRC.o") build/var/${SRC}_$1.o -L/opt/rocm/lib -lrocfft -Wl,-rpath,/opt/rocm/lib
echo lib/variants/lib$1.so
