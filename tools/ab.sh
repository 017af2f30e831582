#!/bin/bash
# Same-box A/B of library variants -- the one tool behind every "measured and dropped" line in
# DESIGN.md (records: profiles/r0*_ab_*.txt).  Boxes differ by up to +-5 %, so variants are only ever
# compared inside one gpurun call, three rounds interleaved.
#
#   tools/ab.sh build NAME SPEC [SRC]   lib/variants/libNAME.so, csrc/SRC.hip (default etsi_rx) changed by
#        SPEC = tools/ab_patches/X.py   a python filter (stdin -> stdout; timing-only patches: a phase
#                                       skipped, outputs wrong -- never #ifdefs in the product kernels)
#             | tools/ab_patches/X.sed  a sed script
#             | head:REV                the file as it was at git revision REV (the "before" side)
#             | "-DFLAG ..."            extra compiler flags
#        and every other object from the current build.
#   tools/ab.sh run LIB...              bench each library (TETRA_HIP_LIB) for AB_ROUNDS rounds (default 3)
#                                       with AB_ARGS (default the serial ETSI bench: --pipeline off)
#   tools/ab.sh env "A=1" "A=0 B=2" ... the same for environment settings on the default bench
# Run `build` here (CPU), `run` / `env` on the GPU box, e.g.
#   gpurun -- 'AB_ARGS=" " bash tools/ab.sh run tetraear-bladerf_amd/lib/libtetra_hip.so \
#              tetraear-bladerf_amd/lib/variants/libX.so > gpurun_out/ab.txt'
set -e
cmd=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
summ() {   # one line per run: label, ms/step, per-stage ms, read floor
    python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[2]) if l.startswith('{')][-1]; print(sys.argv[1], d['ms_per_step'], d['stages_ms_per_step'], d['roofline'].get('measured_read_floor_GBs'))" "$1" "$2"
}
case $cmd in
build)
    NAME=$1; SPEC=$2; SRC=${3:-etsi_rx}
    cd $R/tetraear-bladerf_amd
    make -s
    mkdir -p build/var lib/variants
    IN=build/var/${SRC}_$NAME.hip
    FLAGS="-Icsrc"
    case $SPEC in
        head:*) git show ${SPEC#head:}:tetraear-bladerf_amd/csrc/$SRC.hip > $IN ;;
        *.sed) sed -f "$R/$SPEC" csrc/$SRC.hip > $IN ;;
        *.py) python3 "$R/$SPEC" < csrc/$SRC.hip > $IN ;;
        *) cp csrc/$SRC.hip $IN; FLAGS="-Icsrc $SPEC" ;;
    esac
    if [[ "$SPEC" == *.sed || "$SPEC" == *.py ]] && cmp -s csrc/$SRC.hip $IN; then
        echo "patch $SPEC changed nothing (it no longer applies to csrc/$SRC.hip)" >&2; exit 1
    fi
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function \
        $FLAGS -c $IN -o build/var/${SRC}_$NAME.o
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o lib/variants/lib$NAME.so \
        $(ls build/*.o | grep -v "/$SRC.o") build/var/${SRC}_$NAME.o -L/opt/rocm/lib -lrocfft -Wl,-rpath,/opt/rocm/lib
    echo tetraear-bladerf_amd/lib/variants/lib$NAME.so ;;
run)
    O=$R/gpurun_out/ab; mkdir -p $O; cd $R
    for i in $(seq 1 ${AB_ROUNDS:-3}); do
        for L in "$@"; do
            n=$(basename $L .so)
            TETRA_HIP_LIB=$R/$L timeout -k 10 200 python -u bench.py --no-cpu --steps 30 ${AB_ARGS:---pipeline off} \
                > $O/$n.$i.log 2>&1
            summ "$n" $O/$n.$i.log
        done
    done ;;
env)
    O=$R/gpurun_out/abenv; mkdir -p $O; cd $R
    for i in $(seq 1 ${AB_ROUNDS:-3}); do
        k=0
        for E in "$@"; do
            k=$((k + 1))
            env $E timeout -k 10 200 python -u bench.py --no-cpu --steps 30 ${AB_ARGS} > $O/$k.$i.log 2>&1
            summ "$E" $O/$k.$i.log
        done
    done ;;
*) echo "usage: tools/ab.sh build|run|env ..." >&2; exit 2 ;;
esac
