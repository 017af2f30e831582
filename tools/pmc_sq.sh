#!/bin/bash
# SQ counters (one rocprofv3 --pmc pass, 8 SQ slots) for the serial ETSI bench: where the demod's
# wave cycles go (MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES,
# quad-cycles).  usage: tools/pmc_sq.sh TAG [bench args]
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE --output-format csv -d $O/sq1 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --pipeline off "$@" > $O/sq1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC SQ_WAVES SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD --output-format csv -d $O/sq2 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --pipeline off "$@" > $O/sq2.log 2>&1
