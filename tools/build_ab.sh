#!/bin/bash
# Build an A/B library of one kernel source: errors.cpp + SRC (default
# head_exact.hip; and the headers they include) from a git revision, or from
# the working tree ("-"), into tools/_lib/libab_<name>.so, for
# tools/xbench_exact.py / tools/xbench_hgbwd.py.
#   [SRC=hashgrid.hip] bash tools/build_ab.sh NAME REV|- [extra hipcc flags...]
set -e
NAME=$1; REV=$2; shift 2
SRC=${SRC:-head_exact.hip}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/avr_ab_$NAME
rm -rf $W && mkdir -p $W/src $W/inc
for f in errors.cpp $SRC common.h probe.h stationary.h; do
  if [ "$REV" = "-" ]; then cp $ROOT/avr_amd/csrc/$f $W/src/$f; else git -C $ROOT show $REV:avr_amd/csrc/$f > $W/src/$f; fi
done
if [ "$REV" = "-" ]; then cp $ROOT/include/avr_hip.h $W/inc/; else git -C $ROOT show $REV:include/avr_hip.h > $W/inc/avr_hip.h; fi
FLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -fno-gpu-rdc -Wno-unused-function -Wno-inline-asm --offload-compress -I$W/inc"
mkdir -p $ROOT/tools/_lib
/opt/rocm/bin/hipcc $FLAGS "$@" -c $W/src/$SRC -o $W/he.o
/opt/rocm/bin/hipcc $FLAGS -c $W/src/errors.cpp -o $W/errors.o
/opt/rocm/bin/hipcc $FLAGS -shared $W/he.o $W/errors.o -o $ROOT/tools/_lib/libab_$NAME.so
echo built tools/_lib/libab_$NAME.so
