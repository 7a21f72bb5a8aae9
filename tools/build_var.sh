#!/bin/bash
# Variant library for kernel A/B timing (tools/xbench_exact.py): the named
# sources compiled with extra -D switches into tools/_lib/libvar_<NAME>.so.
#   tools/build_var.sh NAME "-DAVR_EXACT_STAGGER=1" [head_exact.hip ...]
set -e
NAME=$1; DEFS=$2; shift 2
SRCS=${@:-head_exact.hip}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/tools/_lib/libvar_$NAME.so
mkdir -p $ROOT/tools/_lib /tmp/avr_var_$NAME
FLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -fno-gpu-rdc -Wall -Wno-unused-function -Wno-inline-asm -I$ROOT/include"
OBJS=""
for f in errors.cpp $SRCS; do
  /opt/rocm/bin/hipcc $FLAGS ${EXTRA:-} $DEFS -c $ROOT/avr_amd/csrc/$f -o /tmp/avr_var_$NAME/$f.o
  OBJS="$OBJS /tmp/avr_var_$NAME/$f.o"
done
/opt/rocm/bin/hipcc $FLAGS -shared $OBJS -o $OUT
echo $OUT
