#!/bin/bash
# Rebuilds the withdrawn bf16x3 DFT of round 4 from
# the round-4 render core (commit 7cae1df) + tools/dft_bf3.patch, in five
# forms of the statement that separated the permuted B fragments from their
# MFMAs, as tools/_lib/libbf3_<form>.so (render_fwd + errors only):
#   asm   the withdrawn fix: asm volatile("s_nop 7" : "+v" x 4 fragments)
#   noasm nothing (the form that returned stale bins)
#   pin   asm volatile("" : "+v" x 4): the fragments materialised, no wait states
#   nop   asm volatile("s_nop 7"): wait states only, no operands
#   sched __builtin_amdgcn_sched_barrier(0): scheduling order only
# and f32, the unpatched round-4 DFT.  tools/bf3_repro.py runs them.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/avr_bf3
rm -rf $W && mkdir -p $W/src $W/inc
for f in render_fwd.hip errors.cpp common.h probe.h stationary.h; do git -C $ROOT show 7cae1df:avr_amd/csrc/$f > $W/src/$f; done
git -C $ROOT show 7cae1df:include/avr_hip.h > $W/inc/avr_hip.h
FLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -fno-gpu-rdc -Wno-unused-function -Wno-inline-asm -I$W/inc"
mkdir -p $ROOT/tools/_lib
build() {  # form, source
  /opt/rocm/bin/hipcc $FLAGS -c $2 -o $W/$1_rf.o
  /opt/rocm/bin/hipcc $FLAGS -c $W/src/errors.cpp -o $W/errors.o
  /opt/rocm/bin/hipcc $FLAGS -shared $W/$1_rf.o $W/errors.o -o $ROOT/tools/_lib/libbf3_$1.so
}
build f32 $W/src/render_fwd.hip
(cd $W/src && patch -s -p3 < $ROOT/tools/dft_bf3.patch)
ASM='asm volatile("s_nop 7" : "+v"(chi), "+v"(clo), "+v"(shi), "+v"(slo));'
grep -qF "$ASM" $W/src/render_fwd.hip
build asm $W/src/render_fwd.hip
for form in noasm pin nop sched; do
  case $form in
    noasm) R='';;
    pin) R='asm volatile("" : "+v"(chi), "+v"(clo), "+v"(shi), "+v"(slo));';;
    nop) R='asm volatile("s_nop 7");';;
    sched) R='__builtin_amdgcn_sched_barrier(0);';;
  esac
  python3 -c "import sys; s=open('$W/src/render_fwd.hip').read(); open('$W/src/rf_$form.hip','w').write(s.replace(sys.argv[1], sys.argv[2]))" "$ASM" "$R"
  cp $W/src/*.h $W/ 2>/dev/null || true
  build $form $W/src/rf_$form.hip
done
ls $ROOT/tools/_lib/libbf3_*
