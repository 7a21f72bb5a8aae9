#!/bin/bash
# Build a previous commit's exact head as csrc/build/libavr_exact_old.so for
# tools/ab_exact.py (its own header and stationary.h/probe.h of that commit).
set -eu
REV=${1:-HEAD}
D=$(mktemp -d)
mkdir -p $D/inc
git show $REV:include/avr_hip.h > $D/inc/avr_hip.h
for f in head_exact.hip stationary.h probe.h common.h errors.cpp; do git show $REV:avr_amd/csrc/$f > $D/$f; done
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -fno-gpu-rdc -I$D/inc -I$D -shared \
  $D/head_exact.hip $D/errors.cpp -o avr_amd/csrc/build/libavr_exact_old.so
rm -rf $D
