#!/bin/bash
# Phase switches of the exact head (AVR_HEAD_EXACT_DBG: 1 no MFMA, 2 no h loads, 3 neither)
set -u
for d in 0; do
  echo "dbg=$d"; AVR_HEAD_EXACT_DBG=$d timeout -k 10 120 python tools/probe_exact_head.py --modes exact || exit 1
done
for wv in 0; do
  echo "waves=$wv"; AVR_HEAD_EXACT_WAVES=$wv timeout -k 10 120 python tools/probe_exact_head.py --modes exact || exit 1
done
