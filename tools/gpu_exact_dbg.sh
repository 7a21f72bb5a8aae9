#!/bin/bash
# Exact head forms (AVR_HEAD_EXACT_WAVES: 8 register staging; LDS-DMA 16: 32-ray tiles x 3
# buffers, 17: 64 x 2, 18: 32 x 4) and phase switches of form 18
# (AVR_HEAD_EXACT_DBG: 1 no MFMA, 2 no HBM stream, 4 no epilogue)
set -u
for wv in 18; do
  echo "waves=$wv"; AVR_HEAD_EXACT_WAVES=$wv timeout -k 10 120 python tools/probe_exact_head.py --modes exact || exit 1
done
for d in 24; do
  echo "form18 dbg=$d"; AVR_HEAD_EXACT_WAVES=18 AVR_HEAD_EXACT_DBG=$d timeout -k 10 120 python tools/probe_exact_head.py --modes exact || exit 1
done
