#!/bin/bash
# Hash-grid backward reduce tiling A/B (partition size, waves per block;
# variant libraries built by tools/build_ab.sh with -DAVR_HG_PART_BITS /
# -DAVR_HG_REDUCE_WAVES overrides, removed once the A/B kept the defaults),
# config-3 and config-4 training points, libraries interleaved in one process.
set -u
OUT=gpurun_out/${1:-hgab}
mkdir -p $OUT
export TMPDIR=/tmp
L=""
for n in base w2 w8 b9 b9w8 b11 b11w2; do L="$L,$n=tools/_lib/libab_hg_$n.so"; done
L=${L#,}
for w in c3_raf_furnished_b4 c4_raf_empty_b4_per_gpu; do
  timeout -k 10 300 python tools/xbench_hgbwd.py $L --workload $w --rounds 5 --iters 10 > $OUT/$w.log 2>&1 || { echo "$w failed"; tail -20 $OUT/$w.log; exit 1; }
  grep "^{" $OUT/$w.log
done
echo all-ok
