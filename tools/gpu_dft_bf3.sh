#!/bin/bash
# bf16x3 DFT: the render / graph / property / head / criterion tests, then
# the serial IR timeline with the bf16x3 and the fp32 DFT (shape-probe
# library, AVR_DFT_F32_PROBE), twice each.
set -u
OUT=$PWD/gpurun_out/dft_bf3
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -W ignore -m gpu tests/test_gpu_render.py tests/test_gpu_graph.py tests/test_gpu_properties.py tests/test_gpu_head.py tests/test_gpu_knobs.py > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit $rc; }
for i in 1 2; do
  for v in 0 1; do
    (export AVR_DFT_F32_PROBE=$v; timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/f32_$v.$i -o run --output-format csv -- python tools/lat_trace.py --shapes) > $OUT/f32_$v.$i.log 2>&1 || { tail $OUT/f32_$v.$i.log; exit 1; }
    echo "== fp32=$v $(grep latency_ms $OUT/f32_$v.$i.log)"
    python tools/lat_trace.py --report $(ls $OUT/f32_$v.$i/*/run_kernel_trace.csv $OUT/f32_$v.$i/run_kernel_trace.csv 2>/dev/null | head -1) | grep -E "dft|finalize|reduce|median span"
  done
done
