#!/bin/bash
# Render-core change check: render / graph / knob / head tests, then the
# driver's bench line against the round-3 library (_ab_r3/), interleaved.
set -u
OUT=gpurun_out/core_check
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -W ignore -m gpu tests/test_gpu_render.py tests/test_gpu_graph.py tests/test_gpu_knobs.py tests/test_gpu_head.py tests/test_gpu_properties.py > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit $rc; }
bash tools/gpu_ab_r3.sh
