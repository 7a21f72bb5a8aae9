#!/bin/bash
# Run the given GPU test files/node ids in ONE pytest process (stops at the
# first failure), log under gpurun_out/tests/.
set -u
OUT=gpurun_out/tests
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -W ignore "$@" > $OUT/tests.log 2>&1
rc=$?; grep -cE "PASSED" $OUT/tests.log; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -40; exit $rc; }
