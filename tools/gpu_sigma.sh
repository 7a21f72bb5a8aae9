#!/bin/bash
# Fused sigma networks: GPU parity tests, kernel timing per tile config,
# end-to-end inference bench and its kernel-trace profile.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sigma.py -x -v --timeout 120 --timeout-method thread -W ignore > gpurun_out/sigma_tests.log 2>&1
rc=$?; tail -3 gpurun_out/sigma_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/probe_sigma.py --cfgs 0,1,2,3 > gpurun_out/probe_sigma.log 2>&1 || exit 1
timeout -k 10 200 python tools/probe_sigma.py --variant 1 --cfgs 0,1 >> gpurun_out/probe_sigma.log 2>&1 && timeout -k 10 200 python tools/probe_sigma.py --variant 2 --cfgs 0,1 >> gpurun_out/probe_sigma.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/probe_sigma.log
timeout -k 10 300 python tools/bench_infer.py > gpurun_out/infer.log 2>&1 || exit 1
tail -1 gpurun_out/infer.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profinfer -o run --output-format csv -- python tools/bench_infer.py --steps 5 --warmup 2 --variants fused > gpurun_out/profinfer.log 2>&1 || exit 1
