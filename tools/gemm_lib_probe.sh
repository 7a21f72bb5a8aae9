#!/bin/bash
# GEMM library probe for the MLP layer shape: hipBLASLt default, rocBLAS,
# and TunableOp (exhaustive hipBLASLt/rocBLAS solution search).
set -u
mkdir -p gpurun_out
timeout -k 10 120 python tools/fwd_probe.py > gpurun_out/gp_default.log 2>&1; tail -1 gpurun_out/gp_default.log
timeout -k 10 120 python -c "
import torch, sys; sys.argv=['x']; torch.backends.cuda.preferred_blas_library('cublas')
import runpy; runpy.run_path('tools/fwd_probe.py', run_name='__main__')" > gpurun_out/gp_rocblas.log 2>&1; tail -1 gpurun_out/gp_rocblas.log
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop.csv PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=200 timeout -k 10 400 python tools/fwd_probe.py > gpurun_out/gp_tunable.log 2>&1; tail -1 gpurun_out/gp_tunable.log
