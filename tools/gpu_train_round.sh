set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_criterion.py -x -v --timeout 120 --timeout-method thread -W ignore > gpurun_out/train_tests.log 2>&1 || { tail -40 gpurun_out/train_tests.log; exit 1; }
tail -5 gpurun_out/train_tests.log
timeout -k 10 300 python tools/bench_train.py > gpurun_out/bt_crit.log 2>&1 && tail -1 gpurun_out/bt_crit.log
timeout -k 10 300 python tools/bench_train.py --loss l1 > gpurun_out/bt_l1.log 2>&1 && tail -1 gpurun_out/bt_l1.log
timeout -k 10 300 python tools/bench_train.py --nan-check > gpurun_out/bt_nan.log 2>&1 && tail -1 gpurun_out/bt_nan.log
timeout -k 10 300 python tools/bench_train.py --workload c4_raf_empty_b4_per_gpu > gpurun_out/bt_c4.log 2>&1 && tail -1 gpurun_out/bt_c4.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/proftrain -o run --output-format csv -- python tools/bench_train.py --steps 5 --warmup 2 > gpurun_out/proftrain.log 2>&1 && echo profok
