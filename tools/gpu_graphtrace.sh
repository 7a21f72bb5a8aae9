set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gtrace -o run --output-format csv -- python tools/graph_probe.py > gpurun_out/gtrace.log 2>&1 || exit 1
tail -1 gpurun_out/gtrace.log
