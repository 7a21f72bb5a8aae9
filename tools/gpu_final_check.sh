set -u
mkdir -p gpurun_out/fc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -W ignore > gpurun_out/fc/tests.log 2>&1 || { tail -30 gpurun_out/fc/tests.log; exit 1; }
tail -1 gpurun_out/fc/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fc/smoke.log 2>&1 || { tail -20 gpurun_out/fc/smoke.log; exit 1; }
tail -1 gpurun_out/fc/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/fc/bench.log 2>&1 || { tail -20 gpurun_out/fc/bench.log; exit 1; }
tail -1 gpurun_out/fc/bench.log | cut -c1-400
