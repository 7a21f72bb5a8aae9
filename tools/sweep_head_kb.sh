set -u
export TMPDIR=/tmp
for wl in c2_meshrir_1024x256x512 c3_raf_furnished_b4; do
for kb in 8 16; do for sb in 1 2 4; do
  d=gpurun_out/shk_${wl}_k${kb}_s${sb}
  AVR_HEAD_KB=$kb AVR_HEAD_SB=$sb timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- \
    python tools/probe_head.py --workload $wl --dbg 0 --iters 5 > $d.log 2>&1 || exit 1
done; done; done
