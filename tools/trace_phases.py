"""Per-phase statistics of the ray-reduction launches in a rocprofv3
--kernel-trace of `bench.py --gpus 1 --steps 20 --warmup 5` (pose mode): the
bench runs, in order, W eager warmup poses, 20 eager serial-latency poses,
graph captures (+2 side-stream warmups), the graph serial-latency replays,
the roofline phase (K eager poses on one stream, HIP events around each
reduction), graph warmups, K eager and K graph-replayed pipelined poses.
The phases are told apart by queue and launch spacing; the roofline phase
is the run of K launches on one queue after the graph latency phase.

    python tools/trace_phases.py run_kernel_trace.csv [K] > summary.json
"""
import csv
import json
import statistics
import sys


def main(path, k=20):
    rows = list(csv.DictReader(open(path)))
    red = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"])
                 for r in rows if "ray_reduce_fwd" in r["Kernel_Name"])
    dur = [(e - s) / 1e3 for s, e, _ in red]
    # the pipelined phases are the last 2K launches (eager, then graph);
    # before them come the graph warmups, and before those the roofline
    # phase: the K launches preceding the first launch on a third queue
    # after the captures (the warmups start a new graph ring per stream)
    n = len(red)
    graph_pipe = list(range(n - k, n))
    eager_pipe = list(range(n - 2 * k, n - k))
    # roofline: the last run of K consecutive launches on one queue whose
    # spacing is above their duration (no overlap) before eager_pipe
    i = n - 2 * k - 1
    while i >= k:
        win = list(range(i - k + 1, i + 1))
        qs = {red[j][2] for j in win}
        overlap = any(red[j + 1][0] < red[j][1] for j in win[:-1])
        if len(qs) == 1 and not overlap:
            break
        i -= 1
    roof = list(range(i - k + 1, i + 1))

    def stats(ix):
        d = [dur[j] for j in ix]
        span = (red[ix[-1]][1] - red[ix[0]][0]) / 1e3
        return {"launches": len(ix), "first_index": ix[0], "avg_us": statistics.mean(d),
                "median_us": statistics.median(d), "min_us": min(d), "max_us": max(d),
                "span_us_per_launch": span / len(ix)}

    print(json.dumps({"trace": path, "kernel": "ray_reduce_fwd_kernel", "all_launches": n,
                      "all_avg_us": statistics.mean(dur),
                      "roofline_phase": stats(roof), "pipelined_eager": stats(eager_pipe),
                      "pipelined_graph": stats(graph_pipe)}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
