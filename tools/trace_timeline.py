"""Print the kernel timeline of the last N ray-reduction launches of a
rocprofv3 --kernel-trace CSV (gaps between the render kernels)."""
import csv
import sys


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0].split("<")[0][:30]


def main(path, n=20, key="ray_reduce_fwd"):
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"])
                for r in rows)
    red = [i for i, k in enumerate(ks) if key in k[2]]
    last = red[-n:]
    i0 = max(0, last[0] - 3)
    t0 = ks[i0][0]
    for k in ks[i0:last[-1] + 6]:
        print(f"{(k[0] - t0) / 1e3:9.2f} {(k[1] - t0) / 1e3:9.2f} {(k[1] - k[0]) / 1e3:7.2f} q{k[3]} {k[2]}")
    span = (ks[min(len(ks) - 1, last[-1] + 4)][1] - ks[max(0, last[0] - 2)][0]) / 1e3
    print("span us", span, "per step", span / n)
    print("reduce avg us", sum(ks[i][1] - ks[i][0] for i in last) / n / 1e3)
    starts = [ks[i][0] for i in last]
    print("reduce start-to-start avg us", (starts[-1] - starts[0]) / (n - 1) / 1e3)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
