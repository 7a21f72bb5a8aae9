"""Does a TunableOp results file take effect for a plain bf16 mm at run time?
python tools/tunable_probe.py FILE"""
import sys

import torch
import torch.cuda.tunable as tun

dev = torch.device("cuda", 0)
N = 83200
g = torch.randn(N, 128, device=dev).bfloat16()
w = torch.randn(128, 80, device=dev).bfloat16()


def t(fn, it=50):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / it


print("default", t(lambda: g @ w))
tun.tuning_enable(False)
tun.record_untuned_enable(False)
tun.enable(True)
ok = tun.read_file(sys.argv[1])
res = tun.get_results()
print("read", ok, len(res), [r for r in res if r[1].startswith("nn_80_83200")])
print("tuned", t(lambda: g @ w))
print("validators", tun.get_validators())
