"""Time the hash-grid forward (row-major vs level-major output) on the
config-2 ray points (MeshRIR position grid: 20 levels, 2^18, base 16)."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avr_amd import AVRRender  # noqa: E402
from avr_amd.encoding import HashGridEncoding  # noqa: E402
from avr_amd.workloads import MESHRIR_MODEL, WORKLOADS  # noqa: E402


class _Null(torch.nn.Module):
    def forward(self, *a, **k):
        raise RuntimeError


def main():
    dev = torch.device("cuda", 0)
    w = WORKLOADS["c2_meshrir_1024x256x512"]
    r = AVRRender(_Null(), **w.render)
    pts = r.sample(torch.rand(1, 3, device=dev) * 4 - 2, torch.rand(1, 3, device=dev) * 4 - 2)[0]
    x = ((pts.reshape(-1, 3) + 1) / 2).contiguous()
    for dt in (torch.float16, torch.float32):
        enc = HashGridEncoding(3, MESHRIR_MODEL["pos_encoding_sigma"], dtype=dt).to(dev)
        with torch.no_grad():
            enc.params.uniform_(-1, 1)
            a = enc(x)
            b = enc.forward_level_major(x)
            same = bool(torch.equal(a, b.permute(1, 0, 2).reshape(a.shape)))
            res = {"dtype": str(dt), "n": x.size(0), "level_major_equal": same}
            for name, fn in (("row_major", lambda: enc(x)), ("level_major", lambda: enc.forward_level_major(x))):
                for _ in range(3):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res[name + "_us"] = e0.elapsed_time(e1) * 1e3 / 20
        print(json.dumps(res))


if __name__ == "__main__":
    main()
