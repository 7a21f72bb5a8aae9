"""Audit of MFMA operand hazards in the shipped kernels' compiled code
(round-5 task 4).

Compiles each HIP source of the library with -save-temps (the product
flags) and scans the gfx950 assembly of every kernel, within basic blocks:

* WAR: after a `v_mfma_*`, any instruction within WINDOW wait states that
  writes a VGPR of the MFMA's SrcA or SrcB (a VALU result, an LDS or
  global load's return, another MFMA's D), with the number of wait states
  between them (an instruction counts 1, `s_nop N` counts N + 1);
* RAW: before a `v_mfma_*`, a VALU write of one of its SrcA/SrcB VGPRs
  within WINDOW states, and the states between.

The hazard probe (tools/hazard_probe.hip) measures on the hardware which of
these distances are safe; this script lists where the compiled code comes
close.  Output: one JSON line per (source, kind, instruction class) with the
minimum distance seen and an example.

    python tools/isa_mfma_audit.py [--window 8] [sources ...]
"""
from __future__ import annotations

import argparse
import collections
import glob
import json
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "avr_amd", "csrc")
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-ffp-contract=off", "-fno-gpu-rdc",
         "-Wno-unused-function", "-Wno-inline-asm", "-I" + os.path.join(ROOT, "include")]
REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(tok):
    out = set()
    for m in REG.finditer(tok):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def split_ops(line):
    ins = line.split(None, 1)
    if len(ins) == 1:
        return ins[0], []
    # operands separated by commas outside brackets
    ops, depth, cur = [], 0, ""
    for ch in ins[1]:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            ops.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        ops.append(cur.strip())
    return ins[0], ops


def states(op, ops):
    if op == "s_nop":
        try:
            return int(ops[0], 0) + 1
        except (ValueError, IndexError):
            return 1
    return 1


def writes(op, ops):
    """VGPRs the instruction writes (its first operand for VALU / loads)."""
    if not ops:
        return set()
    if op.startswith(("v_", "ds_read", "global_load", "buffer_load", "flat_load", "scratch_load")) \
            and not op.startswith(("v_cmp", "v_readlane", "v_readfirstlane")) and "_lds" not in op:
        return regs(ops[0])
    return set()


def klass(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_read"):
        return "lds_load"
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        return "vmem_load"
    return "other"


def audit_asm(path, window):
    findings = collections.defaultdict(lambda: {"min_states": 1 << 30, "count": 0, "example": None})
    kernel = None
    block = []

    def flush():
        for i, (op, ops, line) in enumerate(block):
            if not op.startswith("v_mfma") or len(ops) < 4:
                continue
            srcab = regs(ops[1]) | regs(ops[2])
            srcb = regs(ops[2])
            # the MFMA issued right behind another one (the matrix pipe busy:
            # it may wait to start while later instructions issue)
            behind = i > 0 and block[i - 1][0].startswith("v_mfma")
            # WAR: later writers of SrcA/B (SrcB separately: the bf16x3 DFT's
            # stale bins were B-operand lanes, §14d)
            dist = 0
            for op2, ops2, line2 in block[i + 1:]:
                if dist >= window:
                    break
                w = writes(op2, ops2)
                if w & srcab:
                    kind = "WAR_after_mfma_B" if w & srcb else "WAR_after_mfma_A"
                    if behind and kind.endswith("B"):
                        kind += "_behind_mfma"
                    key = (kernel, kind, klass(op2))
                    f = findings[key]
                    f["count"] += 1
                    if dist < f["min_states"]:
                        f["min_states"] = dist
                        f["example"] = [line.strip(), line2.strip()]
                dist += states(op2, ops2)
            # RAW: earlier VALU writers of SrcA/B
            dist = 0
            for op2, ops2, line2 in reversed(block[:i]):
                if dist >= window:
                    break
                if klass(op2) == "valu" and writes(op2, ops2) & srcab:
                    key = (kernel, "RAW_before_mfma", "valu")
                    f = findings[key]
                    f["count"] += 1
                    if dist < f["min_states"]:
                        f["min_states"] = dist
                        f["example"] = [line2.strip(), line.strip()]
                    break
                dist += states(op2, ops2)
        block.clear()

    for raw in open(path):
        line = raw.split(";")[0].rstrip()
        if not line.strip():
            continue
        s = line.strip()
        if s.endswith(":") and not s.startswith("."):
            flush()
            if not s.startswith(".L"):
                kernel = s[:-1]
            continue
        if s.startswith(".") or s.startswith(";"):
            if s.startswith(".LBB") or s.startswith(".Lfunc_end"):
                flush()
            continue
        op, ops = split_ops(s)
        block.append((op, ops, s))
        if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_endpgm")):
            flush()
    flush()
    return findings


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sources", nargs="*")
    ap.add_argument("--window", type=int, default=8)
    ap.add_argument("--asm", nargs="*", default=[], help="audit these assembly files instead")
    a = ap.parse_args()
    for path in a.asm:
        for (kern, kind, cls), f in sorted(audit_asm(path, a.window).items()):
            print(json.dumps({"asm": os.path.basename(path), "kernel": kern[:60], "kind": kind, "writer": cls,
                              "pairs": f["count"], "min_wait_states": f["min_states"], "example": f["example"]}))
    if a.asm:
        return
    srcs = a.sources or sorted(os.path.basename(p) for p in glob.glob(os.path.join(CSRC, "*.hip")))
    tmp = tempfile.mkdtemp(prefix="avr_isa_")
    for src in srcs:
        subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, "--save-temps", "-c", os.path.join(CSRC, src), "-o",
                        os.path.join(tmp, src + ".o")], cwd=tmp, check=True, capture_output=True)
        asm = glob.glob(os.path.join(tmp, os.path.splitext(src)[0] + "-hip-amdgcn-amd-amdhsa-gfx950.s"))
        if not asm:
            continue
        found = audit_asm(asm[0], a.window)
        per = collections.defaultdict(lambda: {"min_states": 1 << 30, "count": 0, "example": None, "kernels": 0})
        for (kern, kind, cls), f in found.items():
            g = per[(kind, cls)]
            g["count"] += f["count"]
            g["kernels"] += 1
            if f["min_states"] < g["min_states"]:
                g["min_states"], g["example"] = f["min_states"], f["example"]
        for (kind, cls), g in sorted(per.items()):
            print(json.dumps({"source": src, "kind": kind, "writer": cls, "pairs": g["count"],
                              "kernels": g["kernels"], "min_wait_states": g["min_states"],
                              "example": g["example"]}), flush=True)


if __name__ == "__main__":
    main()
