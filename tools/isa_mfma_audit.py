"""Audit of MFMA operand hazards in the compiled gfx950 code (DESIGN.md
§14d, §15a).

Default: the product library as built.  The gfx950 code objects are taken
out of `avr_amd/libavr_hip.so`'s `.hip_fatbin` (one clang offload bundle per
translation unit), disassembled with llvm-objdump and scanned kernel by
kernel, within basic blocks (split at branches and at branch targets):

* WAR: after a `v_mfma_*`, an instruction within WINDOW wait states that
  writes a VGPR of the MFMA's SrcA or SrcB (a VALU result, an LDS or
  global load's return, another MFMA's D), with the wait states between
  them (an instruction counts 1, `s_nop N` counts N + 1).  The kind
  `WAR_after_mfma_B_behind_mfma` is the one that corrupted results on
  MI355X (§14d: the MFMA issued right behind another MFMA, its B register
  rewritten before the matrix pipe took it): the product must have none;
* RAW: before a `v_mfma_*`, the nearest VALU write of one of its SrcA/SrcB
  VGPRs within WINDOW states (the hardware needs one state, §14d);
* M0: every LDS-DMA load (`global_load_lds_*`, `buffer_load_* ... lds`) and
  every instruction naming m0 as a source must follow an m0 write in its
  own basic block (the inline-asm DMA wrappers set m0 themselves; a compiler
  value of m0 live across one of them would be clobbered).

    python tools/isa_mfma_audit.py                 # product library, JSON lines
    python tools/isa_mfma_audit.py --lib other.so
    python tools/isa_mfma_audit.py --asm file.s    # hipcc -save-temps output

tests/test_isa_audit.py runs `audit_library` in the CPU suite.
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import re
import struct
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "avr_amd", "libavr_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"
REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
BAD_KIND = "WAR_after_mfma_B_behind_mfma"


def regs(tok):
    out = set()
    for m in REG.finditer(tok):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def split_ops(text):
    ins = text.split(None, 1)
    if len(ins) == 1:
        return ins[0], []
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


def is_lds_dma(op, ops):
    return op.startswith("global_load_lds") or (
        op.startswith("buffer_load") and any("lds" in o.split() for o in ops))


def writes(op, ops):
    """VGPRs the instruction writes (its first operand for VALU / loads)."""
    if not ops:
        return set()
    if op.startswith(("v_", "ds_read", "global_load", "buffer_load", "flat_load", "scratch_load")) \
            and not op.startswith(("v_cmp", "v_readlane", "v_readfirstlane", "v_cmpx")) \
            and not is_lds_dma(op, ops):
        return regs(ops[0])
    return set()


def klass(op):
    if op.startswith("v_mfma") or op.startswith("v_smfmac"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_read"):
        return "lds_load"
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        return "vmem_load"
    return "other"


def _m0_write(op, ops):
    return bool(ops) and ops[0] == "m0"


def _m0_read(op, ops):
    return is_lds_dma(op, ops) or any(o == "m0" for o in ops[1:])


def audit_blocks(blocks, window=8):
    """blocks: iterable of (kernel, [(op, ops, text), ...]).  Returns
    {(kernel, kind, writer_class): {"min_states", "count", "example"}}."""
    findings = collections.defaultdict(lambda: {"min_states": 1 << 30, "count": 0, "example": None})

    def note(key, dist, example):
        f = findings[key]
        f["count"] += 1
        if dist < f["min_states"]:
            f["min_states"] = dist
            f["example"] = example

    for kernel, block in blocks:
        m0_set = False
        for i, (op, ops, line) in enumerate(block):
            if _m0_read(op, ops) and not m0_set:
                note((kernel, "M0_read_without_write_in_block", klass(op)), 0, [line])
            if _m0_write(op, ops):
                m0_set = True
            if klass(op) != "mfma" or len(ops) < 4:
                continue
            note((kernel, "MFMA_count", "mfma"), 0, [line])
            srcab = regs(ops[1]) | regs(ops[2])
            srcb = regs(ops[2])
            behind = i > 0 and klass(block[i - 1][0]) == "mfma"
            dist = 0
            for op2, ops2, line2 in block[i + 1:]:
                if dist >= window:
                    break
                w = writes(op2, ops2)
                if w & srcab:
                    kind = "WAR_after_mfma_B" if w & srcb else "WAR_after_mfma_A"
                    if behind and kind.endswith("B"):
                        kind += "_behind_mfma"
                    note((kernel, kind, klass(op2)), dist, [line, line2])
                dist += states(op2, ops2)
            dist = 0
            for op2, ops2, line2 in reversed(block[:i]):
                if dist >= window:
                    break
                if klass(op2) == "valu" and writes(op2, ops2) & srcab:
                    note((kernel, "RAW_before_mfma", "valu"), dist, [line2, line])
                    break
                dist += states(op2, ops2)
    return findings


# ---------------------------------------------------------------- objdump
_FUNC = re.compile(r"^[0-9a-f]+ <(.+)>:$")
_TARGET = re.compile(r"<(.+)\+0x([0-9a-f]+)>\s*$")
_ADDR = re.compile(r"//\s*([0-9A-Fa-f]+):")


def _objdump_blocks(code_object):
    """Basic blocks of every function of a disassembled gfx950 code object."""
    txt = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", "--no-show-raw-insn",
                          code_object], check=True, capture_output=True, text=True).stdout
    funcs = []  # (name, base, [(addr, op, ops, text, target)])
    for raw in txt.splitlines():
        m = _FUNC.match(raw.strip())
        if m:
            funcs.append((m.group(1), None, []))
            continue
        if not raw.startswith("\t") or not funcs:
            continue
        body, _, comment = raw.strip().partition("//")
        body = body.strip()
        if not body:
            continue
        am = _ADDR.search(raw)
        addr = int(am.group(1), 16) if am else None
        tm = _TARGET.search(comment)
        target = (tm.group(1), int(tm.group(2), 16)) if tm else None
        op, ops = split_ops(body)
        name, base, ins = funcs[-1]
        if base is None and addr is not None:
            funcs[-1] = (name, addr, ins)
        ins.append((addr, op, ops, body, target))
    for name, base, ins in funcs:
        starts = {off for (_a, op, _o, _t, tgt) in ins if tgt and tgt[0] == name and op.startswith("s_") and
                  ("branch" in op) for off in [tgt[1]]}
        block = []
        for addr, op, ops, text, tgt in ins:
            if base is not None and addr is not None and (addr - base) in starts and block:
                yield name, block
                block = []
            block.append((op, ops, text))
            if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_endpgm", "s_swappc")):
                yield name, block
                block = []
        if block:
            yield name, block


def code_objects(lib, outdir):
    """gfx950 code objects of the library's offload bundles (one per
    translation unit, each 4096-byte aligned in .hip_fatbin; compressed
    'CCOB' bundles, hipcc --offload-compress, are unpacked by
    clang-offload-bundler), written to outdir; returns their paths."""
    fat = os.path.join(outdir, "fatbin.bin")
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", f".hip_fatbin={fat}", lib,
                    os.path.join(outdir, "stripped.so")], check=True, capture_output=True)
    data = open(fat, "rb").read()
    starts = [i for i in range(0, len(data), 4096)
              if data[i:i + 4] == b"CCOB" or data[i:i + len(BUNDLE_MAGIC)] == BUNDLE_MAGIC]
    paths = []
    for k, i in enumerate(starts):
        end = starts[k + 1] if k + 1 < len(starts) else len(data)
        out = os.path.join(outdir, f"co{len(paths)}.o")
        if data[i:i + 4] == b"CCOB":
            # header: magic, version (u16), method (u16), then the bundle's
            # total size (u32 in version 2, u64 from version 3)
            (ver,) = struct.unpack_from("<H", data, i + 4)
            (total,) = struct.unpack_from("<Q" if ver >= 3 else "<I", data, i + 8)
            blob = os.path.join(outdir, f"bundle{k}.bin")
            with open(blob, "wb") as f:
                f.write(data[i:min(end, i + total)])
            subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--type=o", "--unbundle",
                            f"--input={blob}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={out}"],
                           check=True, capture_output=True)
            paths.append(out)
            continue
        (n,) = struct.unpack_from("<Q", data, i + 24)
        o = i + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, o)
            o += 24
            triple = data[o:o + tlen].decode()
            o += tlen
            if triple.endswith("gfx950"):
                with open(out, "wb") as f:
                    f.write(data[i + off:i + off + size])
                paths.append(out)
    return paths


def audit_library(lib=LIB, window=8):
    """Findings over every kernel of the library (see audit_blocks)."""
    with tempfile.TemporaryDirectory(prefix="avr_isa_") as tmp:
        found = {}
        for co in code_objects(lib, tmp):
            found.update(audit_blocks(_objdump_blocks(co), window))
        return found


def _asm_blocks(path):
    kernel, block = None, []
    for raw in open(path):
        s = raw.split(";")[0].strip()
        if not s:
            continue
        if s.endswith(":") and not s.startswith("."):
            if block:
                yield kernel, block
            block = []
            if not s.startswith(".L"):
                kernel = s[:-1]
            continue
        if s.startswith("."):
            if (s.startswith(".LBB") or s.startswith(".Lfunc_end")) and block:
                yield kernel, block
                block = []
            continue
        op, ops = split_ops(s)
        block.append((op, ops, s))
        if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_endpgm")):
            yield kernel, block
            block = []
    if block:
        yield kernel, block


def _demangle(names):
    try:
        out = subprocess.run([os.path.join(LLVM, "llvm-cxxfilt")], input="\n".join(names), capture_output=True,
                             text=True, check=True).stdout.splitlines()
        return dict(zip(names, out))
    except (OSError, subprocess.CalledProcessError):
        return {n: n for n in names}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=LIB)
    ap.add_argument("--window", type=int, default=8)
    ap.add_argument("--asm", nargs="*", default=[], help="audit these assembly files instead")
    a = ap.parse_args()
    if a.asm:
        found = {}
        for path in a.asm:
            found.update(audit_blocks(_asm_blocks(path), a.window))
    else:
        found = audit_library(a.lib, a.window)
    names = _demangle(sorted({k[0] for k in found}))
    for (kern, kind, cls), f in sorted(found.items()):
        print(json.dumps({"kernel": names.get(kern, kern)[:90], "kind": kind, "writer": cls, "pairs": f["count"],
                          "min_wait_states": f["min_states"], "example": f["example"]}))


if __name__ == "__main__":
    main()
