"""CPU: the compiled gfx950 code of the product library, audited for the
MFMA operand pattern that returned wrong results on MI355X (DESIGN.md §14d,
§15a) and for the m0 protocol of the inline-asm LDS-DMA loads.

tools/isa_mfma_audit.py takes the gfx950 code objects out of
avr_amd/libavr_hip.so as built, disassembles them and scans every kernel
within basic blocks.  The product must have:

* no register that an MFMA issued right behind another MFMA reads as SrcB
  rewritten (VALU result, LDS or global load return, MFMA destination)
  within 8 wait states after it;
* at least one wait state between a VALU write of an MFMA's SrcA/SrcB and
  the MFMA (the hardware probe's requirement; hipcc pads two);
* an m0 write in the basic block before every LDS-DMA load and every
  instruction reading m0 (the inline-asm DMA wrappers set m0 themselves,
  so no compiler value of m0 is live across one).
"""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import isa_mfma_audit as audit  # noqa: E402

pytestmark = pytest.mark.skipif(
    not (os.path.exists(audit.LIB) and shutil.which(os.path.join(audit.LLVM, "llvm-objdump"))),
    reason="needs the built library and ROCm's llvm-objdump")


@pytest.fixture(scope="module")
def findings():
    return audit.audit_library()


def _where(found, pred):
    return {f"{k[0][:80]} {k[1]} {k[2]}": v["example"] for k, v in found.items() if pred(k, v)}


def test_library_has_mfma_kernels(findings):
    # the scan saw the MFMA kernels
    kernels = {k[0] for k in findings if k[1] == "MFMA_count"}
    assert any("head_exact_kernel" in k for k in kernels)
    assert any("sigma_meshrir_h1_kernel" in k for k in kernels)
    assert any("dft_phase_fwd_kernel" in k for k in kernels)


def test_no_b_operand_rewrite_behind_a_queued_mfma(findings):
    bad = _where(findings, lambda k, v: k[1] == audit.BAD_KIND)
    assert not bad, bad


def test_valu_writes_of_mfma_operands_are_padded(findings):
    bad = _where(findings, lambda k, v: k[1] == "RAW_before_mfma" and v["min_states"] < 1)
    assert not bad, bad


def test_m0_is_set_before_every_reader(findings):
    bad = _where(findings, lambda k, v: k[1].startswith("M0_"))
    assert not bad, bad


def test_audit_flags_the_pattern():
    """The scanner itself: the round-5 bf16x3 DFT's sequence is flagged, the
    same sequence with 8 wait states (or a VALU write of SrcA) is not."""
    def ins(text):
        op, ops = audit.split_ops(text)
        return op, ops, text
    seq = [ins("v_mfma_f32_32x32x16_bf16 a[0:15], v[74:77], v[66:69], a[0:15]"),
           ins("v_mfma_f32_32x32x16_bf16 a[16:31], v[74:77], v[70:73], a[16:31]"),
           ins("v_perm_b32 v70, v1, v2, v3")]
    found = audit.audit_blocks([("k", seq)])
    assert ("k", audit.BAD_KIND, "valu") in found
    padded = seq[:2] + [ins("s_nop 7")] + seq[2:]
    assert ("k", audit.BAD_KIND, "valu") not in audit.audit_blocks([("k", padded)])
    a_only = seq[:2] + [ins("v_perm_b32 v74, v1, v2, v3")]
    assert ("k", audit.BAD_KIND, "valu") not in audit.audit_blocks([("k", a_only)])
    dma = [ins("global_load_lds_dwordx4 v[2:3], off")]
    assert ("k", "M0_read_without_write_in_block", "vmem_load") in audit.audit_blocks([("k", dma)])
    assert not audit.audit_blocks([("k", [ins("s_mov_b32 m0, s4")] + dma)])
