"""CPU: the C-ABI library builds, loads, and exports every declared symbol.

No compute calls here (no GPU in the build container)."""
import os
import re
import subprocess

import pytest

from avr_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "avr_hip.h")


def _declared():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    # the shapes build's experiments are not part of the product library
    text = re.sub(r"#ifdef AVR_SHAPE_PROBES.*?#endif", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(avr_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(ROOT, "avr_amd", "csrc"), "-j8"], check=True)
    return _lib.load()


def test_header_declares_expected_entry_points():
    names = _declared()
    for n in ("avr_ray_reduce_fwd", "avr_dft_phase_fwd", "avr_weights_fwd", "avr_irfft",
              "avr_hashgrid_fwd", "avr_hashgrid_bwd", "avr_last_error"):
        assert n in names


def test_every_declared_symbol_is_exported(lib):
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_header():
    assert set(_declared()) == set(_lib.EXPORTS)


def test_abi_version(lib):
    assert lib.avr_abi_version() == 2


def test_argument_errors_are_reported_without_gpu(lib):
    # null params -> AVR_E_ARG with a message; no device work is launched
    rc = lib.avr_tables(None, None, None, None, None, None, None, None)
    assert rc == 1001
    assert b"null" in lib.avr_last_error()
    # a graph launch without an instantiated graph is refused before any HIP call
    assert lib.avr_graph_launch(None, None) == 1001
    assert b"avr_graph_launch" in lib.avr_last_error()


def test_code_object_targets_gfx950(lib):
    """Every HIP translation unit's (compressed) offload bundle holds a gfx950
    code object (unbundled for that target by clang-offload-bundler)."""
    import sys
    import tempfile

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_mfma_audit

    if not os.path.exists(os.path.join(isa_mfma_audit.LLVM, "clang-offload-bundler")):
        pytest.skip("needs ROCm's clang-offload-bundler")
    hips = [f for f in os.listdir(os.path.join(ROOT, "avr_amd", "csrc")) if f.endswith(".hip")]
    srcs = open(os.path.join(ROOT, "avr_amd", "csrc", "Makefile")).read().split("SRCS    :=")[1].split("\n")[0]
    shipped = [f for f in hips if f in srcs.split()]
    with tempfile.TemporaryDirectory() as tmp:
        cos = isa_mfma_audit.code_objects(_lib.LIB_PATH, tmp)
        assert len(cos) == len(shipped), (len(cos), shipped)
        for co in cos:
            assert open(co, "rb").read(4) == b"\x7fELF"


def test_only_validated_knobs_read_the_environment():
    """The shipped library reads exactly two environment variables, both
    validated tuning knobs (tests/test_gpu_knobs.py renders the golden vectors
    under every value); no debug or experiment switch can change results."""
    csrc = os.path.join(ROOT, "avr_amd", "csrc")
    names = set()
    for f in os.listdir(csrc):
        if f.endswith((".hip", ".cpp", ".h")):
            names |= set(re.findall(r'getenv\("([A-Z_0-9]+)"\)', open(os.path.join(csrc, f)).read()))
    assert names == {"AVR_NSPLIT", "AVR_KSPLIT"}, names
