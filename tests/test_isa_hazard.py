"""The shipped machine code is free of the code-generation hazard that broke the round-4 SRB-12 variant
builds ("Root cause of the round-4 variant failures").

The build without amdgpu_waves_per_eu(1, 1) placed the reload of the output loop's index `v` (kept in an
AGPR since the kernel's start) in the flow block that ends the polish's `if (!accepted)` restore, ahead of
the `s_or_b64 exec` that restores the mask -- a mask the register allocator had spilled to VGPR lanes.  With
the polish accepted the block runs under an empty mask, no lane receives `v`, and every lane then stores its
output to the same address: the solution vector came back as zeros with one entry in 64 set.
tools/isa_exec_hazard.py finds that pattern; the fixture is that kernel's disassembly.

A second guard (round 6): no shipped kernel carries a FLAT (generic-address) memory
instruction.  Round 5's first lip_eq_res read x0 (global) or the LDS iterate through one pointer, which the
compiler turned into flat loads; that build rejected the polish of 243 of 512 agents.
The fixture is that build's solve and polish kernels of the instance the failing test ran
(12_3_1_0_0_0, `make lipvar TAG=flat LIPFLAGS=-DSRB_DIAG_FLAT_EQRES`, llvm-objdump with the encodings dropped)."""
import gzip
import os
import sys

import pytest
from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import codeobj  # noqa: E402
import isa_exec_hazard as hz  # noqa: E402

FIXTURE = os.path.join(ROOT, "tests", "golden", "isa", "r04_srb12_2_4_20_12_nowpe.s.gz")
FLAT_FIXTURE = os.path.join(ROOT, "tests", "golden", "isa", "r05_lip_12_3_1_flat_eqres.s.gz")


def test_scanner_finds_the_round4_variant_failure():
    """The failing build's kernel: exactly the two halves of the reloaded 64-bit index are flagged."""
    lines = gzip.open(FIXTURE, "rt").read().splitlines()
    found = [(name, hz.scan(body)) for name, body in hz.kernels(lines)]
    assert len(found) == 1 and found[0][0] == "srb12_kernel_2_4_20_12"
    hits = found[0][1]
    assert sorted(t for _, t, _ in hits) == ["v_accvgpr_read_b32 v200, a36", "v_accvgpr_read_b32 v201, a37"], hits


def test_scanner_finds_the_round5_flat_access():
    """The generic-pointer build: two flat_load_dwordx4 (x0 or xs[4 (k - 1)], four doubles) in each kernel,
    and no exec-mask reload hazard -- the flat accesses are what distinguishes it from the product."""
    lines = gzip.open(FLAT_FIXTURE, "rt").read().splitlines()
    found = {name: (hz.scan(body), hz.flat_mem(body)) for name, body in hz.kernels(lines)}
    assert sorted(found) == ["srb_nmpc_kernel_12_3_1_0_0_0", "srb_polish_kernel_12_3_1_0_0_0"], sorted(found)
    for name, (haz, fl) in found.items():
        assert not haz, (name, haz)
        assert [t.split()[0] for _, t in fl] == ["flat_load_dwordx4"] * 2, (name, fl)


@pytest.fixture(scope="module")
def shipped_kernels(tmp_path_factory):
    import srbnmpc
    if os.path.basename(srbnmpc.LIB_PATH) != "libsrbnmpc.so":
        pytest.skip("a diagnostic build is selected")
    files = codeobj.disassemble(srbnmpc.LIB_PATH, str(tmp_path_factory.mktemp("co")))
    assert len(files) >= 4, files
    out = []
    for f in files:
        with open(f) as fh:
            out += list(hz.kernels(fh))
    assert len(out) >= 30, len(out)
    return out


def test_shipped_library_has_no_flat_memory_instruction(shipped_kernels):
    """Every global access of the product kernels is a global_/buffer_ instruction and every LDS access a
    ds_ one: no generic pointer reaches a load or store (srb_llctrl.hip's tau read was one until round 6)."""
    hits = [(name, t) for name, body in shipped_kernels for _, t in hz.flat_mem(body)]
    assert not hits, hits


def test_shipped_library_has_no_exec_mask_reload_hazard(shipped_kernels):
    """Every kernel of the product library (all gfx950 code objects it carries), disassembled from the
    built .so itself."""
    hits = [(name, t) for name, body in shipped_kernels for _, t, _ in hz.scan(body)]
    assert not hits, hits
