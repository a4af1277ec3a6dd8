"""The shipped machine code is free of the code-generation hazard that broke the round-4 SRB-12 variant
builds ("Root cause of the round-4 variant failures").

The build without amdgpu_waves_per_eu(1, 1) placed the reload of the output loop's index `v` (kept in an
AGPR since the kernel's start) in the flow block that ends the polish's `if (!accepted)` restore, ahead of
the `s_or_b64 exec` that restores the mask -- a mask the register allocator had spilled to VGPR lanes.  With
the polish accepted the block runs under an empty mask, no lane receives `v`, and every lane then stores its
output to the same address: the solution vector came back as zeros with one entry in 64 set.
tools/isa_exec_hazard.py finds that pattern; the fixture is that kernel's disassembly."""
import gzip
import os
import sys

import pytest
from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import codeobj  # noqa: E402
import isa_exec_hazard as hz  # noqa: E402

FIXTURE = os.path.join(ROOT, "tests", "golden", "isa", "r04_srb12_2_4_20_12_nowpe.s.gz")


def test_scanner_finds_the_round4_variant_failure():
    """The failing build's kernel: exactly the two halves of the reloaded 64-bit index are flagged."""
    lines = gzip.open(FIXTURE, "rt").read().splitlines()
    found = [(name, hz.scan(body)) for name, body in hz.kernels(lines)]
    assert len(found) == 1 and found[0][0] == "srb12_kernel_2_4_20_12"
    hits = found[0][1]
    assert sorted(t for _, t, _ in hits) == ["v_accvgpr_read_b32 v200, a36", "v_accvgpr_read_b32 v201, a37"], hits


def test_shipped_library_has_no_exec_mask_reload_hazard(tmp_path):
    """Every kernel of the product library (all gfx950 code objects it carries), disassembled from the
    built .so itself."""
    import srbnmpc
    if os.path.basename(srbnmpc.LIB_PATH) != "libsrbnmpc.so":
        pytest.skip("a diagnostic build is selected")
    files = codeobj.disassemble(srbnmpc.LIB_PATH, str(tmp_path))
    assert len(files) >= 4, files
    kernels, hits = 0, []
    for f in files:
        with open(f) as fh:
            for name, body in hz.kernels(fh):
                kernels += 1
                hits += [(name, t) for _, t, _ in hz.scan(body)]
    assert kernels >= 30, kernels
    assert not hits, hits
