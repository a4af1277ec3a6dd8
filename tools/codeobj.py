"""Extract the gfx950 code objects a HIP shared library carries (its clang offload bundles) and
disassemble them, so that checks run on the machine code that actually ships
(tools/isa_exec_hazard.py, tests/test_isa_hazard.py).  roc-obj-ls needs a Perl module the image lacks.

    python tools/codeobj.py lib.so outdir      -> outdir/co<k>.o and outdir/co<k>.s per bundle
"""
import os
import struct
import subprocess
import sys

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def code_objects(path, arch="gfx950"):
    """[(triple, bytes)] of every code object for `arch` in the bundles of `path`."""
    data = open(path, "rb").read()
    out, pos = [], data.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + len(MAGIC))[0]
        q = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, q)
            triple = data[q + 24:q + 24 + tlen].decode()
            q += 24 + tlen
            if arch in triple and size:
                out.append((triple, data[pos + off:pos + off + size]))
        pos = data.find(MAGIC, pos + 1)
    return out


def disassemble(path, outdir, arch="gfx950"):
    """Write and disassemble every code object; returns the .s paths."""
    os.makedirs(outdir, exist_ok=True)
    files = []
    for k, (_, blob) in enumerate(code_objects(path, arch)):
        o = os.path.join(outdir, f"co{k}.o")
        with open(o, "wb") as f:
            f.write(blob)
        s = os.path.join(outdir, f"co{k}.s")
        with open(s, "w") as f:
            subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", "--no-leading-addr", "--symbolize-operands", o],
                           stdout=f, check=True)
        files.append(s)
    return files


if __name__ == "__main__":
    for s in disassemble(sys.argv[1], sys.argv[2]):
        print(s)
