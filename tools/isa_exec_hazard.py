"""Scan gfx950 kernel assembly for the code-generation hazard behind the round-4 SRB-12 variant failures
("The variant builds' wrong answers"): a spill reload or register copy
(v_accvgpr_read / v_accvgpr_write / v_mov / scratch_load) placed in the flow block that ends a divergent
region -- after the label a `s_cbranch_execz` jumps to, before the `s_or_b64 exec, exec, ...` that restores
the mask -- whose destination is read after the restore.  Such a copy runs under the region's (possibly
empty) exec mask, so the lanes outside the region keep a stale value; the round-4 build without
amdgpu_waves_per_eu(1, 1) put the reload of the output index `v` there, and every lane then stored its
result to the same address.  The scan is linear (no control-flow graph): it reports candidates, and a
clean report for a kernel means no copy sits in such a position.

    python tools/isa_exec_hazard.py file.s [kernel-name-substring ...]
    (file.s: hipcc --cuda-device-only -S output, or llvm-objdump -d of the code object)
"""
import re
import sys

COPY_OPS = ("v_accvgpr_read_b32", "v_accvgpr_write_b32", "v_mov_b32_e32", "v_mov_b64_e32", "scratch_load_dword",
            "scratch_load_dwordx2", "scratch_load_dwordx4", "buffer_load_dword")
SPILLED_ONLY = True
RELOAD_OPS = ("v_accvgpr_read_b32", "scratch_load_dword", "scratch_load_dwordx2", "scratch_load_dwordx4")
REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)(?!\d))")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        k = m.group(1)
        if m.group(2):
            out.update((k, i) for i in range(int(m.group(2)), int(m.group(3)) + 1))
        else:
            out.add((k, int(m.group(4))))
    return out


def split_operands(line):
    body = line.split(";")[0].strip()
    parts = body.split(None, 1)
    if len(parts) < 2:
        return parts[0] if parts else "", "", ""
    op, rest = parts
    ops = [o.strip() for o in rest.split(",")]
    return op, ops[0], ",".join(ops[1:])


def normalize(ln):
    """llvm-objdump -d --symbolize-operands lines into the assembler form the scan reads: `<name>:` kernel
    labels, `<L12>:` block labels and `L12` branch targets; `//` comments (address, encoding) dropped."""
    ln = ln.split("//")[0].rstrip()
    m = re.match(r"^<(L\d+)>:", ln)
    if m:
        return f".LBB{m.group(1)}:"
    m = re.match(r"^<([A-Za-z_][\w.]*)>:", ln)
    if m:
        return f"{m.group(1)}:"
    return re.sub(r"\b(s_c?branch\w*)\s+(L\d+)\b", r"\1 .LBB\2", ln)


def kernels(lines):
    name, body = None, []
    for ln in lines:
        ln = normalize(ln)
        m = re.match(r"^([A-Za-z_][\w.]*):\s*(;.*)?$", ln)
        if m and not ln.startswith(".") and not m.group(1).startswith(".L"):
            if name and body:
                yield name, body
            name, body = m.group(1), []
        elif name is not None:
            body.append(ln.rstrip("\n"))
            if "s_endpgm" in ln:
                yield name, body
                name, body = None, []


def region_open(body, i):
    """Line that saved the mask the restore at line i puts back (the region's opening), following an SGPR
    spill of the saved mask through v_writelane / v_readlane; -1 if not found."""
    m = re.match(r"^\s*s_or_b64\s+exec,\s*exec,\s*s\[(\d+):(\d+)\]", body[i])
    if not m:
        return -1
    lo = int(m.group(1))
    lane = None
    for t in body[max(i - 6, 0):i]:                      # reloaded from VGPR lanes just before the restore?
        r = re.match(r"^\s*v_readlane_b32\s+s(\d+),\s*v(\d+),\s*(\d+)", t)
        if r and int(r.group(1)) == lo:
            lane = (int(r.group(2)), int(r.group(3)))
    k = i - 1
    if lane:
        while k >= 0 and not re.match(rf"^\s*v_writelane_b32\s+v{lane[0]},\s*s(\d+),\s*{lane[1]}\b", body[k]):
            k -= 1
        if k < 0:
            return -1
        lo = int(re.match(r"^\s*v_writelane_b32\s+v\d+,\s*s(\d+)", body[k]).group(1))
    while k >= 0:
        t = body[k]
        if re.match(rf"^\s*s_(and_saveexec_b64|or_saveexec_b64|andn2_saveexec_b64|mov_b64)\s+s\[{lo}:{lo + 1}\],\s*(exec|s\[|vcc)", t):
            return k
        k -= 1
    return -1


def scan(body):
    """(line index, copy line, register) for every hazardous copy in one kernel body."""
    execz_targets = set(re.findall(r"s_cbranch_execz\s+(\.LBB\w+)", "\n".join(body)))
    labels = {m.group(1): k for k, ln in enumerate(body) for m in [re.match(r"^(\.LBB\w+):", ln)] if m}
    found = []
    for i, ln in enumerate(body):
        if not re.match(r"^\s*s_or_b64\s+exec,\s*exec,", ln):
            continue
        # walk back over the flow block(s) to the last label that is an execz target; stop at any other
        # exec change or branch (the window then runs under the inner mask)
        j, window, hit = i - 1, [], False
        while j >= 0:
            t = body[j]
            lab = re.match(r"^(\.LBB\w+):", t)
            if lab:
                hit = hit or lab.group(1) in execz_targets     # flow blocks chain: keep walking back
                j -= 1
                continue
            s = t.strip()
            if s.startswith(";") or not s:
                j -= 1
                continue
            if "exec" in s.split(";")[0] or s.startswith(("s_branch", "s_cbranch", "s_setpc")):
                break
            window.append((j, t))
            j -= 1
        if not hit:
            continue
        r0 = region_open(body, i)
        if r0 < 0:
            continue
        # the trigger: the region's saved exec mask was spilled (an SGPR spill to VGPR lanes, read back just
        # before the restore) -- the register allocator then places a join-block reload ahead of the restore
        spilled = any(re.match(r"^\s*v_readlane_b32\s+s\d+,", t) for t in body[max(i - 6, 0):i])
        if SPILLED_ONLY and not spilled:
            continue
        for k, t in window:
            op, dst, src = split_operands(t)
            if op not in RELOAD_OPS:
                continue
            # a reload of a value last written BEFORE the region (a long-lived spill): under the region's mask
            # the lanes outside the region never receive it
            slot = re.search(r"offset:(\d+)", t)
            key = ("scratch", slot.group(1) if slot else "0") if op.startswith("scratch_load") else None
            sregs = regs(src)
            written_inside = False
            for w in body[max(r0, 0):k]:
                wop, wdst, _ = split_operands(w)
                if key and wop.startswith("scratch_store") and (("offset:" + key[1]) in w if key[1] != "0" else "offset:" not in w):
                    written_inside = True
                    break
                if not key and not wop.startswith(("global_store", "ds_write", "scratch_store", "buffer_store")) and \
                        regs(wdst) & sregs:
                    written_inside = True
                    break
            if written_inside:
                continue
            # on the path that skips the region (a uniform condition false: exec 0 -> the copy has no effect)
            # the destination must already hold the value: harmless when nothing overwrote it since the source
            # was last written (the copy then only restores what the region itself clobbered); a hazard when
            # the destination was reused before the region opened -- then no lane outside the region has it
            def writes(w, rs):
                wop, wdst, _ = split_operands(w)
                if not wop or wop.startswith((";", "global_store", "ds_write", "scratch_store", "buffer_store")):
                    return False
                return bool(regs(wdst) & rs)
            ls = 0
            for w in range(max(r0, 0) - 1, -1, -1):
                t2 = body[w]
                if (key and split_operands(t2)[0].startswith("scratch_store") and
                        (("offset:" + key[1]) in t2 if key[1] != "0" else "offset:" not in t2)) or \
                        (not key and writes(t2, sregs)):
                    ls = w
                    break
            same = lambda w: split_operands(w)[0] == op and split_operands(w)[2].strip() == src.strip()
            last = max((w for w in range(ls + 1, max(r0, 0)) if writes(body[w], regs(dst)) and not same(body[w])), default=-1)
            if last < 0:
                continue
            # a phi: the other path's value materialised in the block that opens the region
            if not any(re.match(r"^\.LBB\w+:", body[w]) for w in range(last + 1, r0)):
                continue
            dregs = regs(dst)
            # still holding the copied value at the restore (not redefined later in the window) ...
            for w in body[k + 1:i]:
                wop, wdst, _ = split_operands(w)
                if wop and not wop.startswith((";", "global_store", "ds_write", "scratch_store", "buffer_store")):
                    dregs -= regs(wdst)
            # ... and read after the restore before a redefinition: every path from the restore (branches
            # followed: s_branch jumps, s_cbranch forks), each ending at a redefinition, the next exec change
            # or the end of the program
            used_regs = read_before_redefined(body, i + 1, set(dregs), labels)
            if used_regs:
                found.append((k, t.strip(), sorted(used_regs)))
    return found


STORES = ("global_store", "ds_write", "scratch_store", "buffer_store")
FLAT_MEM = re.compile(r"^\s*(flat_(load|store|atomic)\w*)\b")


def flat_mem(body):
    """(line index, line) of every FLAT (generic-address) memory instruction in one kernel body.  A flat
    access may target LDS; it is counted in both vmcnt and lgkmcnt, returns out of order with the DS
    operations of its own wave, and falls outside the in-order argument the NW = 1 SYNC() (a wavefront
    fence without s_waitcnt) rests on.  The round-5 build whose lip_eq_res read x0 (global) or the LDS
    iterate through one pointer carried them and broke the polish; the shipped
    kernels carry none (tests/test_isa_hazard.py)."""
    return [(k, ln.strip()) for k, ln in enumerate(body) if FLAT_MEM.match(ln)]


def read_before_redefined(body, start, live0, labels, budget=6000):
    """Registers of live0 read on some path from body[start] before that path redefines them."""
    hits, seen, work, steps = set(), set(), [(start, frozenset(live0))], 0
    while work and steps < budget:
        pos, live = work.pop()
        while pos < len(body) and live and steps < budget:
            if (pos, live) in seen:
                break
            seen.add((pos, live))
            steps += 1
            u = body[pos]
            uop, udst, usrc = split_operands(u)
            if not uop or uop.startswith((";", ".")) or uop.endswith(":"):
                pos += 1
                continue
            used = regs(usrc) | (regs(udst) if uop.startswith(STORES + ("v_cmp", "s_")) else set())
            if live & used:
                hits |= live & used
                break
            if not uop.startswith(STORES):
                live = live - regs(udst)
            if re.match(r"^\s*s_\w+\s+exec", u) or "s_endpgm" in u or "s_setpc" in u:
                break
            m = re.match(r"^\s*s_branch\s+(\.LBB\w+)", u)
            if m:
                pos = labels.get(m.group(1), len(body))
                continue
            m = re.match(r"^\s*s_cbranch_\w+\s+(\.LBB\w+)", u)
            if m and m.group(1) in labels:
                work.append((labels[m.group(1)], live))
            pos += 1
    return hits


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    total = 0
    for name, body in kernels(open(path)):
        if subs and not any(s in name for s in subs):
            continue
        f = scan(body)
        total += len(f)
        for k, t, r in f:
            print(f"{name}: line {k}: {t}   (read after the exec restore: {r})")
        fl = flat_mem(body)
        total += len(fl)
        for k, t in fl:
            print(f"{name}: line {k}: {t}   (flat memory instruction)")
    print(f"{total} findings (hazardous copies + flat memory instructions)")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
