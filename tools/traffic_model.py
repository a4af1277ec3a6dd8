"""Byte-level model of the LIP solve / polish kernels' HBM traffic per launch, to set
against the PMC-measured FETCH_SIZE / WRITE_SIZE (profiles/r05x_pmc_traffic_c*.json, r05_traffic_ab_c3_xcd.json).

What the model counts, each term measured on its own by a microbenchmark ("Bytes"):
  - machine code: the kernel's code bytes x 16 per dispatch (tools/ubench/code_fetch.hip: a 68.7 KB kernel
    adds 16.0x its size to FETCH_SIZE whatever the grid -- each of the 8 XCDs fetches it twice);
  - kernel arguments: nothing per workgroup (tools/ubench/kernarg_fetch.hip: a 640-B by-value block is read
    once per XCD, not per workgroup);
  - inputs: the 128-B lines each XCD's agents touch -- agent-major arrays (x0, ref, foot, the selection
    rows) and the gathered table rows (obstacles 16 B, neighbour snapshot 32 B), with workgroups dealt
    round-robin over the 8 XCDs and each XCD given a contiguous block of agents (csrc/srb_wave.h xcd_agent);
  - outputs: bytes rounded to 32-B sectors per XCD block (kernarg_fetch.hip: 8-B stores cost 32 B each,
    partially written lines are not filled from HBM);
  - spilled registers: the kernel's scratch bytes per lane x 64 x the resident waves (one per SIMD), written
    back once.

    python tools/traffic_model.py [--config 3|5] [--round-robin]
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd"), os.path.join(ROOT, "tools")]
LINE, SECTOR, XCDS, CODE_FACTOR = 128, 32, 8, 16


def code_sizes(lib):
    """{kernel symbol: code bytes} of every gfx950 code object in the library."""
    import codeobj
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for k, (_, blob) in enumerate(codeobj.code_objects(lib)):
            o = os.path.join(d, f"co{k}.o")
            open(o, "wb").write(blob)
            txt = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-s", "--wide", o], capture_output=True,
                                 text=True, check=True).stdout
            for m in re.finditer(r"^\s*\d+:\s+[0-9a-f]+\s+(\d+)\s+FUNC\s+\w+\s+\w+\s+\d+\s+(\S+)$", txt, re.M):
                out[m.group(2)] = int(m.group(1))
            for m in re.finditer(r"^\s*\d+:\s+([0-9a-f]+)\s+0\s+NOTYPE\s+\w+\s+\w+\s+ABS\s+(\S+)\.private_seg_size$",
                                 txt, re.M):
                out[m.group(2) + ".scratch"] = int(m.group(1), 16)
    return out


def blocks(n, rr):
    """agents of each XCD: round-robin (agent = workgroup) or xcd_agent's contiguous blocks"""
    if rr:
        return [range(x, n, XCDS) for x in range(XCDS)]
    q, r = divmod(n, XCDS)
    return [range(x * q + min(x, r), x * q + min(x, r) + q + (x < r)) for x in range(XCDS)]


def lines(off, size):
    return range(off // LINE, (off + size - 1) // LINE + 1)


def model(config, rr=False, lib=None):
    import bench
    import oracle
    cfg = bench.CONFIGS[config]
    A, b, _, _ = bench.rank_batch(config, cfg["agents"], 1, 0)
    N, C, Ko, Kn = cfg["N"], cfg["C"], cfg["K_obs"], cfg["K_nbr"]
    K = Ko + Kn
    p = oracle.params(N, C, K_obs=Ko, K_nbr=Kn, use_nlp=1)
    sel = np.array([oracle.select_idx(p, b["x0"][a], b["obstacles"], b["nbr_state"], a) for a in range(A)])
    nv = (6 + C) * N + 1
    per_agent_in = {"x0": 32, "ref": 32 * N, "foot": 16 * C * N, "sel": 4 * K}
    fetch = {k: 0 for k in list(per_agent_in) + ["obstacle rows", "neighbour rows"]}
    for ags in blocks(A, rr):
        seen = set()
        for a in ags:
            for arr, sz in per_agent_in.items():
                seen |= {(arr, ln) for ln in lines(a * sz, sz)}
            for j in range(K):
                i = int(sel[a, j])
                if i < 0:
                    continue
                seen |= ({("obstacle rows", ln) for ln in lines(i * 16, 16)} if j < Ko else
                         {("neighbour rows", ln) for ln in lines(i * 32, 32)})
        for arr, _ in seen:
            fetch[arr] += LINE
    out_bytes = {"x": 8 * nv, "obj": 8, "status": 8, "iters": 8, "alpha": 160}
    write = {}
    for arr, sz in out_bytes.items():
        write[arr] = sum(SECTOR * len({o // SECTOR for a in ags for o in range(a * sz, a * sz + sz, 8)})
                         for ags in blocks(A, rr))
    code = code_sizes(lib or os.path.join(ROOT, "srb-cbf-nmpc_amd", "srbnmpc", "libsrbnmpc.so"))
    return dict(A=A, N=N, C=C, K=K, nv=nv, fetch=fetch, write=write, code=code)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--round-robin", action="store_true", help="model the pre-round-5 workgroup -> agent mapping")
    ap.add_argument("--kernel", default=None, help="solve kernel symbol (default: the config's compiled instance)")
    a = ap.parse_args()
    m = model(a.config, a.round_robin)
    inst = {3: "12_4_1_10_2_11", 5: "24_4_2_20_2_11"}.get(a.config)
    kern = a.kernel or "srb_nmpc_kernel_" + inst
    meas = {}
    mp = os.path.join(ROOT, "profiles", {3: "r05x_pmc_traffic_c3.json", 5: "r05f_pmc_traffic_c5.json"}.get(a.config, ""))
    if os.path.isfile(mp) and not a.round_robin:
        import json
        meas = json.load(open(mp))["kernels"]
    rows = []                                           # (kernel, direction, [(term, bytes)], measured)
    fs = [(f"code {m['code'][kern]} B x {CODE_FACTOR}", m["code"][kern] * CODE_FACTOR)] + list(m["fetch"].items())
    rows.append(("srb_nmpc_kernel", "fetch", fs, meas.get("srb_nmpc_kernel", {}).get("fetch_bytes")))
    # spilled registers: each resident wave's scratch lines are written back once (one wave per SIMD)
    nw = {3: 1, 5: 2}.get(a.config, 1)
    scr = m["code"].get(kern + ".scratch", 0) * 64 * min(m["A"] * nw, 4 * 256)
    ws = list(m["write"].items()) + ([(f"scratch {m['code'][kern + '.scratch']} B/lane, resident waves", scr)] if scr else [])
    rows.append(("srb_nmpc_kernel", "write", ws, meas.get("srb_nmpc_kernel", {}).get("write_bytes")))
    print(f"config {a.config}: {m['A']} agents, N = {m['N']}, C = {m['C']}, K = {m['K']}, "
          f"{'round-robin' if a.round_robin else 'XCD-blocked'} agents")
    for k, d, terms, mv in rows:
        tot = sum(v for _, v in terms)
        print(f"  {k} {d}: model {tot / 1e6:.3f} MB" +
              (f", measured {mv / 1e6:.3f} MB ({100 * (tot / mv - 1):+.1f} %)" if mv else ""))
        for t, v in terms:
            print(f"      {t:24s} {v / 1e6:.3f} MB")


if __name__ == "__main__":
    main()
