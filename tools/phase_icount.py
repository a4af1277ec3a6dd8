"""Static instruction counts between consecutive s_memtime stamps of the stamps build
(diagnostic): python tools/phase_icount.py [kernel-name-substring]"""
import re, subprocess, sys, tempfile, os
lib = os.path.join(os.path.dirname(__file__), '..', 'srb-cbf-nmpc_amd', 'srbnmpc', 'libsrbnmpc_stamps.so')
name = sys.argv[1] if len(sys.argv) > 1 else 'srb_nmpc_kernel_12_4_1_10_2_11'
d = tempfile.mkdtemp()
subprocess.run(['/opt/rocm/lib/llvm/bin/llvm-objcopy', '--dump-section=.hip_fatbin=%s/f' % d, lib], check=True)
subprocess.run(['/opt/rocm/lib/llvm/bin/clang-offload-bundler', '--unbundle', '--type=o', '--input=%s/f' % d,
                '--targets=hipv4-amdgcn-amd-amdhsa--gfx950', '--output=%s/k.co' % d], check=True)
asm = subprocess.run(['/opt/rocm/lib/llvm/bin/llvm-objdump', '-d', '%s/k.co' % d], capture_output=True, text=True).stdout
body, on = [], False
for ln in asm.splitlines():
    if ln.endswith('<%s>:' % name):
        on = True; continue
    if on and re.match(r'^[0-9a-f]+ <.*>:$', ln):
        break
    if on and '\t' in ln:
        body.append(ln.split('//')[0].strip())
marks = [i for i, l in enumerate(body) if l.startswith('s_memtime')]
print(name, 'instructions', len(body), 'stamps', len(marks))
for a, b in zip(marks, marks[1:]):
    seg = body[a + 1:b]
    kinds = {}
    for l in seg:
        op = l.split()[0] if l else ''
        k = 'mfma' if 'mfma' in op else 'ds' if op.startswith('ds_') else 'readlane' if 'readlane' in op or 'writelane' in op else \
            'salu' if op.startswith('s_') else 'valu' if op.startswith('v_') else 'other'
        kinds[k] = kinds.get(k, 0) + 1
    print(f"  [{a:6d}..{b:6d}] {len(seg):5d}  " + ' '.join(f'{k}={v}' for k, v in sorted(kinds.items())))
