#!/usr/bin/env python3
"""Per-kernel register budget and instruction mix of one HIP source, compiled for gfx950.

    python tools/isa_mix.py kompressor_amd/csrc/kmp_codec_wave2dp.hip [name-filter]

Prints VGPRs, scratch bytes, static instruction count and the counts of the instruction classes
that matter for the codec kernels (global loads / stores, ds_bpermute shuffles, DPP moves, VALU).
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

src = os.path.abspath(sys.argv[1])
filt = sys.argv[2] if len(sys.argv) > 2 else ''
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
with tempfile.TemporaryDirectory() as d:
    subprocess.run(['/opt/rocm/bin/hipcc', '-O3', '-std=c++17', '-fPIC', '--offload-arch=gfx950', '-c', src,
                    '-o', os.path.join(d, 'x.o'), '-save-temps=obj', f'-I{root}'], check=True, cwd=d)
    asm = [f for f in os.listdir(d) if f.endswith('gfx950.s')][0]
    s = open(os.path.join(d, asm)).read()
meta = {m.group(1): m.group(2) for m in re.finditer(r'\.name:\s+(\S+)\n(.*?)(?=\n\s+- \.|\Z)', s, re.S)}
for m in re.finditer(r'^(\S+):\s*;\s*@', s, re.M):
    name = m.group(1)
    if filt not in name:
        continue
    end = s.index('.Lfunc_end', m.end())
    c = collections.Counter()
    for line in s[m.end():end].split('\n'):
        t = line.strip().split()
        if not t or t[0].startswith(('.', ';')) or t[0].endswith(':'):
            continue
        c[t[0]] += 1
    md = meta.get(name, '')
    vg = re.search(r'\.vgpr_count:\s+(\d+)', md)
    sp = re.search(r'\.private_segment_fixed_size:\s+(\d+)', md)
    cls = lambda p: sum(v for k, v in c.items() if k.startswith(p))  # noqa: E731
    print(f"{name[:90]}\n  vgpr {vg and vg.group(1)} scratch {sp and sp.group(1)} insts {sum(c.values())} "
          f"gload {cls('global_load')} gstore {cls('global_store')} bperm {c['ds_bpermute_b32']} "
          f"dpp {sum(v for k, v in c.items() if 'dpp' in k)} valu {cls('v_')} salu {cls('s_')}")
