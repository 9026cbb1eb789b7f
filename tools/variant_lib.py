"""Build an experiment variant of the library: every object from the release build except ONE
source recompiled with extra flags, linked to kompressor_amd/libkompressor_hip_<name>.so (load it
with KOMPRESSOR_HIP_LIB=...; delete it after the A/B -- it is not a product library).

    python tools/variant_lib.py NAME kmp_codec_linear3d.hip -DL3Y_EXP=1 [...]
    python tools/variant_lib.py NAME /tmp/edited_copy.hip=kmp_rice.hip [...]   (an edited copy replaces one source)"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), 'kompressor_amd')
sys.path.insert(0, PKG)
import _build  # noqa: E402

name, src, flags = sys.argv[1], sys.argv[2], sys.argv[3:]
path = None
if '=' in src:
    path, src = src.split('=', 1)
_build.build(verbose=False)
objs = sorted(os.path.join(_build.BUILD, f) for f in os.listdir(_build.BUILD) if f.endswith('.o'))
vobj = os.path.join('/tmp', f'variant_{name}_' + src.replace('.hip', '.o'))
subprocess.run([_build.HIPCC, *_build.FLAGS, *_build.FILE_FLAGS.get(src, []), *flags, '-I', _build.CSRC, '-c',
                path or os.path.join(_build.CSRC, src), '-o', vobj], check=True)
objs = [vobj if os.path.basename(o) == src.replace('.hip', '.o') else o for o in objs]
out = os.path.join(PKG, f'libkompressor_hip_{name}.so')
subprocess.run([_build.HIPCC, f'--offload-arch={_build.ARCH}', '-shared', '-fPIC', *objs, '-o', out], check=True)
print(out)
