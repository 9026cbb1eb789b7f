"""Build ``libkompressor_hip.so`` in-tree with hipcc for gfx950 (no JIT, no torch extension).

``python kompressor_amd/_build.py`` or ``__graft_entry__.build()`` (by path: ``-m`` would import
the package first, which needs a library that already exports every symbol).  Objects are compiled in
parallel and cached by source mtime under ``kompressor_amd/build/``.
"""

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
BUILD = os.path.join(HERE, 'build')
LIB = os.path.join(HERE, 'libkompressor_hip.so')
# the debug variant: device bounds checks (KMP_DCHECK / KMP_SPAN in kmp_common.h) compiled in;
# loaded instead of the release library when KMP_DEBUG=1 (kompressor_amd/_lib.py)
BUILD_DEBUG = os.path.join(HERE, 'build_debug')
LIB_DEBUG = os.path.join(HERE, 'libkompressor_hip_debug.so')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = 'gfx950'
FLAGS = ['-O3', '-std=c++17', '-fPIC', f'--offload-arch={ARCH}', '-Wall', '-Wno-unused-function',
         '-Wno-unused-variable', '-Wno-unused-but-set-variable']


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith('.hip'))


def _headers_mtime():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith('.h')]
    hs.append(os.path.join(HERE, '..', 'include', 'kompressor_hip.h'))
    return max(os.path.getmtime(h) for h in hs)


# per-file flags: the matrix-core LinearPredictor kernels keep MFMA accumulators in ordinary VGPRs
# (-amdgpu-mfma-vgpr-form): with AGPRs every tile paid 4 accvgpr writes (the bias) and 4 reads
# (the results) per MFMA, 256 VALU instructions per wave step of kmp_codec_linear3m.hip
FILE_FLAGS = {'kmp_codec_linear3m.hip': ['-mllvm', '-amdgpu-mfma-vgpr-form'],
              'kmp_codec_linear3pm.hip': ['-mllvm', '-amdgpu-mfma-vgpr-form'],
              'kmp_linear.hip': ['-mllvm', '-amdgpu-mfma-vgpr-form']}


def _compile(src, hdr_mtime, verbose, debug=False):
    obj = os.path.join(BUILD_DEBUG if debug else BUILD, os.path.basename(src).replace('.hip', '.o'))
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hdr_mtime,
                                                            os.path.getmtime(os.path.abspath(__file__))):
        return obj
    cmd = [HIPCC, *FLAGS, *FILE_FLAGS.get(os.path.basename(src), []), *(['-DKMP_DEBUG'] if debug else []),
           '-c', src, '-o', obj]
    if verbose:
        print(' '.join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return obj


def build(verbose=True, jobs=None, debug=False):
    """Compile and link the release library (``debug=False``) or the bounds-checked debug variant."""
    bdir, lib = (BUILD_DEBUG, LIB_DEBUG) if debug else (BUILD, LIB)
    os.makedirs(bdir, exist_ok=True)
    hdr = _headers_mtime()
    srcs = sources()
    jobs = jobs or min(len(srcs), max(1, min(8, os.cpu_count() or 1)))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdr, verbose, debug), srcs))
    stamp = os.path.join(bdir, 'objects.txt')  # relink when the set of sources changes too
    listing = '\n'.join(sorted(objs))
    same_set = os.path.exists(stamp) and open(stamp).read() == listing
    if not (same_set and os.path.exists(lib) and os.path.getmtime(lib) >= max(os.path.getmtime(o) for o in objs)):
        cmd = [HIPCC, f'--offload-arch={ARCH}', '-shared', '-fPIC', *objs, '-o', lib + '.tmp']
        if verbose:
            print(' '.join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(lib + '.tmp', lib)
        with open(stamp, 'w') as f:
            f.write(listing)
    if not debug:
        _build_capi_example(verbose)
    return lib


def _build_capi_example(verbose):
    """tools/capi_example: the C-ABI from a plain C++ host (no Python), linked to the in-tree
    library by a relative rpath so it runs from any checkout."""
    root = os.path.dirname(HERE)
    src = os.path.join(root, 'tools', 'capi_example.cpp')
    exe = os.path.join(root, 'tools', 'capi_example')
    if not os.path.exists(src):
        return
    if os.path.exists(exe) and os.path.getmtime(exe) >= max(os.path.getmtime(src), os.path.getmtime(LIB)):
        return
    cmd = [HIPCC, '-O2', f'--offload-arch={ARCH}', src, '-o', exe, f'-L{HERE}', '-lkompressor_hip',
           '-Wl,-rpath,$ORIGIN/../kompressor_amd']
    if verbose:
        print(' '.join(cmd), flush=True)
    subprocess.run(cmd, check=True)


if __name__ == '__main__':
    print(build(verbose='-q' not in sys.argv, debug=os.environ.get('KMP_DEBUG', '0') != '0' or '--debug' in sys.argv))
