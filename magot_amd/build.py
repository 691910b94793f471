"""Build libmagot.so in-tree for gfx950 (``python -m magot_amd.build``).

One hipcc invocation per translation unit, then a shared link, so a rebuild
after a kernel edit recompiles one file.  Objects go to ``magot_amd/_build``;
the library to ``magot_amd/libmagot.so`` (both git-ignored, both travel to
the GPU box with the gpurun snapshot).
"""

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, 'csrc')
OBJ = os.path.join(HERE, '_build')
LIB = os.path.join(HERE, 'libmagot.so')
ARCH = os.environ.get('MAGOT_OFFLOAD_ARCH', 'gfx950')

SOURCES = ['abi.hip', 'extract.hip', 'seqops.hip', 'pack.cpp', 'gffplan.cpp', 'fasta.cpp',
           'render.hip', 'devpack.hip', 'wire.hip']
HEADERS = ['common.h', 'wavecopy.h', os.path.join('..', '..', 'include', 'magot.h')]

CXXFLAGS = ['-O3', '-std=c++17', '-fPIC', '-Wall', '-Wno-unused-function',
            '--offload-arch=' + ARCH, '-I' + os.path.join(ROOT, 'include')]


def _hipcc():
    for cand in (os.environ.get('HIPCC'), '/opt/rocm/bin/hipcc', 'hipcc'):
        if cand and (os.path.sep not in cand or os.path.exists(cand)):
            return cand
    raise RuntimeError('hipcc not found')


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force=False, verbose=False):
    os.makedirs(OBJ, exist_ok=True)
    hipcc = _hipcc()
    headers = [os.path.join(CSRC, h) for h in HEADERS]
    objs = []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(OBJ, src + '.o')
        objs.append(o)
        if force or _newer(o, [s] + headers + [__file__]):
            lang = ['-x', 'hip'] if src.endswith('.hip') else []
            cmd = [hipcc] + CXXFLAGS + lang + ['-c', s, '-o', o]
            if verbose:
                print(' '.join(cmd), flush=True)
            subprocess.check_call(cmd)
    if force or _newer(LIB, objs):
        cmd = [hipcc, '-shared', '-fPIC', '--offload-arch=' + ARCH, '-o', LIB] + objs + ['-lpthread']
        if verbose:
            print(' '.join(cmd), flush=True)
        subprocess.check_call(cmd)
    return LIB


if __name__ == '__main__':
    build(force='--force' in sys.argv, verbose=True)
    print(LIB)
