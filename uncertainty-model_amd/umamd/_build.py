"""Build libumamd.so (HIP kernels + C ABI) for gfx950 with hipcc.

In-tree build: objects under csrc/build/, the shared library at
umamd/libumamd.so (git-ignored, travels to the GPU box with the snapshot).
Incremental on mtimes of the sources and headers.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
CSRC = os.path.join(PKG, 'csrc')
INCLUDE = os.path.join(os.path.dirname(PKG), 'include')
OBJDIR = os.path.join(CSRC, 'build')
LIB = os.path.join(HERE, 'libumamd.so')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = os.environ.get('UMAMD_ARCH', 'gfx950')
FLAGS = ['-O3', '-fPIC', '-std=c++17', f'--offload-arch={ARCH}', '-I', INCLUDE, '-I', CSRC]


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, '*.hip')) + glob.glob(os.path.join(CSRC, '*.cpp')))


def _headers():
    return glob.glob(os.path.join(CSRC, '*.h')) + glob.glob(os.path.join(INCLUDE, '*.h'))


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src):
    obj = os.path.join(OBJDIR, os.path.basename(src) + '.o')
    if _stale(obj, [src] + _headers()):
        cmd = [HIPCC] + FLAGS + ['-c', src, '-o', obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f'hipcc failed for {src}:\n{r.stderr}')
    return obj


STAMP = LIB + '.stamp'


def _digest() -> str:
    """Content hash of every source and header (mtimes do not survive every
    copy of the tree, so staleness of the library is judged on content)."""
    h = hashlib.sha256()
    for f in sorted(_sources() + _headers()):
        h.update(os.path.basename(f).encode())
        with open(f, 'rb') as fh:
            h.update(fh.read())
    h.update(' '.join(FLAGS).encode())
    return h.hexdigest()


def needs_build() -> bool:
    """True when the library is missing or was built from other sources."""
    if not os.path.isfile(LIB) or not os.path.isfile(STAMP):
        return True
    with open(STAMP) as fh:
        return fh.read().strip() != _digest()


def can_build() -> bool:
    return os.path.isfile(HIPCC) and os.access(HIPCC, os.X_OK)


def build(verbose: bool = False) -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = _sources()
    jobs = min(len(srcs), int(os.environ.get('MAX_JOBS', os.cpu_count() or 4)), 16)
    with cf.ThreadPoolExecutor(max_workers=max(jobs, 1)) as ex:
        objs = list(ex.map(_compile, srcs))
    if _stale(LIB, objs):
        cmd = [HIPCC, f'--offload-arch={ARCH}', '-shared', '-fPIC', '-o', LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f'link failed:\n{r.stderr}')
    with open(STAMP, 'w') as fh:
        fh.write(_digest() + '\n')
    if verbose:
        print(f'built {LIB}')
    return LIB


if __name__ == '__main__':
    build(verbose=True)
    sys.exit(0)
