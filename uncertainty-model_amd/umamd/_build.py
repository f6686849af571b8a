"""Build libumamd.so (HIP kernels + C ABI) for gfx950 with hipcc.

In-tree build: objects under csrc/build/, the shared library at
umamd/libumamd.so (git-ignored, travels to the GPU box with the snapshot).

Staleness is judged on content, never on mtimes (mtimes do not survive every
copy of the tree: ``cp -p``, ``rsync -t`` and snapshot restores keep old
times on new contents):
  * each object file has a ``.hash`` stamp = sha256 of its source, every
    header and the flags; an object whose stamp differs is recompiled;
  * the library's stamp = the hash of all sources + headers + flags; it is
    written only after a link that used the freshly checked objects.

Concurrent builders (every rank of a torchrun job importing the package at
once) serialise on an ``fcntl.flock`` of ``umamd/.build.lock``; the library is
linked to a temporary file and ``os.replace``d into place, so no process can
load a half-written ``.so``.
"""
from __future__ import annotations

import concurrent.futures as cf
import contextlib
import fcntl
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
LOCK = os.path.join(HERE, '.build.lock')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = os.environ.get('UMAMD_ARCH', 'gfx950')
FLAGS = ['-O3', '-fPIC', '-std=c++17', f'--offload-arch={ARCH}', '-I', INCLUDE, '-I', CSRC]
STAMP = LIB + '.stamp'


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, '*.hip')) + glob.glob(os.path.join(CSRC, '*.cpp')))


def _headers():
    return sorted(glob.glob(os.path.join(CSRC, '*.h')) + glob.glob(os.path.join(INCLUDE, '*.h')))


def _flags_key() -> str:
    """the compile flags as they enter the stamps: the include directories
    relative to the repository, so a copy of the tree at another path (the
    GPU box's snapshot) sees the same stamps and loads the shipped library
    instead of rebuilding it"""
    root = os.path.dirname(PKG)
    return ' '.join(os.path.relpath(f, root) if os.path.isabs(f) else f for f in FLAGS)


def _hash_files(files, extra=b'') -> str:
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, 'rb') as fh:
            h.update(fh.read())
    h.update(_flags_key().encode())
    h.update(extra)
    return h.hexdigest()


def _obj_hash(src) -> str:
    """content hash of one translation unit (its source + every header)"""
    return _hash_files([src] + _headers())


def _digest() -> str:
    """content hash of every source and header (the library's stamp)"""
    return _hash_files(sorted(_sources() + _headers()))


def _read(path):
    try:
        with open(path) as fh:
            return fh.read().strip()
    except OSError:
        return None


def _write_atomic(path, text):
    tmp = f'{path}.tmp{os.getpid()}'
    with open(tmp, 'w') as fh:
        fh.write(text + '\n')
    os.replace(tmp, path)


def _compile(src):
    """-> (object path, recompiled?)"""
    obj = os.path.join(OBJDIR, os.path.basename(src) + '.o')
    want = _obj_hash(src)
    if os.path.isfile(obj) and _read(obj + '.hash') == want:
        return obj, False
    tmp = f'{obj}.tmp{os.getpid()}'
    cmd = [HIPCC] + FLAGS + ['-c', src, '-o', tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        with contextlib.suppress(OSError):
            os.remove(tmp)
        raise RuntimeError(f'hipcc failed for {src}:\n{r.stderr}')
    os.replace(tmp, obj)
    _write_atomic(obj + '.hash', want)
    return obj, True


def needs_build() -> bool:
    """True when the library is missing or was built from other sources."""
    if not os.path.isfile(LIB):
        return True
    return _read(STAMP) != _digest()


def can_build() -> bool:
    return os.path.isfile(HIPCC) and os.access(HIPCC, os.X_OK)


@contextlib.contextmanager
def build_lock():
    """exclusive inter-process lock around check-and-build"""
    fd = os.open(LOCK, os.O_RDWR | os.O_CREAT, 0o644)
    try:
        fcntl.flock(fd, fcntl.LOCK_EX)
        yield
    finally:
        fcntl.flock(fd, fcntl.LOCK_UN)
        os.close(fd)


def _build_locked(verbose: bool) -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    digest = _digest()
    srcs = _sources()
    jobs = min(len(srcs), int(os.environ.get('MAX_JOBS', os.cpu_count() or 4)), 16)
    with cf.ThreadPoolExecutor(max_workers=max(jobs, 1)) as ex:
        res = list(ex.map(_compile, srcs))
    objs = [o for o, _ in res]
    if any(c for _, c in res) or not os.path.isfile(LIB) or _read(STAMP) != digest:
        tmp = f'{LIB}.tmp{os.getpid()}'
        cmd = [HIPCC, f'--offload-arch={ARCH}', '-shared', '-fPIC', '-o', tmp] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            with contextlib.suppress(OSError):
                os.remove(tmp)
            raise RuntimeError(f'link failed:\n{r.stderr}')
        os.replace(tmp, LIB)
        _write_atomic(STAMP, digest)  # only after a link of the checked objects
    if verbose:
        print(f'built {LIB}')
    return LIB


def build(verbose: bool = False) -> str:
    with build_lock():
        return _build_locked(verbose)


def ensure_built() -> bool:
    """Build under the lock when stale (re-checked once the lock is held, so
    a rank that waited for another's build does not rebuild).  -> built?"""
    if not needs_build():
        return False
    with build_lock():
        if not needs_build():
            return False
        _build_locked(False)
        return True


if __name__ == '__main__':
    build(verbose=True)
    sys.exit(0)
