"""Build libxagents_hip.so for gfx950 with hipcc (in-tree, so it travels with the repo).

The library is plain C-ABI (include/xagents_hip.h); no torch headers are involved.
"""
import hashlib
import os
import re
import subprocess
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
CSRC = PKG_DIR / 'csrc'
LIB_PATH = PKG_DIR / 'libxagents_hip.so'
BUILD_DIR = PKG_DIR.parent / 'build' / 'hip'
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = 'gfx950'
CFLAGS = [
    f'--offload-arch={ARCH}',
    '-O3',
    '-std=c++17',
    '-fPIC',
    # every fused multiply-add is written explicitly (fmaf); nothing else may be
    # contracted, so the CPU oracle can restate the exact f32 operation order
    '-ffp-contract=off',
    '-Wall',
    '-Wno-unused-function',
]


def sources():
    return sorted(CSRC.glob('*.hip'))


def _inputs():
    return sorted(list(sources()) + list(CSRC.glob('*.hpp'))) + [
        PKG_DIR.parent / 'include' / 'xagents_hip.h']


def _flags_key():
    return (' '.join([HIPCC, *CFLAGS]) + '\0').encode()


def source_hash():
    """16 hex digits of SHA-256 over every library input (name + bytes) and the compiler
    command (HIPCC + CFLAGS): baked into the library as xa_build_hash(), compared by
    needs_build() and _lib.load()."""
    h = hashlib.sha256()
    for f in _inputs():
        h.update(f.name.encode() + b'\0' + f.read_bytes() + b'\0')
    h.update(_flags_key())
    return h.hexdigest()[:16]


_INCLUDE_RE = re.compile(rb'^\s*#\s*include\s+"([^"]+)"', re.M)


def _local_includes(src):
    """The quoted #include files of src, transitively (resolved next to the including
    file: csrc headers and ../../include/xagents_hip.h), src itself first."""
    seen, todo = [], [Path(src)]
    while todo:
        f = todo.pop()
        if f in seen or not f.exists():
            continue
        seen.append(f)
        todo += [(f.parent / m.decode()).resolve() for m in _INCLUDE_RE.findall(f.read_bytes())]
    return seen


def _object_key(src):
    """What one object depends on: its source, the csrc / C-ABI headers it includes
    (transitively), the compiler command."""
    h = hashlib.sha256()
    deps = _local_includes(src)
    for f in deps[:1] + sorted(deps[1:]):
        h.update(f.name.encode() + b'\0' + f.read_bytes() + b'\0')
    h.update(_flags_key())
    return h.hexdigest()


def library_hash(path=LIB_PATH):
    """The source hash baked into a built library (read from its bytes, no load)."""
    try:
        m = re.search(rb'XA_BUILD_HASH:([0-9a-f]{16})', Path(path).read_bytes())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def needs_build():
    return not LIB_PATH.exists() or library_hash() != source_hash()


def build_library(force=False, verbose=False):
    """Compile every csrc/*.hip for gfx950 and link libxagents_hip.so."""
    if not force and not needs_build():
        return LIB_PATH
    BUILD_DIR.mkdir(parents=True, exist_ok=True)
    digest = source_hash()

    def compile_one(src):
        # only xa_runtime.hip carries the library hash; every other object is rebuilt
        # when its own inputs change (key file next to the object)
        obj = BUILD_DIR / (src.stem + '.o')
        stamp = obj.with_suffix('.key')
        runtime = src.name == 'xa_runtime.hip'
        key = _object_key(src)
        if not force and not runtime and obj.exists() and stamp.exists() and \
                stamp.read_text() == key:
            return obj
        extra = [f'-DXA_BUILD_HASH="{digest}"'] if runtime else []
        cmd = [HIPCC, *CFLAGS, *extra, '-c', str(src), '-o', str(obj)]
        if verbose:
            print(' '.join(cmd))
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f'hipcc failed for {src.name}:\n{res.stderr}')
        stamp.write_text(key)
        return obj

    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as pool:
        objs = list(pool.map(compile_one, sources()))
    tmp = LIB_PATH.with_suffix('.so.tmp')
    cmd = [HIPCC, f'--offload-arch={ARCH}', '-shared', '-o', str(tmp), *map(str, objs)]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f'link failed:\n{res.stderr}')
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == '__main__':
    print(build_library(force=True, verbose=True))
