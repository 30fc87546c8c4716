"""Build a diagnostic variant of the HIP library: ppo_update.hip (or another csrc file) compiled
with extra -D flags and linked with the product build's other objects, into
tools/diag_lib/libxa_<name>.so. Load it with `bench.py --lib <path>` for an A/B inside one GPU
session (diagnostic only: the product path always loads xagents_amd/libxagents_hip.so, which
_lib.load() checks against the tree's sources).

usage: python tools/build_variant.py <name> [-DFLAG ...] [--src ppo_update]"""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
OUT = ROOT / 'tools' / 'diag_lib'


def main(name, *rest):
    from xagents_amd._build import BUILD_DIR, CFLAGS, HIPCC, build_library, source_hash
    src = 'ppo_update'
    flags = []
    it = iter(rest)
    for a in it:
        if a == '--src':
            src = next(it)
        else:
            flags.append(a)
    build_library()
    OUT.mkdir(exist_ok=True)
    others = [str(o) for o in sorted(BUILD_DIR.glob('*.o')) if o.stem != src]
    obj = OUT / f'{src}_{name}.o'
    subprocess.run([HIPCC, *CFLAGS, f'-DXA_BUILD_HASH="{source_hash()}"', *flags, '-c',
                    str(ROOT / 'xagents_amd' / 'csrc' / f'{src}.hip'), '-o', str(obj)], check=True)
    lib = OUT / f'libxa_{name}.so'
    subprocess.run([HIPCC, '--offload-arch=gfx950', '-shared', '-o', str(lib), str(obj), *others],
                   check=True)
    print(lib)


if __name__ == '__main__':
    main(*sys.argv[1:])
