"""Build libdrpo_hip.so (gfx950) in-tree: hipcc each csrc/*.hip to an object, link a
shared library. Incremental (skips objects newer than their sources/headers)."""
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
OBJ = os.path.join(HERE, 'build')
LIB = os.path.join(HERE, 'libdrpo_hip.so')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
FLAGS = ['-O3', '--offload-arch=gfx950', '-std=c++17', '-fPIC', '-Wall', '-Wno-unused-function',
         '-Wno-unused-variable', '-Wno-unused-but-set-variable', '-fvisibility=hidden']


def _stale(src, obj, headers):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(p) > t for p in [src] + headers)


def build(verbose=False, jobs=8, variant=None):
    """variant='stamps': profiling build with in-kernel s_memtime stamps (-DDRPO_STAMPS)
    into libdrpo_hip_stamps.so; never loaded by the product."""
    if variant == 'stamps':
        return _build_variant(['-DDRPO_STAMPS'], os.path.join(HERE, 'libdrpo_hip_stamps.so'), 'build_stamps', verbose,
                              jobs)
    os.makedirs(OBJ, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, '*.hip')))
    headers = glob.glob(os.path.join(CSRC, '*.hpp')) + glob.glob(os.path.join(HERE, '..', 'include', '*.h'))
    objs = [os.path.join(OBJ, os.path.basename(s)[:-4] + '.o') for s in srcs]
    todo = [(s, o) for s, o in zip(srcs, objs) if _stale(s, o, headers)]

    def cc(so):
        s, o = so
        cmd = [HIPCC] + FLAGS + ['-I', os.path.join(HERE, '..', 'include'), '-c', s, '-o', o]
        if verbose:
            print(' '.join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f'hipcc failed for {s}:\n{r.stderr}')
        return o

    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(cc, todo))
    if todo or not os.path.exists(LIB) or any(os.path.getmtime(o) > os.path.getmtime(LIB) for o in objs):
        cmd = [HIPCC, '--offload-arch=gfx950', '-shared', '-fPIC', '-o', LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f'link failed:\n{r.stderr}')
    return LIB


def _build_variant(defs, lib, objdir, verbose, jobs):
    od = os.path.join(HERE, objdir)
    os.makedirs(od, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, '*.hip')))
    objs = [os.path.join(od, os.path.basename(s)[:-4] + '.o') for s in srcs]

    def cc(so):
        s, o = so
        cmd = [HIPCC] + FLAGS + defs + ['-I', os.path.join(HERE, '..', 'include'), '-c', s, '-o', o]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f'hipcc failed for {s}:\n{r.stderr}')

    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(cc, zip(srcs, objs)))
    r = subprocess.run([HIPCC, '--offload-arch=gfx950', '-shared', '-fPIC', '-o', lib] + objs, capture_output=True,
                       text=True)
    if r.returncode != 0:
        raise RuntimeError(f'link failed:\n{r.stderr}')
    return lib


if __name__ == '__main__':
    print(build(verbose='-v' in sys.argv, variant='stamps' if '--stamps' in sys.argv else None))
