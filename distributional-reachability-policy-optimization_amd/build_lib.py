"""Build libdrpo_hip.so (gfx950) in-tree: hipcc each csrc/*.hip to an object, link a
shared library. Incremental by content: an object is rebuilt unless the SHA-256 of
(compiler version, flags, its source, every header) matches the digest stored next
to it, so copied trees with shuffled mtimes still rebuild exactly what changed."""
import hashlib
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


_CC_VERSION = None


def _cc_version():
    global _CC_VERSION
    if _CC_VERSION is None:
        r = subprocess.run([HIPCC, '--version'], capture_output=True, text=True)
        _CC_VERSION = r.stdout if r.returncode == 0 else HIPCC
    return _CC_VERSION


def _digest(src, headers, flags):
    h = hashlib.sha256()
    h.update(_cc_version().encode())
    h.update('\0'.join(flags).encode())
    for p in [src] + sorted(headers):
        h.update(os.path.basename(p).encode())
        with open(p, 'rb') as f:
            h.update(f.read())
    return h.hexdigest()


def _stale(obj, digest):
    try:
        with open(obj + '.sha256') as f:
            return f.read().strip() != digest or not os.path.exists(obj)
    except OSError:
        return True


def _compile(src, obj, flags, digest, verbose=False):
    cmd = [HIPCC] + flags + ['-I', os.path.join(HERE, '..', 'include'), '-c', src, '-o', obj]
    if verbose:
        print(' '.join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f'hipcc failed for {src}:\n{r.stderr}')
    with open(obj + '.sha256', 'w') as f:
        f.write(digest)
    return obj


def _link(objs, lib, force):
    """Relink when an object changed or the library's recorded object digests differ."""
    key = hashlib.sha256()
    for o in objs:
        with open(o + '.sha256') as f:
            key.update(f.read().encode())
    key = key.hexdigest()
    if not force and os.path.exists(lib):
        try:
            with open(lib + '.sha256') as f:
                if f.read().strip() == key:
                    return lib
        except OSError:
            pass
    r = subprocess.run([HIPCC, '--offload-arch=gfx950', '-shared', '-fPIC', '-o', lib] + objs, capture_output=True,
                       text=True)
    if r.returncode != 0:
        raise RuntimeError(f'link failed:\n{r.stderr}')
    with open(lib + '.sha256', 'w') as f:
        f.write(key)
    return lib


def _headers():
    return glob.glob(os.path.join(CSRC, '*.hpp')) + glob.glob(os.path.join(HERE, '..', 'include', '*.h'))


def source_digest():
    """SHA-256 of every source the library is built from (csrc/*.hip, csrc/*.hpp,
    include/*.h; names and contents). It is compiled INTO the library
    (drpo_build_digest) and _lib.lib() refuses a library whose digest differs, so a
    stale binary can never be tested or benched."""
    h = hashlib.sha256()
    files = glob.glob(os.path.join(CSRC, '*.hip')) + _headers()
    for p in sorted(files, key=os.path.basename):
        h.update(os.path.basename(p).encode() + b'\0')
        with open(p, 'rb') as f:
            h.update(f.read())
        h.update(b'\0')
    return h.hexdigest()


def _digest_object(objdir, flags):
    """A one-function object exporting drpo_build_digest() -> the source digest."""
    dig = source_digest()
    src = os.path.join(objdir, 'build_digest.cpp')
    text = ('extern "C" __attribute__((visibility("default"))) const char* drpo_build_digest(void) '
            '{ return "%s"; }\n' % dig)
    obj = os.path.join(objdir, 'build_digest.o')
    if not _stale(obj, dig):
        return obj
    with open(src, 'w') as f:
        f.write(text)
    r = subprocess.run(['g++', '-O2', '-fPIC', '-c', src, '-o', obj], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f'digest object failed:\n{r.stderr}')
    with open(obj + '.sha256', 'w') as f:
        f.write(dig)
    return obj


def _build(flags, lib, objdir, verbose, jobs):
    os.makedirs(objdir, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, '*.hip')))
    headers = _headers()
    objs = [os.path.join(objdir, os.path.basename(s)[:-4] + '.o') for s in srcs]
    digs = [_digest(s, headers, flags) for s in srcs]
    todo = [(s, o, d) for s, o, d in zip(srcs, objs, digs) if _stale(o, d)]
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(lambda t: _compile(t[0], t[1], flags, t[2], verbose), todo))
    objs.append(_digest_object(objdir, flags))
    return _link(objs, lib, force=bool(todo))


def build(verbose=False, jobs=8, variant=None, defines=(), tag=None):
    """variant='stamps': profiling build with in-kernel s_memtime stamps (-DDRPO_STAMPS)
    into libdrpo_hip_stamps.so; never loaded by the product. ``defines`` + ``tag``: an
    A/B build with extra -D macros into libdrpo_hip[_stamps]_<tag>.so (loaded only via
    DRPO_LIB_OVERRIDE by the profiling scripts)."""
    if defines and not tag:
        # an A/B build must never overwrite the production library (nor silently drop its -D's)
        raise ValueError('build(defines=...) needs a tag: the variant goes to libdrpo_hip[_stamps]_<tag>.so')
    flags = FLAGS + ['-D' + d for d in defines]
    suffix = f'_{tag}' if tag else ''
    if variant == 'stamps':
        return _build(flags + ['-DDRPO_STAMPS'], os.path.join(HERE, f'libdrpo_hip_stamps{suffix}.so'),
                      os.path.join(HERE, 'build_stamps' + suffix), verbose, jobs)
    if tag:
        return _build(flags, os.path.join(HERE, f'libdrpo_hip{suffix}.so'), os.path.join(HERE, 'build' + suffix),
                      verbose, jobs)
    return _build(FLAGS, LIB, OBJ, verbose, jobs)


if __name__ == '__main__':
    # python build_lib.py [--stamps] [--tag NAME -D MACRO ...]
    a = sys.argv[1:]
    tag = a[a.index('--tag') + 1] if '--tag' in a else None
    defs = [a[i + 1] for i, x in enumerate(a) if x == '-D']
    print(build(verbose='-v' in a, variant='stamps' if '--stamps' in a else None, defines=defs, tag=tag))
