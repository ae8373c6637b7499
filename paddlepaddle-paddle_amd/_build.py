"""In-tree build of the native libraries (HIP kernels for gfx950 + C++ host runtime).

* ``_lib/libpaddle_amd_kernels.so`` — every ``csrc/*.hip`` compiled with
  ``hipcc --offload-arch=gfx950`` (no torch headers: a plain C ABI called through ctypes,
  so each TU builds in seconds and the library has no ABI coupling to the torch build).
* ``_lib/libpaddle_amd_runtime.so`` — ``csrc/runtime/*.cpp`` host code (data-loader
  prefetch ring, host tracer, flags), compiled with g++.
* ``_lib/libpaddle_amd_alloc.so`` — ``csrc/alloc/allocator.cpp``, the native auto-growth
  best-fit device allocator (host code over the HIP runtime, compiled with hipcc), loaded by
  torch's pluggable-allocator hook when enabled.

Incremental: an object is rebuilt only when its source or a header is newer.
"""
import concurrent.futures
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
LIB = os.path.join(HERE, '_lib')
OBJ = os.path.join(LIB, 'obj')
ARCH = os.environ.get('PADDLE_AMD_ARCH', 'gfx950')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')

KERNEL_LIB = os.path.join(LIB, 'libpaddle_amd_kernels.so')
RUNTIME_LIB = os.path.join(LIB, 'libpaddle_amd_runtime.so')
ALLOC_LIB = os.path.join(LIB, 'libpaddle_amd_alloc.so')


def _newer(src, dst, deps=()):
    if not os.path.exists(dst):
        return True
    t = os.path.getmtime(dst)
    return any(os.path.getmtime(p) > t for p in (src, *deps))


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def build_kernels(verbose=False, jobs=None):
    os.makedirs(OBJ, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, '*.hip')))
    headers = glob.glob(os.path.join(CSRC, '*.h'))
    objs = []
    todo = []
    for s in srcs:
        o = os.path.join(OBJ, os.path.basename(s) + '.o')
        objs.append(o)
        if _newer(s, o, headers):
            todo.append((s, o))
    cmds = [[HIPCC, '-O3', f'--offload-arch={ARCH}', '-fPIC', '-std=c++17', '-ffp-contract=fast', '-munsafe-fp-atomics',
             '-I', CSRC, '-c', s, '-o', o] for s, o in todo]
    jobs = jobs or min(8, os.cpu_count() or 4)
    with concurrent.futures.ThreadPoolExecutor(jobs) as ex:
        for out in ex.map(_run, cmds):
            if verbose and out.strip():
                print(out)
    if todo or not os.path.exists(KERNEL_LIB) or any(os.path.getmtime(o) > os.path.getmtime(KERNEL_LIB) for o in objs):
        _run([HIPCC, f'--offload-arch={ARCH}', '-shared', '-fPIC', '-o', KERNEL_LIB + '.tmp', *objs])
        os.replace(KERNEL_LIB + '.tmp', KERNEL_LIB)
    return KERNEL_LIB


def build_runtime(verbose=False):
    os.makedirs(OBJ, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, 'runtime', '*.cpp')))
    if not srcs:
        return None
    headers = glob.glob(os.path.join(CSRC, 'runtime', '*.h'))
    if not os.path.exists(RUNTIME_LIB) or any(_newer(s, RUNTIME_LIB, headers) for s in srcs):
        _run(['g++', '-O3', '-std=c++17', '-fPIC', '-shared', '-pthread', '-I', os.path.join(CSRC, 'runtime'), *srcs,
              '-o', RUNTIME_LIB + '.tmp'])
        os.replace(RUNTIME_LIB + '.tmp', RUNTIME_LIB)
    return RUNTIME_LIB


def build_alloc(verbose=False):
    os.makedirs(LIB, exist_ok=True)
    src = os.path.join(CSRC, 'alloc', 'allocator.cpp')
    if _newer(src, ALLOC_LIB):
        _run([HIPCC, '-O2', '-std=c++17', '-fPIC', '-shared', src, '-o', ALLOC_LIB + '.tmp'])
        os.replace(ALLOC_LIB + '.tmp', ALLOC_LIB)
    return ALLOC_LIB


def build_all(verbose=False):
    k = build_kernels(verbose)
    r = build_runtime(verbose)
    a = build_alloc(verbose)
    return k, r, a


if __name__ == '__main__':
    print(build_all(verbose='-v' in sys.argv))
