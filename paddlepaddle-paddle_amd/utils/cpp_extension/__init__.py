"""paddle.utils.cpp_extension (reference: python/paddle/utils/cpp_extension/{cpp_extension,
extension_utils}.py — load, setup, CppExtension, CUDAExtension).

Custom operators are built for gfx950 with hipcc:
* ``load(name, sources)`` — pybind11 extensions (torch C++ extension API, HIP sources compiled
  with ``--offload-arch=gfx950``), built in-tree under ``get_build_directory()``;
* ``load_hip_library(name, sources)`` — plain C-ABI ``extern "C"`` launchers (the way this
  framework's own kernels are built), returned as a ctypes library.
"""
import ctypes
import hashlib
import os
import subprocess

_BUILD = os.environ.get('PADDLE_EXTENSION_DIR', os.path.join(os.getcwd(), '.paddle_extensions'))


def get_build_directory(verbose=False):
    os.makedirs(_BUILD, exist_ok=True)
    return _BUILD


def _arch():
    return os.environ.get('PADDLE_AMD_ARCH', 'gfx950')


def load(name, sources, extra_cxx_cflags=None, extra_cuda_cflags=None, extra_ldflags=None, extra_include_paths=None,
         build_directory=None, verbose=False):
    os.environ.setdefault('PYTORCH_ROCM_ARCH', _arch())
    from torch.utils import cpp_extension as tce
    bdir = build_directory or os.path.join(get_build_directory(), name)
    os.makedirs(bdir, exist_ok=True)
    return tce.load(name=name, sources=list(sources), extra_cflags=extra_cxx_cflags or [],
                    extra_cuda_cflags=(extra_cuda_cflags or []) + [f'--offload-arch={_arch()}'],
                    extra_ldflags=extra_ldflags or [], extra_include_paths=extra_include_paths or [],
                    build_directory=bdir, verbose=verbose)


def load_hip_library(name, sources, extra_cflags=None, build_directory=None):
    """hipcc-compile ``sources`` into lib<name>.so for gfx950 and dlopen it (C ABI)."""
    bdir = build_directory or os.path.join(get_build_directory(), name)
    os.makedirs(bdir, exist_ok=True)
    h = hashlib.sha1()
    for s in sources:
        with open(s, 'rb') as f:
            h.update(f.read())
    h.update(' '.join(extra_cflags or []).encode())
    out = os.path.join(bdir, f"lib{name}_{h.hexdigest()[:10]}.so")
    if not os.path.exists(out):
        hipcc = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
        cmd = [hipcc, '-O3', f'--offload-arch={_arch()}', '-fPIC', '-shared', '-std=c++17', *(extra_cflags or []),
               *sources, '-o', out + '.tmp']
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed:\n{r.stdout}\n{r.stderr}")
        os.replace(out + '.tmp', out)
    return ctypes.CDLL(out)


def CppExtension(sources, *args, **kwargs):  # noqa: N802
    from torch.utils import cpp_extension as tce
    return tce.CppExtension(kwargs.pop('name', 'paddle_custom_ops'), sources, *args, **kwargs)


def CUDAExtension(sources, *args, **kwargs):  # noqa: N802
    os.environ.setdefault('PYTORCH_ROCM_ARCH', _arch())
    from torch.utils import cpp_extension as tce
    return tce.CUDAExtension(kwargs.pop('name', 'paddle_custom_ops'), sources, *args, **kwargs)


def setup(**attr):
    from setuptools import setup as _setup
    from torch.utils import cpp_extension as tce
    attr.setdefault('cmdclass', {})['build_ext'] = tce.BuildExtension
    return _setup(**attr)


BuildExtension = None
