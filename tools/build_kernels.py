"""Incremental in-tree rebuild of the native libraries (same as __graft_entry__.build without the
package import); loads _build.py by path so the package's own module names (signal.py, ...) do
not shadow the standard library."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location('_pa_build', os.path.join(ROOT, 'paddlepaddle-paddle_amd', '_build.py'))
mod = importlib.util.module_from_spec(spec)
spec.loader.exec_module(mod)
print(mod.build_all())
