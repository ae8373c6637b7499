"""paddle.hub (reference: python/paddle/hapi/hub.py): load models from a local repo dir
containing ``hubconf.py`` (no network here, so only ``source='local'``)."""
import importlib.util
import os
import sys


def _load_hubconf(repo_dir):
    path = os.path.join(repo_dir, 'hubconf.py')
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} not found")
    sys.path.insert(0, repo_dir)
    try:
        spec = importlib.util.spec_from_file_location('hubconf', path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        sys.path.remove(repo_dir)
    return mod


def _check_source(source):
    if source != 'local':
        raise RuntimeError("only source='local' is supported (no network access)")


def list(repo_dir, source='github', force_reload=False):  # noqa: A001
    _check_source(source)
    m = _load_hubconf(repo_dir)
    return [k for k in dir(m) if callable(getattr(m, k)) and not k.startswith('_')]


def help(repo_dir, model, source='github', force_reload=False):  # noqa: A001
    _check_source(source)
    return getattr(_load_hubconf(repo_dir), model).__doc__


def load(repo_dir, model, source='github', force_reload=False, **kwargs):
    _check_source(source)
    return getattr(_load_hubconf(repo_dir), model)(**kwargs)
