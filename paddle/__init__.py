"""``import paddle`` → the MI355X-native framework in ``paddlepaddle-paddle_amd/``.

The framework's source directory name is not a valid Python identifier, so this package
adopts it as its search path: ``paddle.nn`` resolves to ``paddlepaddle-paddle_amd/nn`` and the
framework's ``__init__`` runs in this module's namespace.
"""
import os as _os

_ROOT = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), 'paddlepaddle-paddle_amd')
__path__ = [_ROOT]
__file__ = _os.path.join(_ROOT, '__init__.py')
with open(__file__) as _f:
    exec(compile(_f.read(), __file__, 'exec'))
