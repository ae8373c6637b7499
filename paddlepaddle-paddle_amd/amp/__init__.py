"""paddle.amp (reference: python/paddle/amp/{auto_cast,grad_scaler}.py).

* ``auto_cast(level='O1'|'O2'|'OD')`` applies the reference's per-op cast rule (white list ->
  bf16/fp16, black list -> fp32, custom lists, O2 = pure low precision) at the paddle op
  boundary (``core.amp_dispatch``); ``level='O2'`` expects parameters cast by ``decorate``.
* ``decorate(level='O2')`` casts parameters to the low-precision dtype except normalisation
  layers (kept fp32, like the reference) and turns on optimizer master weights.
* ``GradScaler`` — dynamic loss scaling with found-inf skip (needed for fp16; bf16 runs
  with ``enable=False`` semantics by default).
"""
from .auto_cast import auto_cast, amp_guard, decorate, amp_decorate, is_float16_supported, is_bfloat16_supported  # noqa: F401
from .grad_scaler import GradScaler, AmpScaler, OptimizerState  # noqa: F401
from . import debugging  # noqa: F401
from .amp_lists import white_list, black_list  # noqa: F401
from ..ops.fp8 import fp8_autocast, DelayedScaling  # noqa: F401  (fp8 training: ops/fp8.py)
