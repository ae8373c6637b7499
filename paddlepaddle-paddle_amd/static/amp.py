"""paddle.static.amp — mixed precision for static Programs (O1 / O2, float16 / bfloat16).

Reference: python/paddle/static/amp/decorator.py:891 (``decorate``), :86 (``OptimizerWithMixedPrecision``:
``minimize``/``amp_init``/``get_loss_scaling``, dynamic loss scaling with
``check_finite_and_unscale`` + ``update_loss_scaling``), fp16_utils.py (``cast_model_to_fp16``,
``cast_parameters_to_fp16``, ``fp16_guard``), bf16/ (``decorate_bf16``, ``AutoMixedPrecisionListsBF16``,
``bf16_guard``).

Design here: the reference rewrites the ProgramDesc, inserting ``cast`` ops around white/black-list
ops.  Our Program is a recorded list of storage-layer ops replayed by the Executor, so the same
effect is obtained at replay time: a Program carrying an AMP config is executed under the storage
layer's autocast (white-list ops — matmul/linear/conv/attention — in the low-precision dtype,
black-list ops — softmax/norms/reductions/losses — in fp32).  O2 additionally casts the
program's parameters (normalisation parameters excepted) to the low-precision dtype, with fp32
master weights kept by the optimizer (``multi_precision``).  Loss scaling (dynamic for float16
by default) runs inside the recorded minimize node: scale → backward → unscale + finite check →
skip-or-step → scale update, exactly the reference's ``update_loss_scaling`` rule.
"""
import contextlib

import torch

from ..core import dtype as _dt
from ..amp.amp_lists import white_list as _white_list, black_list as _black_list
from ..core.tensor import register_param as _register_param


class AutoMixedPrecisionLists:
    """White / black / gray op-name lists (reference fp16_lists.py AutoMixedPrecisionLists)."""

    def __init__(self, custom_white_list=None, custom_black_list=None, custom_black_varnames=None,
                 dtype='float16'):
        d = 'bfloat16' if 'bf' in str(dtype) else 'float16'
        self.amp_dtype = d
        self.white_list = set(_white_list()[d]['O1'])
        self.black_list = set(_black_list()[d]['O1'])
        self.gray_list = set()
        self.black_varnames = set(custom_black_varnames or [])
        for op in custom_white_list or []:
            self.white_list.add(op)
            self.black_list.discard(op)
        for op in custom_black_list or []:
            self.black_list.add(op)
            self.white_list.discard(op)


CustomOpLists = AutoMixedPrecisionLists


def _is_norm_param(p):
    name = (getattr(p, 'name', None) or '').lower()
    return 'norm' in name or name.startswith('bn') or '_bn' in name


def cast_parameters_to_fp16(place=None, program=None, scope=None, to_fp16_var_names=None, dtype=torch.float16):
    """Casts the program's floating parameters (normalisation ones excepted) in place."""
    from .program import default_main_program
    program = program or default_main_program()
    names = set(to_fp16_var_names) if to_fp16_var_names else None
    n = 0
    for p in program.all_parameters():
        t = p._t
        if not t.is_floating_point() or t.dtype == dtype or _is_norm_param(p):
            continue
        if names is not None and p.name not in names:
            continue
        req = t.requires_grad
        with torch.no_grad():
            p._t = t.detach().to(dtype).requires_grad_(req)
        _register_param(p)
        n += 1
    return n


def cast_parameters_to_bf16(place=None, program=None, scope=None, to_bf16_var_names=None):
    return cast_parameters_to_fp16(place, program, scope, to_bf16_var_names, dtype=torch.bfloat16)


def cast_model_to_fp16(program, amp_lists=None, use_fp16_guard=True, dest_type='float16', level='O2',
                       use_promote=False):
    """Marks ``program`` for low-precision replay (the reference inserts cast ops instead)."""
    program._amp = {'level': level, 'dtype': _dt.to_torch_dtype(dest_type), 'lists': amp_lists}
    return set()


def cast_model_to_bf16(program, startup_prog=None, amp_lists=None, use_bf16_guard=True):
    return cast_model_to_fp16(program, amp_lists, use_bf16_guard, 'bfloat16', 'O2')


@contextlib.contextmanager
def fp16_guard():
    yield


bf16_guard = fp16_guard


class OptimizerWithMixedPrecision:
    def __init__(self, optimizer, amp_lists, level, dtype, init_loss_scaling, use_dynamic_loss_scaling,
                 incr_every_n_steps, decr_every_n_nan_or_inf, incr_ratio, decr_ratio, master_weight=None,
                 use_promote=False, fp8_recipe=None):
        self._optimizer = optimizer
        self._fp8 = fp8_recipe
        self._amp_lists = amp_lists or AutoMixedPrecisionLists(dtype=dtype)
        self._level = level
        self._dtype = _dt.to_torch_dtype(dtype)
        is_fp16 = self._dtype == torch.float16
        if use_dynamic_loss_scaling is None:
            use_dynamic_loss_scaling = is_fp16
        self._use_scaling = is_fp16 or bool(use_dynamic_loss_scaling)
        self._dynamic = bool(use_dynamic_loss_scaling)
        self._scale_host = float(init_loss_scaling) if self._use_scaling else 1.0
        self._scale_t = None   # device-resident loss scale (+ good / bad step counters), created
        self._counts_t = None  # on the first scaled backward, updated by csrc/amp.hip
        self._incr_every = incr_every_n_steps
        self._decr_every = decr_every_n_nan_or_inf
        self._incr_ratio = incr_ratio
        self._decr_ratio = decr_ratio
        self._good = 0
        self._bad = 0
        self._master_weight = True if master_weight is None else bool(master_weight)
        self._program = None
        self._params = None
        self._casted = False
        self.found_inf = False

    def __getattr__(self, name):  # get_lr, set_lr_scheduler, state_dict, ...
        return getattr(self.__dict__['_optimizer'], name)

    @property
    def _scale(self):
        if self._scale_t is not None:
            return float(self._scale_t.item())
        return self._scale_host

    @_scale.setter
    def _scale(self, v):
        self._scale_host = float(v)
        if self._scale_t is not None:
            self._scale_t.fill_(float(v))

    def get_loss_scaling(self):
        return torch.tensor([self._scale], dtype=torch.float32)

    def _state(self, dev):
        if self._scale_t is None or self._scale_t.device != dev:
            self._scale_t = torch.full((1,), self._scale_host, dtype=torch.float32, device=dev)
            self._counts_t = torch.tensor([float(self._good), float(self._bad)], dtype=torch.float32, device=dev)
        return self._scale_t

    def _cast_params(self):
        if self._level == 'O2' and not self._casted and self._program is not None:
            cast_parameters_to_fp16(program=self._program, dtype=self._dtype)
            self._optimizer._multi_precision = self._master_weight
            self._casted = True

    def minimize(self, loss, startup_program=None, parameter_list=None, no_grad_set=None):
        from .program import default_main_program, _static_minimize
        prog = default_main_program()
        prog._amp = {'level': self._level, 'dtype': self._dtype, 'lists': self._amp_lists, 'fp8': self._fp8}
        self._program = prog
        opt_ops, params_grads = _static_minimize(self._optimizer, loss, parameter_list, no_grad_set)
        prog.nodes[-1].target = self  # executed through _static_minimize_exec (loss scaling)
        self._params = [p for p, _ in params_grads]
        self._cast_params()
        return opt_ops, params_grads

    def amp_init(self, place=None, scope=None, test_program=None, use_fp16_test=False):
        """Casts the parameters for O2 (idempotent: minimize already did on this runtime)."""
        self._cast_params()
        if test_program is not None and use_fp16_test:
            test_program._amp = dict(self._program._amp)

    # ---- executed by the Executor for the recorded minimize node
    def _static_minimize_exec(self, loss):
        self._scaled_backward(loss)
        self._apply_update()

    def _scaled_backward(self, loss, div=1.0):
        """backward of loss * scale / div (gradients accumulate; static.minimize.StaticMinimize
        splits the step so gradient merge / data-parallel reduction run in between)."""
        if not self._use_scaling and div == 1.0:
            loss.backward()
            return
        if not self._use_scaling:
            (loss.float() / div).backward()
            return
        sc = self._state(loss.device)  # device scale: no host read
        (loss.float() * (sc / div)).backward()

    def _apply_update(self, sync_found_inf=None):
        """Unscale, check for inf/nan (``sync_found_inf``: a callable reducing the flag over the
        data-parallel ranks), step unless found, clear, update the dynamic loss scale."""
        if not self._use_scaling:
            self._optimizer.step()
            release_grads(self._optimizer)
            return
        params = [p._t for p in (self._params or []) if p._t.requires_grad]
        grads = [t.grad for t in params if t.grad is not None]
        dev = grads[0].device if grads else (params[0].device if params else torch.device('cpu'))
        from ..ops.amp import check_finite_and_unscale_, update_loss_scaling_
        sc = self._state(dev)
        found_t = torch.zeros(1, dtype=torch.float32, device=dev)
        # one multi-tensor launch per 48 gradients (csrc/amp.hip): unscale + inf/nan flag on device
        check_finite_and_unscale_(grads, sc, found_t)
        found = bool(found_t.item() != 0)  # the one host read of the step: skip-or-step
        if sync_found_inf is not None:
            found = sync_found_inf(found)
            found_t.fill_(1.0 if found else 0.0)
        self.found_inf = found
        if not found:
            self._optimizer.step()
        release_grads(self._optimizer)
        if self._dynamic:
            cnt = self._counts_t
            update_loss_scaling_(found_t, sc, cnt[0:1], cnt[1:2], self._incr_every, self._decr_every,
                                 self._incr_ratio, self._decr_ratio)
            # host mirrors of the counters (state_dict / tests); the scale itself stays on device
            if found:
                self._good, self._bad = 0, (self._bad + 1) % max(1, self._decr_every)
            else:
                self._bad, self._good = 0, (self._good + 1) % max(1, self._incr_every)


def release_grads(opt):
    """End of a static training step: drop the gradients instead of zero-filling them.  A static
    program's gradients live for one step (the reference's append_backward creates them per step
    and only for parameters on the loss path), so the next backward assigns fresh ones — no fill
    kernel per parameter now and no accumulate-add per parameter then."""
    try:
        opt.clear_grad(set_to_zero=False)
    except TypeError:
        opt.clear_grad()


def decorate(optimizer, amp_lists=None, level='O1', dtype='float16', master_weight=None, master_grad=False,
             init_loss_scaling=2 ** 16, incr_every_n_steps=2000, decr_every_n_nan_or_inf=1, incr_ratio=2.0,
             decr_ratio=0.5, use_dynamic_loss_scaling=None, use_amp_guard=False, use_promote=False,
             use_pure_fp16=False, use_fp16_guard=None, use_bf16=False, use_fp8=False, fp8_recipe=None, **kw):
    """Static AMP decorator (reference static/amp/decorator.py:755).

    ``use_fp8=True`` (or ``dtype='float8_e4m3fn'``) additionally runs every recorded Linear /
    matmul whose weight is a trainable 2-D parameter through the fp8 path (ops/fp8.py: e4m3
    forward, e5m2 gradients, delayed scaling from ``fp8_recipe`` — a ``paddle.amp.DelayedScaling``);
    the remaining white-list ops run in bfloat16.  The reference framework has no fp8 AMP; this
    is the MI355X extension named by BASELINE config 5.
    """
    if str(dtype).lower().replace('paddle.', '') in ('float8_e4m3fn', 'fp8', 'float8'):
        use_fp8, dtype = True, 'bfloat16'
    if use_pure_fp16:
        level = 'O2'
    if use_bf16 or use_fp8:
        dtype = 'bfloat16'
    if level not in ('O1', 'O2', 'OD'):
        raise ValueError(f"static amp level must be O1/O2/OD, got {level}")
    recipe = None
    if use_fp8:
        from ..ops.fp8 import DelayedScaling
        recipe = fp8_recipe or DelayedScaling()
    return OptimizerWithMixedPrecision(optimizer, amp_lists, 'O1' if level == 'OD' else level, dtype,
                                       init_loss_scaling, use_dynamic_loss_scaling, incr_every_n_steps,
                                       decr_every_n_nan_or_inf, incr_ratio, decr_ratio, master_weight, use_promote,
                                       fp8_recipe=recipe)


class _BF16Namespace:  # paddle.static.amp.bf16
    AutoMixedPrecisionListsBF16 = staticmethod(
        lambda custom_bf16_list=None, custom_fp32_list=None, custom_fp32_varnames=None:
        AutoMixedPrecisionLists(custom_bf16_list, custom_fp32_list, custom_fp32_varnames, 'bfloat16'))
    bf16_guard = staticmethod(bf16_guard)
    cast_model_to_bf16 = staticmethod(cast_model_to_bf16)
    cast_parameters_to_bf16 = staticmethod(cast_parameters_to_bf16)

    @staticmethod
    def decorate_bf16(optimizer, amp_lists=None, use_pure_bf16=False, use_bf16_guard=None):
        return decorate(optimizer, amp_lists, level='O2' if use_pure_bf16 else 'O1', dtype='bfloat16')

    @staticmethod
    def rewrite_program_bf16(main_prog, amp_lists=None):
        cast_model_to_fp16(main_prog, amp_lists, dest_type='bfloat16', level='O1')


bf16 = _BF16Namespace()


@contextlib.contextmanager
def autocast_context(program, dev):
    """Replay context for a Program carrying an AMP config (used by the Executor)."""
    cfg = getattr(program, '_amp', None)
    if not cfg:
        yield None
        return
    from ..ops import fp8 as _fp8
    prev = _fp8._STATIC_RECIPE['recipe']
    _fp8._STATIC_RECIPE['recipe'] = cfg.get('fp8')
    if cfg.get('fp8') is not None and dev.type == 'cuda':
        _fp8.begin_static_step()  # this replay's weight casts: one launch
    try:
        with torch.autocast(device_type='cuda' if dev.type == 'cuda' else 'cpu', dtype=cfg['dtype']):
            yield _fp8.STATIC_SUBS if cfg.get('fp8') is not None else None
    finally:
        _fp8._STATIC_RECIPE['recipe'] = prev


class _FP8Namespace:  # paddle.static.amp.fp8
    @staticmethod
    def decorate_fp8(optimizer, amp_lists=None, fp8_recipe=None, use_pure_bf16=True, **kw):
        return decorate(optimizer, amp_lists, level='O2' if use_pure_bf16 else 'O1', use_fp8=True,
                        fp8_recipe=fp8_recipe, **kw)

    @staticmethod
    def DelayedScaling(*a, **k):
        from ..ops.fp8 import DelayedScaling
        return DelayedScaling(*a, **k)


fp8 = _FP8Namespace()
