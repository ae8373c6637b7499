"""Concrete passes over this framework's recorded static programs.

The reference passes rewrite ProgramDesc ops (distributed/passes/auto_parallel_*.py,
fuse_all_reduce.py).  A program here is a recorded op list whose backward + optimizer update is
one ``minimize`` node; these passes configure how that node trains (static/minimize.py
StaticMinimize) or which precision its forward replays in (static/amp.py):

  auto_parallel_gradient_merge   k_steps / avg: accumulate k runs, update on the k-th
  auto_parallel_amp              O1 autocast (+ dynamic loss scaling for fp16)
  auto_parallel_fp16             O2: parameters cast to dtype (fp32 masters), loss scaling
  auto_parallel_bf16             O2 bfloat16 (the fp16 pass with dtype='bfloat16')
  auto_parallel_data_parallel_optimization / fuse_all_reduce
                                 gradients averaged over a process group in fused buckets,
                                 parameters broadcast from the group's first rank
  auto_parallel_grad_clip        gradient clipping (ClipGradBy*) applied by the update
"""
import torch.distributed as dist

from .core import PassBase, PassType, register_pass


def _policy(program):
    from ...static.minimize import step_policy
    return step_policy(program)


def _base_optimizer(pol):
    from ...static.amp import OptimizerWithMixedPrecision
    o = pol.inner_optimizer
    return o._optimizer if isinstance(o, OptimizerWithMixedPrecision) else o


@register_pass("auto_parallel_gradient_merge")
class GradientMergePass(PassBase):
    def __init__(self):
        super().__init__()
        self.set_attr("k_steps", -1)
        self.set_attr("avg", True)

    def _check_self(self):
        return int(self.get_attr("k_steps", -1)) > 1

    def _check_conflict(self, other_pass):
        return other_pass.name != self.name

    def _type(self):
        return PassType.CALC_OPT

    def _apply_single_impl(self, main_program, startup_program, context):
        pol = _policy(main_program)
        pol.k_steps = int(self.get_attr("k_steps"))
        pol.avg = bool(self.get_attr("avg", True))


class _AMPPassBase(PassBase):
    level = 'O1'

    def __init__(self):
        super().__init__()
        self.set_attr("dtype", "float16")
        self.set_attr("init_loss_scaling", 32768.0)
        self.set_attr("incr_every_n_steps", 1000)
        self.set_attr("decr_every_n_nan_or_inf", 2)
        self.set_attr("incr_ratio", 2.0)
        self.set_attr("decr_ratio", 0.8)
        self.set_attr("use_dynamic_loss_scaling", None)
        self.set_attr("custom_white_list", [])
        self.set_attr("custom_black_list", [])
        self.set_attr("custom_black_varnames", [])

    def _check_self(self):
        return str(self.get_attr("dtype")).replace('paddle.', '') in ('float16', 'bfloat16')

    def _check_conflict(self, other_pass):
        return not isinstance(other_pass, _AMPPassBase)

    def _type(self):
        return PassType.CALC_OPT

    def _apply_single_impl(self, main_program, startup_program, context):
        from ...static import amp as samp
        pol = _policy(main_program)
        if isinstance(pol.inner_optimizer, samp.OptimizerWithMixedPrecision):
            raise RuntimeError("the program's optimizer is already mixed-precision decorated")
        dtype = str(self.get_attr("dtype")).replace('paddle.', '')
        lists = samp.AutoMixedPrecisionLists(custom_white_list=self.get_attr("custom_white_list") or None,
                                             custom_black_list=self.get_attr("custom_black_list") or None,
                                             custom_black_varnames=self.get_attr("custom_black_varnames") or None,
                                             dtype=dtype)
        opt = pol.inner_optimizer
        amp = samp.decorate(opt, amp_lists=lists, level=self.level, dtype=dtype,
                            init_loss_scaling=self.get_attr("init_loss_scaling"),
                            use_dynamic_loss_scaling=self.get_attr("use_dynamic_loss_scaling"),
                            incr_every_n_steps=self.get_attr("incr_every_n_steps"),
                            decr_every_n_nan_or_inf=self.get_attr("decr_every_n_nan_or_inf"),
                            incr_ratio=self.get_attr("incr_ratio"), decr_ratio=self.get_attr("decr_ratio"))
        main_program._amp = {'level': amp._level, 'dtype': amp._dtype, 'lists': amp._amp_lists, 'fp8': None}
        amp._program = main_program
        amp._params = list(opt._parameter_list or [])
        amp._cast_params()
        pol._opt = amp


@register_pass("auto_parallel_amp")
class AMPPass(_AMPPassBase):
    level = 'O1'


@register_pass("auto_parallel_fp16")
class FP16Pass(_AMPPassBase):
    level = 'O2'


@register_pass("auto_parallel_bf16")
class BF16Pass(_AMPPassBase):
    level = 'O2'

    def __init__(self):
        super().__init__()
        self.set_attr("dtype", "bfloat16")
        self.set_attr("use_dynamic_loss_scaling", False)


@register_pass("auto_parallel_data_parallel_optimization")
class DataParallelOptimizationPass(PassBase):
    """attrs: group (paddle.distributed Group; default: every rank), fuse_grad_size_in_MB."""

    def __init__(self):
        super().__init__()
        self.set_attr("group", None)
        self.set_attr("fuse_grad_size_in_MB", 32)

    def _group(self):
        g = self.get_attr("group")
        if g is not None:
            return g
        if not dist.is_initialized() or dist.get_world_size() < 2:
            return None
        from ..communication import new_group
        return new_group(list(range(dist.get_world_size())))

    def _check_self(self):
        g = self.get_attr("group")
        return (g is not None and g.nranks > 1) or (dist.is_initialized() and dist.get_world_size() > 1)

    def _check_conflict(self, other_pass):
        return not isinstance(other_pass, DataParallelOptimizationPass)

    def _type(self):
        return PassType.COMM_OPT

    def _apply_single_impl(self, main_program, startup_program, context):
        from ..fleet import _broadcast_params
        pol = _policy(main_program)
        pol.dp_group = self._group()
        pol.fuse_grad_size_in_MB = float(self.get_attr("fuse_grad_size_in_MB", 32))
        if pol.dp_group is not None:
            _broadcast_params(pol._params(), pol.dp_group)


@register_pass("fuse_all_reduce")
class FuseAllReducePass(DataParallelOptimizationPass):
    """The data-parallel gradient reduction with the bucket size given as ``max_memory_size``
    (bytes, reference fuse_all_reduce.py) or ``fuse_grad_size_in_MB``."""

    def _apply_single_impl(self, main_program, startup_program, context):
        mx = self.get_attr("max_memory_size")
        if mx:
            self.set_attr("fuse_grad_size_in_MB", float(mx) / (1 << 20))
        super()._apply_single_impl(main_program, startup_program, context)


@register_pass("auto_parallel_grad_clip")
class GradClipPass(PassBase):
    """attrs: clip (paddle.nn.ClipGradByGlobalNorm / ByNorm / ByValue)."""

    def _check_self(self):
        return self.get_attr("clip") is not None

    def _check_conflict(self, other_pass):
        return True

    def _type(self):
        return PassType.CALC_OPT

    def _apply_single_impl(self, main_program, startup_program, context):
        _base_optimizer(_policy(main_program))._grad_clip = self.get_attr("clip")
