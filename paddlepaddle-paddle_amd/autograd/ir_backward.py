"""Program-level reverse-mode differentiation entry points (reference:
python/paddle/autograd/ir_backward.py:1033 calc_gradient, calc_gradient_helper, :1078 grad).

In static mode these append gradient ops to the recorded program through
``paddle.static.gradients`` (static/program.py); in dygraph they defer to the tape
(``paddle.grad``)."""
__all__ = ['grad', 'calc_gradient', 'calc_gradient_helper']


def _as_list(x):
    if x is None:
        return []
    return list(x) if isinstance(x, (list, tuple)) else [x]


def _static():
    from ..framework import in_dynamic_mode
    return not in_dynamic_mode()


def calc_gradient_helper(outputs, inputs, grad_outputs=None, no_grad_set=None):
    """{input: [[gradient]]} ([] where the input does not reach the outputs)."""
    ins = _as_list(inputs)
    gs = calc_gradient(outputs, ins, grad_outputs, no_grad_set)
    return {id(i): ([[g]] if g is not None else []) for i, g in zip(ins, gs)}


def calc_gradient(outputs, inputs, grad_outputs, no_grad_set):
    outs, ins = _as_list(outputs), _as_list(inputs)
    gouts = _as_list(grad_outputs) or None
    if _static():
        from ..static.program import gradients
        return list(gradients(outs, ins, gouts, no_grad_set))
    from . import grad as _grad
    return list(_grad(outs, ins, gouts, retain_graph=True, allow_unused=True,
                      no_grad_vars=list(no_grad_set) if no_grad_set else None))


def grad(outputs, inputs, grad_outputs=None, retain_graph=None, create_graph=False, only_inputs=True,
         allow_unused=False, no_grad_vars=None):
    if _static():
        gs = calc_gradient(outputs, inputs, grad_outputs, no_grad_vars)
        if not allow_unused and any(g is None for g in gs):
            raise ValueError("some inputs do not reach the outputs; pass allow_unused=True")
        return gs
    from . import grad as _grad
    return _grad(outputs, inputs, grad_outputs, retain_graph, create_graph, only_inputs, allow_unused, no_grad_vars)
