"""Registry of composite-op decomposition rules (reference: python/paddle/decomposition/register.py).

A rule is keyed by the reference operator name (``'pd_op.softmax'``) and is a Python function over
the recorded op's own arguments (torch-level: the same positional / keyword arguments the recorded
node carries) that computes the op from primitive tensor operations.  ``decompose`` traces the rule
on the node's meta values, so the primitives it calls are recorded as program nodes.
"""


class Registry:
    def __init__(self, name):
        self.name = name
        self.rules = {}

    def register(self, op_type, rule):
        if not isinstance(op_type, str) or not callable(rule):
            raise TypeError("register(op_type: str, rule: callable)")
        self.rules[op_type] = rule

    def lookup(self, op_type):
        return self.rules.get(op_type)

    def __contains__(self, op_type):
        return op_type in self.rules


_decomposition_ops = Registry('decomposition')


def register_decomp(op_type):
    """Decorator: ``@register_decomp('pd_op.softmax') def softmax(x, dim, ...)`` (a later
    registration of the same name replaces the earlier rule)."""
    def wrapper(f):
        _decomposition_ops.register(op_type, f)
        return f
    return wrapper


def get_decomp_rule(op_type):
    return _decomposition_ops.lookup(op_type)
