"""Program-pass framework (reference: python/paddle/distributed/passes/pass_base.py:20-420).

A pass is registered by name (``@register_pass``), created with ``new_pass(name, attrs)`` and
applied to lists of (main, startup) programs; ``PassContext`` records what was applied and
``PassManager`` orders a set of passes so that no pass runs after one it conflicts with (the
reference's longest-path solve over the pairwise "may follow" relation).
"""
from abc import ABC, abstractmethod


class PassContext:
    """What has been applied so far (in order) plus free-form attributes shared by passes."""

    def __init__(self):
        self._applied, self._attrs = [], {}

    def set_attr(self, key, value):
        self._attrs[key] = value

    def get_attr(self, key, default=None):
        return self._attrs.get(key, default)

    @property
    def passes(self):
        return self._applied

    def _add_pass(self, pass_obj):
        self._applied.append(pass_obj)

    def _pop_pass(self):
        self._applied.pop()


class PassType:
    UNKNOWN = 0
    COMM_OPT = 1
    CALC_OPT = 2
    PARALLEL_OPT = 3
    FUSION_OPT = 4


class PassBase(ABC):
    _REGISTERED_PASSES = {}
    _COMMON_RULES = []

    name = None

    @staticmethod
    def _register(pass_name, pass_class):
        if not issubclass(pass_class, PassBase):
            raise TypeError(f"{pass_class} is not a PassBase")
        PassBase._REGISTERED_PASSES[pass_name] = pass_class

    def __init__(self):
        self._attrs = {}

    def set_attr(self, key, value):
        self._attrs[key] = value
        return self

    def get_attr(self, key, default=None):
        return self._attrs.get(key, default)

    @abstractmethod
    def _check_self(self):
        """Whether the attributes make this pass applicable."""

    @abstractmethod
    def _check_conflict(self, other_pass):
        """Whether this pass may run after ``other_pass``."""

    def _type(self):
        return PassType.UNKNOWN

    def _check_conflict_including_common_rules(self, other_pass):
        return self._check_conflict(other_pass) and all(r(other_pass, self) for r in PassBase._COMMON_RULES)

    def apply(self, main_programs, startup_programs, context=None):
        if context is None:
            context = PassContext()
        if not self._check_self():
            return context
        if not all(self._check_conflict_including_common_rules(p) for p in context.passes):
            return context
        if not isinstance(main_programs, list) or not isinstance(startup_programs, list):
            raise TypeError("apply() takes lists of main and startup programs")
        if len(main_programs) != len(startup_programs):
            raise ValueError("main and startup program lists differ in length")
        self._apply_impl(main_programs, startup_programs, context)
        context._add_pass(self)
        return context

    def _apply_impl(self, main_programs, startup_programs, context):
        for main_program, startup_program in zip(main_programs, startup_programs):
            self._apply_single_impl(main_program, startup_program, context)

    @abstractmethod
    def _apply_single_impl(self, main_program, startup_program, context):
        """Rewrite one (main, startup) program pair."""


def register_pass(name):
    def impl(cls):
        PassBase._register(name, cls)
        cls.name = name
        return cls

    return impl


def new_pass(name, pass_attrs={}):  # noqa: B006 (reference signature)
    pass_class = PassBase._REGISTERED_PASSES.get(name)
    if pass_class is None:
        raise AssertionError(f"Pass {name} is not registered")
    pass_obj = pass_class()
    for k, v in pass_attrs.items():
        pass_obj.set_attr(k, v)
    return pass_obj


def _fusion_opt_last_rule(pass_before, pass_after):
    """Fusion passes run after everything else."""
    return not (pass_before._type() == PassType.FUSION_OPT and pass_after._type() != PassType.FUSION_OPT)


def _make_rule_from_white_lists_dict(before_white_lists_dict, after_white_lists_dict):
    def rule(pass_before, pass_after):
        b = before_white_lists_dict.get(pass_after.name)
        if b is not None and pass_before.name not in b:
            return False
        a = after_white_lists_dict.get(pass_before.name)
        if a is not None and pass_after.name not in a:
            return False
        return True
    return rule


PassBase._COMMON_RULES = [_fusion_opt_last_rule]


def _find_longest_path(adjacent_matrix):
    """Longest path in the DAG given by adjacent_matrix[i][j] (i may precede j), over every start
    node; ties keep the lowest indices (the passes' given order)."""
    n = len(adjacent_matrix)
    best = {}

    def longest_from(i, visiting):
        if i in best:
            return best[i]
        visiting.add(i)
        path = [i]
        for j in range(n):
            if j != i and adjacent_matrix[i][j] and j not in visiting:
                cand = [i] + longest_from(j, visiting)
                if len(cand) > len(path):
                    path = cand
        visiting.discard(i)
        best[i] = path
        return path

    out = []
    for i in range(n):
        p = longest_from(i, set())
        if len(p) > len(out):
            out = p
    return out


def _solve_pass_conflict(passes, context):
    passes = [p for p in passes if p._check_self()]
    if not passes:
        return []
    old_passes = passes
    passes = []
    for p in old_passes:
        if all(p._check_conflict_including_common_rules(applied) for applied in context.passes):
            passes.append(p)
    if not passes:
        return []
    n = len(passes)
    adjacent_matrix = [[False] * n for _ in range(n)]
    for i in range(n):
        for j in range(n):
            adjacent_matrix[i][j] = passes[j]._check_conflict_including_common_rules(passes[i])
    return [passes[idx] for idx in _find_longest_path(adjacent_matrix)]


class PassManager:
    def __init__(self, passes, context=None, auto_solve_conflict=True):
        if context is None:
            context = PassContext()
        self._context = context
        self._passes = _solve_pass_conflict(passes, context) if auto_solve_conflict else list(passes)

    def apply(self, main_programs, startup_programs):
        context = self._context
        for p in self._passes:
            context = p.apply(main_programs, startup_programs, context)
        self._context = context
        return context

    @property
    def context(self):
        return self._context

    @property
    def names(self):
        return [p.name for p in self.passes]

    @property
    def passes(self):
        return tuple(self._passes)
