"""Rule-based tensor-parallel planner — fully automatic placements for ``dist.to_static``
(reference: python/paddle/distributed/auto_parallel/static/tuner/rule_based_tuner.py — QKVPattern,
FFNPattern, RowMatmulPattern over the program graph — and static/planner_v2.py, which runs it when
``strategy.auto_mode == 'full'``).

The model's forward is recorded once into a throwaway static Program (the same recorder the static
path uses), so the patterns are matched on the op graph, not on module names:

* **FFN** — a weight matmul B whose activation operand comes, through elementwise ops only
  (activations, bias adds, dropout, casts, reshapes, the product of two branches as in SwiGLU),
  from one or more weight matmuls A_i with out-features == B's in-features: every A_i column
  parallel (weight ``Shard(out)``, bias ``Shard(0)``), B row parallel (weight ``Shard(in)``).
* **Attention** — the same, but the path may also hold the attention core (reshape / transpose
  into heads, activation x activation matmuls, softmax, additive masks, scaled-dot-product
  attention): separate q / k / v
  projections column parallel, the output projection row parallel; the head split of the reshape
  keeps the shard on the heads axis (auto_parallel_spmd reshape rule).

Only ops the SPMD propagation has a rule for may sit inside a match (a fused qkv split by
``split`` / ``chunk``, or a fused attention op without a rule, leaves the block replicated): an op
without a rule runs on local pieces, which is only exact on replicated values.

Matches are taken in program order and never overlap, so a stack of blocks alternates column /
row per block and a weight feeding a row-parallel layer is never re-planned.  Everything else stays
replicated; the SPMD propagation (auto_parallel_spmd) inserts the reshards the placements need, so
a plan only affects speed, never the math.  Weights whose sharded extent does not divide by the
model-parallel degree are left replicated.
"""
import torch

from ... import auto_parallel_spmd as _spmd

# Only ops the SPMD propagation has a rule for may sit inside a matched block: an op without one
# runs on the local pieces and drops the dist attribute, which is only safe on replicated values.
# Ops that keep a value's feature axis aligned with the producing matmul's output features:
_ELEMENTWISE = set(_spmd._EW) | set(_spmd._UNARY) | {'reshape', 'view'}
# plus, inside an attention block, the per-head core (head split / merge, QK^T and PV, softmax)
_ATTENTION = _ELEMENTWISE | set(_spmd._MATMUL) | set(_spmd._SOFTMAX) | {'transpose', 'permute', 't',
                                                                         'scaled_dot_product_attention'}
_WEIGHT_MM = {'addmm', 'mm', 'matmul', 'linear'}


def _name(n):
    return _spmd._norm_name(n.target) if n.target is not None else ''


class Plan(dict):
    """{parameter name: placements}; ``patterns`` lists the matches as (kind, [names])."""

    def __init__(self):
        super().__init__()
        self.patterns = []


class RuleBasedPlanner:
    """Plans tensor-parallel placements for ``layer`` on ``mesh`` (model-parallel axis ``mp_axis``:
    the dim named 'mp' / 'tp' / 'model', else the last one)."""

    def __init__(self, mesh, mp_axis=None):
        self.mesh = mesh
        names = list(getattr(mesh, 'dim_names', None) or [])
        if mp_axis is None:
            mp_axis = next((names.index(n) for n in ('mp', 'tp', 'model') if n in names), mesh.ndim - 1)
        elif isinstance(mp_axis, str):
            mp_axis = names.index(mp_axis)
        self.axis = int(mp_axis)
        self.degree = int(mesh.shape[self.axis])

    # ------------------------------------------------------------------ recording
    def _record(self, layer, inputs):
        from ... import fleet  # noqa: F401  (paddle.distributed import side effects)
        from .... import static as _st
        from .... import framework as _fw
        from ....core.tensor import Tensor, _unwrap
        vals = [_unwrap(a) if isinstance(a, Tensor) else torch.as_tensor(a) for a in inputs]
        dt = {torch.float32: 'float32', torch.float16: 'float16', torch.bfloat16: 'bfloat16', torch.int64: 'int64',
              torch.int32: 'int32', torch.float64: 'float64', torch.bool: 'bool'}
        was_dynamic = _fw.in_dynamic_mode()
        if was_dynamic:
            _fw.enable_static()
        try:
            main, startup = _st.Program(), _st.Program()
            with _st.program_guard(main, startup):
                feeds = [_st.data(f'plan_in_{i}', list(v.shape), dt[v.dtype]) for i, v in enumerate(vals)]
                with torch.no_grad():
                    layer(*feeds)
        finally:
            if was_dynamic:
                _fw.disable_static()
        return main

    # ------------------------------------------------------------------ matching
    def _weight_mm(self, prog, n):
        """(weight param, bias param | None, activation Ref, torch layout) of a weight matmul node."""
        from ....static.program import Const, Ref
        nm = _name(n)
        if n.kind != 'torch' or nm not in _WEIGHT_MM:
            return None
        owner = getattr(prog, '_const_owner', {})
        a = list(n.args)
        if nm == 'addmm' and len(a) >= 3:
            b, x, w = a[0], a[1], a[2]
            layout_t = False
        elif nm == 'linear' and len(a) >= 2:
            x, w = a[0], a[1]
            b = a[2] if len(a) > 2 else n.kwargs.get('bias')
            layout_t = True
        elif len(a) >= 2:
            x, w, b = a[0], a[1], None
            layout_t = False
        else:
            return None
        if not (isinstance(w, Const) and isinstance(x, Ref)):
            return None
        wp = owner.get(w.cid)
        if wp is None or len(wp.shape) != 2:
            return None
        bp = owner.get(b.cid) if isinstance(b, Const) else None
        return wp, bp, x, layout_t

    def _leaves(self, prog, producer, vid, allowed, seen):
        """Weight-matmul nodes reached backwards from value ``vid`` through ``allowed`` ops only
        (None when the path leaves the set or reaches a program input)."""
        from ....static.program import Ref
        if vid in seen:
            return set()
        seen.add(vid)
        ni = producer.get(vid)
        if ni is None:
            return set()  # a fed value (input, mask): replicated, broadcast by the SPMD rules
        n = prog.nodes[ni]
        if self._weight_mm(prog, n) is not None:
            return {ni}
        if n.kind != 'torch' or _name(n) not in allowed:
            return None
        out = set()
        refs = [a for a in list(n.args) + list(n.kwargs.values()) if isinstance(a, Ref)]
        for a in list(n.args) + list(n.kwargs.values()):
            if isinstance(a, (list, tuple)):
                refs += [r for r in a if isinstance(r, Ref)]
        for r in refs:
            sub = self._leaves(prog, producer, r.vid, allowed, seen)
            if sub is None:
                return None
            out |= sub
        return out

    def plan(self, layer, *inputs):
        prog = self._record(layer, inputs)
        producer = {}
        for i, n in enumerate(prog.nodes):
            outs = n.outs if isinstance(n.outs, list) else [n.outs]
            for o in outs:
                if isinstance(o, int):
                    producer[o] = i
        names = {id(p): k for k, p in layer.named_parameters()}
        plan, used = Plan(), set()
        for i, n in enumerate(prog.nodes):
            wm = self._weight_mm(prog, n)
            if wm is None or i in used:
                continue
            wb, bb, x, tl_b = wm
            in_b = wb.shape[1] if tl_b else wb.shape[0]
            for kind, allowed in (('ffn', _ELEMENTWISE), ('attention', _ATTENTION)):
                leaves = self._leaves(prog, producer, x.vid, allowed, set())
                if not leaves or leaves & used:
                    continue
                cols = [self._weight_mm(prog, prog.nodes[j]) for j in sorted(leaves)]
                outs = [(w.shape[0] if tl else w.shape[1]) for w, _, _, tl in cols]
                if kind == 'ffn' and any(o != in_b for o in outs):
                    continue
                if kind == 'attention' and any(o != in_b for o in outs):
                    continue  # a fused qkv would be split by an op without an SPMD rule
                if in_b % self.degree or any(o % self.degree for o in outs):
                    continue
                if any(id(w) not in names for w, _, _, _ in cols) or id(wb) not in names:
                    continue
                for w, b, _, tl in cols:
                    plan[names[id(w)]] = self._pl(0 if tl else 1)
                    if b is not None and id(b) in names:
                        plan[names[id(b)]] = self._pl(0)
                plan[names[id(wb)]] = self._pl(1 if tl_b else 0)
                plan.patterns.append((kind, [names[id(w)] for w, _, _, _ in cols] + [names[id(wb)]]))
                used |= leaves | {i}
                break
        return plan

    def _pl(self, dim):
        from ..api import Replicate, Shard
        pl = [Replicate() for _ in range(self.mesh.ndim)]
        pl[self.axis] = Shard(dim)
        return pl

    # ------------------------------------------------------------------ application
    def apply(self, layer, plan, optimizer=None):
        """Replace the planned parameters by their dist tensors (and in ``optimizer``'s lists)."""
        from ..api import shard_tensor
        swap = {}
        for name, pl in plan.items():
            owner = layer
            *path, attr = name.split('.')
            for p in path:
                owner = getattr(owner, p)
            old = getattr(owner, attr)
            new = shard_tensor(old, self.mesh, pl)
            setattr(owner, attr, new)
            swap[id(old)] = new
        inner = getattr(optimizer, '_inner_opt', optimizer)
        if inner is not None and swap:
            for g in getattr(inner, '_param_groups', []) or []:
                g['params'] = [swap.get(id(p), p) for p in g['params']]
            if getattr(inner, '_parameter_list', None) is not None:
                inner._parameter_list = [swap.get(id(p), p) for p in inner._parameter_list]
        return swap


Planner = RuleBasedPlanner
