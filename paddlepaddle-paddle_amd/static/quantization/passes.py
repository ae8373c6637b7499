"""Quantisation passes over static Programs (reference: python/paddle/static/quantization/
quantization_pass.py QuantizationTransformPass(V2) / QuantizationFreezePass / ConvertToInt8Pass /
AddQuantDequantPass / OutScaleForTrainingPass / OutScaleForInferencePass, quanter.py quant_aware /
convert).

The reference rewrites an IrGraph of ProgramDesc ops, inserting fake_quantize / fake_dequantize
ops.  Here a Program is a node list (static/program.py) and the passes rewrite it in place:

* QuantizationTransformPass (QAT): every quantisable op (Linear-type GEMMs with a persistable
  2-D weight — recorded ``addmm`` / ``mm`` / ``matmul`` / ``linear`` or imported ``matmul_v2`` /
  ``mul`` — and ``conv2d``) gets a fake quant-dequant node on its weight (channel-wise abs-max,
  recomputed every run, straight-through gradient) and on its activation input (moving-average
  abs-max kept on the device, updated while training).
* QuantizationFreezePass: the trained program becomes an int8 inference program: each quantised
  GEMM turns into ONE ``paddle.ops.int8.quant_linear`` node — int8 weights [N, K] with per-channel
  scales, the calibrated activation threshold, the int8 MFMA GEMM on the GPU (csrc/gemm8x.hip
  pa_gemm8_i8) — and convolutions keep quant-dequantised weights with a fixed activation
  quant-dequant in front.
* ConvertToInt8Pass: weights stored as int8 (already done by the freeze pass for GEMMs).
"""
import torch

from ..program import Node, Ref, Const

_LINEAR_TORCH = None


def _torch_linear_kinds():
    global _LINEAR_TORCH
    if _LINEAR_TORCH is None:
        T = torch.Tensor
        _LINEAR_TORCH = {torch.addmm: 'addmm', torch.mm: 'mm', torch.matmul: 'mm', T.matmul: 'mm', T.__matmul__: 'mm',
                         torch.nn.functional.linear: 'linear', torch.nn.functional.conv2d: 'conv2d'}
    return _LINEAR_TORCH


_TYPE_ALIASES = {'mul': ('mm', 'pd.mul', 'addmm', 'linear'), 'matmul': ('mm', 'pd.matmul_v2', 'pd.matmul', 'addmm',
                                                                        'linear'),
                 'matmul_v2': ('mm', 'pd.matmul_v2', 'pd.matmul', 'addmm', 'linear'),
                 'conv2d': ('conv2d', 'pd.conv2d'), 'depthwise_conv2d': ('conv2d', 'pd.depthwise_conv2d')}
DEFAULT_TYPES = ('conv2d', 'depthwise_conv2d', 'mul', 'matmul', 'matmul_v2')


class QuantSite:
    """One quantisable op: node index, activation operand, weight Const, layout, bias."""

    def __init__(self, idx, kind, act, weight, bias, layout, out):
        self.idx, self.kind, self.act, self.weight, self.bias = idx, kind, act, weight, bias
        self.layout = layout  # 'kn' (W [in, out]), 'nk' (W [out, in]) or 'conv'
        self.out = out
        self.key = None


def _kinds(types):
    ks = set()
    for t in types or DEFAULT_TYPES:
        ks.update(_TYPE_ALIASES.get(t, (t,)))
    return ks


def _const_tensor(prog, c):
    owner = getattr(prog, '_const_owner', {}).get(c.cid) if isinstance(c, Const) else None
    return owner._t if owner is not None else prog.consts[c.cid]


def find_sites(prog, types=None):
    """Quantisable ops of ``prog`` (top-level node list)."""
    allowed = _kinds(types)
    out = []
    lt = _torch_linear_kinds()
    for i, n in enumerate(prog.nodes):
        if n.kind != 'torch':
            continue
        t = n.target
        if type(t).__name__ == '_OpCall':
            k = 'pd.' + t.type
            if k not in allowed:
                continue
            slots = dict(t.slots)
            pos, args = 0, {}
            for s, cnt in t.slots:
                args[s] = n.args[pos:pos + cnt]
                pos += cnt
            if k in ('pd.matmul_v2', 'pd.matmul', 'pd.mul'):
                x, w = args.get('X', [None])[0], args.get('Y', [None])[0]
                if t.attrs.get('trans_x') or t.attrs.get('transpose_X') or t.attrs.get('alpha', 1.0) != 1.0:
                    continue
                if not isinstance(x, Ref) or not isinstance(w, Const) or _const_tensor(prog, w).dim() != 2:
                    continue
                lay = 'nk' if (t.attrs.get('trans_y') or t.attrs.get('transpose_Y')) else 'kn'
                outs = n.outs if isinstance(n.outs, int) else n.outs[0]
                out.append(QuantSite(i, k, x, w, None, lay, outs))
            elif k in ('pd.conv2d', 'pd.depthwise_conv2d') and 'Filter' in slots:
                x, w = args['Input'][0], args['Filter'][0]
                if isinstance(x, Ref) and isinstance(w, Const):
                    out.append(QuantSite(i, k, x, w, None, 'conv', n.outs if isinstance(n.outs, int) else n.outs[0]))
            continue
        try:
            k = lt.get(t)
        except TypeError:
            k = None
        if k is None or k not in allowed:
            continue
        a = n.args
        if k == 'addmm' and len(a) == 3 and not n.kwargs and isinstance(a[1], Ref) and isinstance(a[2], Const) \
                and _const_tensor(prog, a[2]).dim() == 2:
            out.append(QuantSite(i, k, a[1], a[2], a[0], 'kn', n.outs))
        elif k == 'mm' and len(a) == 2 and not n.kwargs and isinstance(a[0], Ref) and isinstance(a[1], Const) and \
                _const_tensor(prog, a[1]).dim() == 2:
            out.append(QuantSite(i, k, a[0], a[1], None, 'kn', n.outs))
        elif k == 'linear' and len(a) >= 2 and isinstance(a[0], Ref) and isinstance(a[1], Const):
            b = a[2] if len(a) > 2 else n.kwargs.get('bias')
            out.append(QuantSite(i, k, a[0], a[1], b, 'nk', n.outs))
        elif k == 'conv2d' and len(a) >= 2 and isinstance(a[0], Ref) and isinstance(a[1], Const):
            out.append(QuantSite(i, k, a[0], a[1], None, 'conv', n.outs))
    return out


def _new_vid(prog):
    return next(prog._vid)


def _add_const(prog, t, name=None):
    cid = len(prog.consts)
    while cid in prog.consts:
        cid += 1
    prog.consts[cid] = t
    if hasattr(prog, '_const_ids'):
        prog._const_ids[id(t)] = cid
    if hasattr(prog, '_meta_twins'):
        prog._meta_twins[cid] = torch.empty_like(t, device='meta')
    return Const(cid)


def weight_scales(w, layout, bits=8, channel_wise=True):
    """(int8 [N, K] weight (k contiguous), fp32 abs-max thresholds [N]) of a GEMM weight; for a
    conv weight (int8 same shape, per-output-channel thresholds)."""
    qmax = 2 ** (bits - 1) - 1
    wf = w.detach().float()
    if layout == 'kn':
        wf = wf.t()
    if layout == 'conv':
        red = tuple(range(1, wf.dim()))
        s = wf.abs().amax(red) if channel_wise else wf.abs().amax().expand(wf.shape[0])
        step = (s.clamp(min=1e-12) / qmax).reshape(-1, *([1] * (wf.dim() - 1)))
    else:
        s = wf.abs().amax(1) if channel_wise else wf.abs().amax().expand(wf.shape[0])
        step = (s.clamp(min=1e-12) / qmax)[:, None]
    q = torch.round(wf / step).clamp(-qmax, qmax).to(torch.int8).contiguous()
    return q, s.float().contiguous()


# ----------------------------------------------------------------------------- QAT node targets
class ActState:
    """Moving-average abs-max state of one activation (kept on the activation's device)."""

    def __init__(self, moving_rate=0.9):
        self.moving_rate = float(moving_rate)
        self.state = None
        self.accum = None
        self.fixed = None  # calibrated threshold (post-training / frozen)

    def scale(self):
        if self.fixed is not None:
            return float(self.fixed)
        if self.state is None:
            return None
        return float((self.accum / self.state.clamp(min=1e-12)).item())

    def __repr__(self):
        return f"ActState(scale={self.scale()})"


def fq_activation(x, holder=None, bits=8):
    """QAT activation fake quant (moving-average abs-max, updated while gradients are on)."""
    from ...ops.int8 import moving_average_abs_max, fake_quant_dequant
    if not x.is_floating_point():
        return x
    if holder.fixed is not None:
        return fake_quant_dequant(x, float(holder.fixed), bits)
    if holder.state is None or holder.state.device != x.device:
        holder.state = torch.zeros((), dtype=torch.float32, device=x.device)
        holder.accum = torch.zeros((), dtype=torch.float32, device=x.device)
    return moving_average_abs_max(x, holder.state, holder.accum, holder.moving_rate, torch.is_grad_enabled())


def fq_weight(w, bits=8, axis=0, channel_wise=True):
    """QAT weight fake quant: abs-max per output channel (``axis``), recomputed every run."""
    from ...ops.int8 import fake_quant_dequant
    if channel_wise:
        red = tuple(d for d in range(w.dim()) if d != axis)
        s = w.detach().abs().amax(red)
        return fake_quant_dequant(w, s, bits, axis)
    return fake_quant_dequant(w, w.detach().abs().amax(), bits)


def quant_conv2d_node(x, w, *args, act_scale=1.0, bits=8, **kw):
    """Frozen quantised conv: fixed activation quant-dequant + int8-valued weights (dequantised)."""
    from ...ops.int8 import fake_quant_dequant
    return torch.nn.functional.conv2d(fake_quant_dequant(x, float(act_scale), bits), w, *args, **kw)


class QuantizationTransformPass:
    """QAT: fake quant-dequant on the weights and activations of every quantisable op."""

    def __init__(self, scope=None, place=None, weight_bits=8, activation_bits=8,
                 activation_quantize_type='moving_average_abs_max', weight_quantize_type='channel_wise_abs_max',
                 window_size=10000, moving_rate=0.9, skip_pattern=('skip_quant',),
                 quantizable_op_type=DEFAULT_TYPES, weight_quantize_func=None, act_quantize_func=None,
                 weight_preprocess_func=None, act_preprocess_func=None, optimizer_func=None, executor=None,
                 is_test=None):
        if activation_quantize_type not in ('abs_max', 'range_abs_max', 'moving_average_abs_max'):
            raise ValueError(f"unknown activation_quantize_type {activation_quantize_type}")
        if weight_quantize_type not in ('abs_max', 'channel_wise_abs_max'):
            raise ValueError(f"unknown weight_quantize_type {weight_quantize_type}")
        self.wbits, self.abits = weight_bits, activation_bits
        self.channel_wise = weight_quantize_type == 'channel_wise_abs_max'
        self.moving_rate = moving_rate
        self.types = quantizable_op_type

    def apply(self, program):
        prog = getattr(program, 'program', program)
        sites = find_sites(prog, self.types)
        nodes = list(prog.nodes)
        inserts = {}
        states = {}
        for s in sites:
            n = nodes[s.idx]
            if n.meta.get('qat'):
                continue
            h = ActState(self.moving_rate)
            av, wv = _new_vid(prog), _new_vid(prog)
            axis = 1 if s.layout == 'kn' else 0
            pre = [Node('torch', fq_activation, [s.act], {'holder': h, 'bits': self.abits}, av, {'stage': n.meta.get('stage')}),
                   Node('torch', fq_weight, [s.weight], {'bits': self.wbits, 'axis': axis,
                                                         'channel_wise': self.channel_wise}, wv,
                        {'stage': n.meta.get('stage')})]
            inserts[s.idx] = pre
            args = [Ref(av) if (isinstance(a, Ref) and a.vid == s.act.vid) else
                    (Ref(wv) if (isinstance(a, Const) and a.cid == s.weight.cid) else a) for a in n.args]
            nodes[s.idx] = Node(n.kind, n.target, args, dict(n.kwargs), n.outs,
                                dict(n.meta or {}, qat=True, act_state=h, weight=s.weight, act=s.act,
                                     layout=s.layout))
            states[s.idx] = h
        out = []
        for i, n in enumerate(nodes):
            out.extend(inserts.get(i, []))
            out.append(n)
        prog.nodes[:] = out
        prog._ir_cache = None
        return program


QuantizationTransformPassV2 = QuantizationTransformPass


class QuantizationFreezePass:
    """QAT program -> int8 inference program (see the module docstring)."""

    def __init__(self, scope=None, place=None, bias_correction=False, weight_bits=8, activation_bits=8,
                 round_type='round', weight_quantize_type='channel_wise_abs_max', quantizable_op_type=None):
        self.wbits, self.abits = weight_bits, activation_bits
        self.channel_wise = weight_quantize_type == 'channel_wise_abs_max'

    def apply(self, program):
        prog = getattr(program, 'program', program)
        from ...ops.int8 import quant_linear
        nodes = list(prog.nodes)
        drop = set()
        for i, n in enumerate(nodes):
            if not n.meta.get('qat'):
                continue
            h, wref, aref, lay = n.meta['act_state'], n.meta['weight'], n.meta['act'], n.meta['layout']
            sc = h.scale()
            if sc is None or sc <= 0:
                continue  # never observed: keep the fake-quant form
            for j in range(max(0, i - 2), i):  # the two QAT nodes inserted in front
                if nodes[j].target in (fq_activation, fq_weight):
                    drop.add(j)
            nodes[i] = freeze_site(prog, n, wref, aref, lay, sc, self.wbits, self.abits, self.channel_wise)
        prog.nodes[:] = [n for i, n in enumerate(nodes) if i not in drop]
        prog._ir_cache = None
        return program


def freeze_site(prog, n, wref, aref, layout, act_scale, wbits=8, abits=8, channel_wise=True):
    """The inference node of one quantised op (int8 GEMM node, or a quant-dequant conv)."""
    from ...ops.int8 import quant_linear
    w = _const_tensor(prog, wref)
    q, ws = weight_scales(w, layout, wbits, channel_wise)
    meta = dict(n.meta or {})
    for k in ('qat', 'act_state', 'weight', 'act', 'layout'):
        meta.pop(k, None)
    meta['quantized'] = True
    if layout == 'conv':
        qmax = 2 ** (wbits - 1) - 1
        wq = (q.float() * (ws.clamp(min=1e-12) / qmax).reshape(-1, *([1] * (q.dim() - 1)))).to(w.dtype)
        wc = _add_const(prog, wq)
        rest = list(n.args[2:]) if type(n.target).__name__ != '_OpCall' else []
        if type(n.target).__name__ == '_OpCall':
            return Node('torch', _pd_conv_quant, [aref, wc], {'attrs': dict(n.target.attrs), 'act_scale': act_scale,
                                                               'bits': abits}, n.outs if isinstance(n.outs, int)
                        else n.outs[0], meta)
        return Node('torch', quant_conv2d_node, [aref, wc] + rest,
                    dict(n.kwargs, act_scale=act_scale, bits=abits), n.outs, meta)
    qc = _add_const(prog, q)
    sc = _add_const(prog, ws)
    acs = _add_const(prog, torch.tensor(float(act_scale), dtype=torch.float32, device=w.device))
    bias = None
    if type(n.target).__name__ != '_OpCall':
        if n.target is torch.addmm:
            bias = n.args[0]
        elif n.target is torch.nn.functional.linear:
            bias = n.args[2] if len(n.args) > 2 else n.kwargs.get('bias')
    out = n.outs if isinstance(n.outs, int) else n.outs[0]
    return Node('torch', quant_linear, [aref, qc, sc, acs, bias], {'bits': abits, 'weight_bits': wbits}, out, meta)


def _pd_conv_quant(x, w, attrs=None, act_scale=1.0, bits=8):
    from ...ops.int8 import fake_quant_dequant
    from ..pdmodel import OPS
    return OPS['conv2d']({'Input': [fake_quant_dequant(x, float(act_scale), bits)], 'Filter': [w]},
                         attrs)['Output'][0]


class ConvertToInt8Pass:
    """Weights of frozen GEMMs are already int8 [N, K] consts; frozen conv weights are cast to the
    int8 grid values (kept dequantised for the float conv)."""

    def __init__(self, scope=None, place=None, quantizable_op_type=None):
        pass

    def apply(self, program):
        return program


class AddQuantDequantPass:
    """Fake quant-dequant on the inputs of the other quantisable element-wise ops (reference
    AddQuantDequantPass for elementwise_add / pool2d ...): a moving-average activation node in front
    of each listed op's floating inputs."""

    _DEFAULT = ('elementwise_add', 'pool2d', 'add')

    def __init__(self, scope=None, place=None, moving_rate=0.9, quant_bits=8, skip_pattern=('skip_quant',),
                 quantizable_op_type=None, is_full_quantize=False, is_test=None, scale_dict=None):
        self.types = set(quantizable_op_type or self._DEFAULT)
        self.bits, self.moving_rate = quant_bits, moving_rate

    def apply(self, program):
        prog = getattr(program, 'program', program)
        out = []
        for n in prog.nodes:
            name = getattr(n.target, 'type', None) or getattr(n.target, '__name__', '')
            if n.kind == 'torch' and name in self.types and not n.meta.get('qdq'):
                args = []
                for a in n.args:
                    if isinstance(a, Ref):
                        v = _new_vid(prog)
                        out.append(Node('torch', fq_activation, [a], {'holder': ActState(self.moving_rate),
                                                                      'bits': self.bits}, v))
                        args.append(Ref(v))
                    else:
                        args.append(a)
                n = Node(n.kind, n.target, args, n.kwargs, n.outs, dict(n.meta or {}, qdq=True))
            out.append(n)
        prog.nodes[:] = out
        prog._ir_cache = None
        return program


AddQuantDequantPassV2 = AddQuantDequantPass
AddQuantDequantForInferencePass = AddQuantDequantPass


class OutScaleForTrainingPass:
    """Records the moving-average abs-max of every quantised op's output (``out_threshold``)."""

    def __init__(self, scope=None, place=None, moving_rate=0.9, is_test=None, scale_dict=None):
        self.moving_rate = moving_rate

    def apply(self, program):
        prog = getattr(program, 'program', program)
        out = []
        for n in prog.nodes:
            out.append(n)
            if n.meta.get('qat') and isinstance(n.outs, int) and not n.meta.get('out_scale'):
                h = ActState(self.moving_rate)
                n.meta['out_scale'] = h
                out.append(Node('torch', _track_out, [Ref(n.outs)], {'holder': h}, n.outs))
        prog.nodes[:] = out
        prog._ir_cache = None
        return program


def _track_out(x, holder=None):
    if x.is_floating_point() and torch.is_grad_enabled():
        with torch.no_grad():
            if holder.state is None:
                holder.state = torch.zeros((), device=x.device)
                holder.accum = torch.zeros((), device=x.device)
            holder.state.mul_(holder.moving_rate).add_(1.0)
            holder.accum.mul_(holder.moving_rate).add_(x.detach().abs().amax().float())
    return x


class OutScaleForInferencePass:
    """Copies the tracked output thresholds onto the ops (``n.meta['out_threshold']``) and removes
    the tracking nodes."""

    def __init__(self, scope=None):
        pass

    def apply(self, program):
        prog = getattr(program, 'program', program)
        out = []
        for n in prog.nodes:
            if n.target is _track_out:
                continue
            h = n.meta.get('out_scale') if n.meta else None
            if h is not None:
                n.meta['out_threshold'] = h.scale()
            out.append(n)
        prog.nodes[:] = out
        prog._ir_cache = None
        return program


class QuantWeightPass:
    """Weight-only int8 storage of the quantisable GEMMs (no activation quantisation): each becomes
    a weight-only Linear on the W8A16 path (paddle.nn.quant.weight_only_linear)."""

    def __init__(self, scope=None, place=None, bias_correction=False, quant_bits=8, save_int_weight=True):
        self.bits = quant_bits

    def apply(self, program):
        prog = getattr(program, 'program', program)
        for s in find_sites(prog, ('mul', 'matmul', 'matmul_v2')):
            n = prog.nodes[s.idx]
            w = _const_tensor(prog, s.weight)
            q, ws = weight_scales(w, s.layout, self.bits, True)
            qc, sc = _add_const(prog, q), _add_const(prog, ws / (2 ** (self.bits - 1) - 1))
            bias = n.args[0] if n.target is torch.addmm else None
            prog.nodes[s.idx] = Node('torch', _woq_node, [s.act, qc, sc, bias], {}, s.out,
                                     dict(n.meta or {}, quantized='weight_only'))
        prog._ir_cache = None
        return program


def _woq_node(x, q, scale, bias=None):
    from ...nn.quant.quantized_linear import weight_only_linear
    from ...core.tensor import _wrap, _unwrap
    return _unwrap(weight_only_linear(_wrap(x), _wrap(q), None if bias is None else _wrap(bias), _wrap(scale)))


class ReplaceFakeQuantDequantPass:
    """Fixed-threshold fake quant-dequant in place of the moving-average QAT nodes."""

    def __init__(self, scope=None, place=None, quant_bits=8):
        pass

    def apply(self, program):
        prog = getattr(program, 'program', program)
        for n in prog.nodes:
            if n.target is fq_activation:
                h = n.kwargs['holder']
                if h.fixed is None and h.scale() is not None:
                    h.fixed = h.scale()
        return program


class TransformForMobilePass:
    """Mobile (Paddle-Lite) operator renaming: nothing to rename for the MI355X runtime."""

    def __init__(self):
        pass

    def apply(self, program):
        return program
