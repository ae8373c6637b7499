"""General and convolution IR passes over static Programs, registered into static/ir_passes.py.

Reference passes (same names):
  paddle/fluid/pir/transforms/general/constant_folding_pass.cc      constant_folding_pass
  paddle/fluid/pir/transforms/general/dead_code_elimination_pass.cc dead_code_elimination_pass
  paddle/fluid/pir/transforms/general/common_subexpression_elimination_pass.cc
                                                                    common_subexpression_elimination_pass
  paddle/fluid/pir/transforms/gpu/conv2d_bn_fuse_pass.cc            conv2d_bn_fuse_pass
  paddle/fluid/pir/transforms/gpu/conv2d_add_act_fuse_pass.cc       conv2d_add_act_fuse_pass
  paddle/fluid/framework/ir/embedding_eltwise_layernorm_fuse_pass.cc embedding_eltwise_layernorm_fuse_pass
  paddle/fluid/pir/transforms/gpu/fused_weight_only_linear_pass.cc  fused_weight_only_linear_pass

Design notes (MI355X): a convolution node, folded or not, runs on the hand-written implicit-GEMM
kernels (csrc/conv.hip, channels-last with NCHW served as views) whenever its operands fit, with
the bias in the kernel's epilogue; the folded batch norm costs nothing at run time (the predictor
of a ResNet runs no standalone batch-norm kernel), and the residual add + ReLU of a bottleneck
run in place on the conv output.  Folding and constant folding read parameter VALUES at rewrite
time, so they only apply to inference programs (no backward / minimize node); dead-code and
common-subexpression elimination are pure graph rewrites, safe for training programs too.
"""
import torch
import torch.nn.functional as TF

from .program import Node, Ref, Const
from . import ir_passes as IP

_RANDOM = ('rand', 'randn', 'randint', 'randperm', 'normal', 'bernoulli', 'dropout', 'multinomial', 'rand_like',
           'randn_like', 'randint_like', 'uniform', 'exponential', 'poisson', 'alpha_dropout', 'feature_alpha_dropout')


def _name(n):
    t = n.target
    if type(t).__name__ == '_OpCall':
        return 'pd.' + t.type
    return getattr(t, '__name__', '') or ''


def _pure(n):
    """A side-effect-free, deterministic torch node (safe to drop when unused, to merge when equal)."""
    if n.kind != 'torch':
        return False
    nm = _name(n)
    if nm.endswith('_') and not nm.endswith('__'):  # in-place method (add_, copy_, ...)
        return False
    if nm in ('__setitem__', 'copy_', 'set_', 'resize_', 'record_stream', 'backward'):
        return False
    if any(r in nm for r in _RANDOM):
        return False
    if nm.startswith('pd.'):
        return False  # imported operators may carry outputs bound by slot (kept)
    if n.kwargs.get('inplace') or n.kwargs.get('out') is not None:
        return False
    return True


def _training(prog):
    return any(n.kind in ('minimize', 'backward', 'grad') for n in prog.nodes)


def _refs(obj):
    out = []
    IP._refs_in(obj, out)
    return out


# ============================================================================ fused entry points
def conv2d_static(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1):
    """torch.conv2d semantics (NCHW) on the hand-written kernels when the operands fit
    (nn.functional.conv._conv routing), else torch."""
    from ..nn.functional.conv import _conv
    from ..core.tensor import _wrap, _unwrap
    return _unwrap(_conv(_wrap(x), _wrap(weight), None if bias is None else _wrap(bias), stride, padding, dilation,
                         groups, 'NCHW', 2, TF.conv2d))


def conv2d_add_act(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, residual=None, act=None):
    """conv2d (+ bias in the kernel epilogue) (+ residual) (-> relu), the add and the activation in
    place on the convolution's output."""
    y = conv2d_static(x, weight, bias, stride, padding, dilation, groups)
    if residual is not None:
        y = y + residual if y.requires_grad or residual.requires_grad else y.add_(residual)
    if act == 'relu':
        y = torch.relu(y) if y.requires_grad else y.relu_()
    return y


def embedding_sum_layer_norm(ids_list, tables, ln_weight, ln_bias, eps=1e-5, padding_idx=None):
    """sum_i embedding(ids_i, table_i) -> layer_norm over the last dim; the last add and the norm run
    as one fused add + LayerNorm kernel (csrc/norm.hip) on the GPU."""
    embs = [TF.embedding(i, t) for i, t in zip(ids_list, tables)]
    acc = embs[0]
    for e in embs[1:-1]:
        acc = acc + e
    if len(embs) > 1:
        return IP.fused_dropout_add_layer_norm(embs[-1], acc, ln_weight, ln_bias, eps, 0.0)[0]
    return IP.fused_layer_norm(acc, ln_weight, ln_bias, eps)


def const_value(c):
    """A constant-folded value (the node binds the precomputed tensor)."""
    return c


# ============================================================================ passes
_CONV = None


def _is_conv(n):
    global _CONV
    if _CONV is None:
        _CONV = {torch.conv2d, TF.conv2d, conv2d_static}
    return n is not None and n.kind == 'torch' and n.target in _CONV


def _conv_args(n):
    """(x, w, b, stride, padding, dilation, groups) of a recorded conv2d node."""
    names = ('input', 'weight', 'bias', 'stride', 'padding', 'dilation', 'groups')
    dflt = (None, None, None, 1, 0, 1, 1)
    vals = []
    for i, (nm, d) in enumerate(zip(names, dflt)):
        vals.append(n.args[i] if len(n.args) > i else n.kwargs.get(nm, d))
    if isinstance(vals[4], str):
        return None  # 'same' / 'valid' string padding: left to torch
    return vals


def _bn_args(n):
    """(x, mean, var, weight, bias, eps) of an inference batch norm node, else None."""
    if n.kind != 'torch':
        return None
    if n.target in (TF.batch_norm, torch.batch_norm):
        a, k = n.args, n.kwargs
        if n.target is torch.batch_norm:  # (input, weight, bias, mean, var, training, momentum, eps, cudnn)
            if len(a) < 8 or a[5]:
                return None
            return a[0], a[3], a[4], a[1], a[2], a[7]
        x = a[0]
        mean = a[1] if len(a) > 1 else k.get('running_mean')
        var = a[2] if len(a) > 2 else k.get('running_var')
        w = a[3] if len(a) > 3 else k.get('weight')
        b = a[4] if len(a) > 4 else k.get('bias')
        training = a[5] if len(a) > 5 else k.get('training', False)
        eps = a[7] if len(a) > 7 else k.get('eps', 1e-5)
        if training:
            return None
        return x, mean, var, w, b, eps
    return None


def _const_t(g, c):
    if isinstance(c, Const):
        owner = getattr(g.prog, '_const_owner', {}).get(c.cid)
        return owner._t if owner is not None else g.prog.consts[c.cid]
    return None


def _new_const(g, t):
    return Const(g.prog._const(t))


def _conv_bn(g, i):
    n = g.nodes[i]
    ba = _bn_args(n)
    if ba is None or _training(g.prog):
        return None
    x, mean, var, gw, gb, eps = ba
    if not isinstance(x, Ref):
        return None
    j = g.producer(x.vid, i)
    cn = g.node(j)
    if not _is_conv(cn) or not g.private([j], users=[i]):
        return None
    ca = _conv_args(cn)
    if ca is None or not isinstance(ca[1], Const) or (ca[2] is not None and not isinstance(ca[2], Const)):
        return None
    tw, tm, tv = _const_t(g, ca[1]), _const_t(g, mean), _const_t(g, var)
    if tw is None or tm is None or tv is None or (gw is not None and _const_t(g, gw) is None) or \
            (gb is not None and _const_t(g, gb) is None):
        return None
    with torch.no_grad():
        dt = tw.dtype
        inv = torch.rsqrt(tv.float() + float(eps))
        scale = inv * (_const_t(g, gw).float() if gw is not None else 1.0)
        w2 = (tw.float() * scale.reshape(-1, *([1] * (tw.dim() - 1)))).to(dt)
        b0 = _const_t(g, ca[2]).float() if ca[2] is not None else torch.zeros_like(tm, dtype=torch.float32)
        b2 = (b0 - tm.float()) * scale + (_const_t(g, gb).float() if gb is not None else 0.0)
        b2 = b2.to(dt)
    node = Node('torch', conv2d_static, [ca[0], _new_const(g, w2), _new_const(g, b2), ca[3], ca[4], ca[5], ca[6]], {},
                n.outs, dict(n.meta or {}, fused='conv2d_bn_fuse_pass'))
    return [j, i], {i: node}


def _relu_node(n):
    return n is not None and n.kind == 'torch' and n.target in (torch.relu, TF.relu, torch.Tensor.relu) and \
        not n.kwargs.get('inplace') and (len(n.args) < 2 or not n.args[1])


def _conv_add_act(g, i):
    """conv (-> + residual) (-> relu) as one node; inference programs."""
    n = g.nodes[i]
    if not _is_conv(n) or _training(g.prog):
        return None
    ca = _conv_args(n)
    if ca is None:
        return None
    body, cur, residual, act, tail = [i], IP._one_out(n), None, None, i
    j = IP._sole_user(g, cur, body)
    m = g.node(j)
    if m is not None and IP._kind(m) == 'add' and len(m.args) == 2 and not m.kwargs:
        a, b = m.args
        other = b if isinstance(a, Ref) and a.vid == cur else (a if isinstance(b, Ref) and b.vid == cur else None)
        if isinstance(other, Ref) and other.vid != cur:
            residual, tail = other, j
            body.append(j)
            cur = IP._one_out(m)
            j = IP._sole_user(g, cur, body)
            m = g.node(j)
    if _relu_node(m) and isinstance(m.args[0], Ref) and m.args[0].vid == cur:
        act, tail = 'relu', j
        body.append(j)
    if len(body) == 1 or not g.private(body[:-1], users=body[-1:]):
        return None
    node = Node('torch', conv2d_add_act, list(ca), {'residual': residual, 'act': act}, IP._one_out(g.nodes[tail]),
                dict(n.meta or {}, fused='conv2d_add_act_fuse_pass'))
    return body, {tail: node}


def _bn_args_full(n):
    """(x, running_mean, running_var, weight, bias, training, torch momentum, eps) of a recorded
    torch.nn.functional.batch_norm node, else None."""
    if n is None or n.kind != 'torch' or n.target is not TF.batch_norm:
        return None
    names = ('input', 'running_mean', 'running_var', 'weight', 'bias', 'training', 'momentum', 'eps')
    defaults = (None, None, None, None, None, False, 0.1, 1e-5)
    if set(n.kwargs) - set(names):
        return None
    v = list(n.args) + [None] * (len(names) - len(n.args))
    out = [n.kwargs.get(k, v[j] if j < len(n.args) else defaults[j]) for j, k in enumerate(names)]
    if not isinstance(out[0], Ref):
        return None
    return out


def _bn_add_act(g, i):
    """batch_norm (-> + residual) (-> relu) as one node on the channels-last HIP kernels (reference
    paddle/fluid/framework/ir/fused_bn_add_act_pass.cc, batch_norm_act_fuse_pass.cc); training and
    inference.  A recorded program holds the library form (its ops were recorded on meta tensors);
    the fused node routes to csrc/batchnorm.hip on the GPU — statistics, apply, residual add and
    ReLU in one autograd op — and runs the composite elsewhere."""
    n = g.nodes[i]
    ba = _bn_args_full(n)
    if ba is None:
        return None
    body, cur, residual, act, tail = [i], IP._one_out(n), None, False, i
    j = IP._sole_user(g, cur, body)
    m = g.node(j)
    if m is not None and IP._kind(m) == 'add' and len(m.args) == 2 and not m.kwargs:
        a, b = m.args
        other = b if isinstance(a, Ref) and a.vid == cur else (a if isinstance(b, Ref) and b.vid == cur else None)
        if isinstance(other, Ref) and other.vid != cur:
            residual, tail = other, j
            body.append(j)
            cur = IP._one_out(m)
            j = IP._sole_user(g, cur, body)
            m = g.node(j)
    if _relu_node(m) and isinstance(m.args[0], Ref) and m.args[0].vid == cur:
        act, tail = True, j
        body.append(j)
    if len(body) > 1 and not g.private(body[:-1], users=body[-1:]):
        return None
    node = Node('torch', batch_norm_add_act, list(ba) + [residual, act], {}, IP._one_out(g.nodes[tail]),
                dict(n.meta or {}, fused='fused_bn_add_act_pass'))
    return body, {tail: node}


def batch_norm_add_act(x, run_mean, run_var, weight, bias, training, momentum, eps, residual=None, relu=False):
    """relu?(batch_norm(x) + residual?) — x NCHW (torch batch_norm layout, torch momentum)."""
    from ..ops import batchnorm as _bn
    from ..ops import use_hip
    if x.dim() == 4 and use_hip(x) and (residual is None or residual.shape == x.shape):
        xc = x.permute(0, 2, 3, 1)
        if _bn.supported(xc, weight) and (training or not (torch.is_grad_enabled() and any(
                t is not None and t.requires_grad for t in (x, weight, bias, residual)))):
            if not xc.is_contiguous():
                xc = xc.contiguous()
            rc = None
            if residual is not None:
                rc = residual.permute(0, 2, 3, 1)
                rc = rc if rc.is_contiguous() else rc.contiguous()
            y = _bn.bn_act_nhwc(xc, weight, bias, run_mean, run_var, eps, 1.0 - momentum, bool(training), bool(relu),
                                residual=rc)
            return y.permute(0, 3, 1, 2)
    y = TF.batch_norm(x, run_mean, run_var, weight, bias, training, momentum, eps)
    if residual is not None:
        y = y + residual
    return torch.relu(y) if relu else y


def _is_embedding(n):
    from ..ops import matmul as _hm
    return n is not None and n.kind == 'torch' and (n.target is TF.embedding or n.target is _hm._embedding_sub) and \
        len(n.args) >= 2 and isinstance(n.args[0], Ref) and isinstance(n.args[1], Const) and \
        not any(k in n.kwargs and n.kwargs[k] not in (None, False, 2.0) for k in ('max_norm', 'sparse',
                                                                                    'scale_grad_by_freq'))


def _emb_ln(g, i):
    """(word + position + token-type) embeddings summed -> layer_norm as one node."""
    n = g.nodes[i]
    la = IP._ln_args(n) if IP._kind(n) == 'layer_norm' else None
    if la is None or _training(g.prog):
        return None
    x, w, b, eps = la
    if not isinstance(x, Ref):
        return None
    body, embs, stack = [i], [], [x]
    while stack:
        r = stack.pop()
        j = g.producer(r.vid, i)
        m = g.node(j)
        if m is None:
            return None
        if _is_embedding(m):
            embs.append(m)
            body.append(j)
        elif IP._kind(m) == 'add' and len(m.args) == 2 and not m.kwargs and all(isinstance(a, Ref) for a in m.args):
            body.append(j)
            stack.extend(m.args)
        else:
            return None
    if len(embs) < 2 or not g.private([j for j in body if j != i], users=[i]):
        return None
    embs.sort(key=lambda m: g.nodes.index(m))
    node = Node('torch', embedding_sum_layer_norm, [[m.args[0] for m in embs], [m.args[1] for m in embs], w, b],
                {'eps': eps}, IP._ln_out(n), dict(n.meta or {}, fused='embedding_eltwise_layernorm_fuse_pass'))
    return sorted(body), {i: node}


_PD_IMPURE = ('random', 'dropout', 'print', 'save', 'load', 'c_', 'send', 'recv', 'fetch', 'feed', 'increment',
              'while', 'conditional_block', 'seed', 'uniform', 'gaussian', 'share', 'memcpy', 'coalesce')


def _foldable(n):
    if n.kind != 'torch':
        return False
    nm = _name(n)
    if nm.startswith('pd.'):  # imported operators: pure ones only
        return not any(k in nm for k in _PD_IMPURE)
    return _pure(n)


def const_values(*cs):
    """Constant-folded outputs of a multi-output node."""
    return list(cs)


def _const_fold(g, i):
    """A node computed from constants only, evaluated once at rewrite time (imported programs carry
    such chains — shape constants, weight reshapes / transposes / casts; a recorded program folds
    them while it is built).  Parameters count as constants only in inference programs."""
    n = g.nodes[i]
    if not _foldable(n) or n.meta.get('factory') or _refs(n.args) or _refs(n.kwargs):
        return None
    train = _training(g.prog)
    consts = []

    def scan(o):
        if isinstance(o, Const):
            consts.append(o)
        elif isinstance(o, (list, tuple)):
            for x in o:
                scan(x)
        elif isinstance(o, dict):
            for x in o.values():
                scan(x)
    scan(n.args)
    scan(n.kwargs)
    if not consts:
        return None
    owners = getattr(g.prog, '_const_owner', {})
    if train and any(owners.get(c.cid) is not None for c in consts):
        return None
    from .executor import _resolve
    try:
        with torch.no_grad():
            val = n.target(*_resolve(g.prog, n.args, {}, {}, None), **_resolve(g.prog, n.kwargs, {}, {}, None))
    except Exception:  # noqa: BLE001 — leave anything unusual to run time
        return None
    meta = dict(n.meta or {}, fused='constant_folding_pass')
    if isinstance(n.outs, int):
        if not isinstance(val, torch.Tensor):
            return None
        return [i], {i: Node('torch', const_value, [_new_const(g, val.detach())], {}, n.outs, meta)}
    if isinstance(n.outs, list) and isinstance(val, (list, tuple)) and len(val) == len(n.outs) and \
            all(o is None or isinstance(o, int) for o in n.outs) and \
            all(v is None or isinstance(v, torch.Tensor) for v in val):
        args = [None if v is None else _new_const(g, v.detach()) for v in val]
        return [i], {i: Node('torch', const_values, args, {}, n.outs, meta)}
    return None


def dead_code_elimination(prog, nodes):
    """Drop pure nodes whose outputs nothing reads (to a fixpoint); returns (nodes, removed count)."""
    removed = 0
    while True:
        g = IP._Graph(prog, nodes)
        keep = []
        drop = 0
        for i, n in enumerate(nodes):
            outs = g.outs[i]
            if _pure(n) and outs and not any(v in g.external or g.uses.get(v) for v in outs):
                drop += 1
                continue
            keep.append(n)
        if not drop:
            return nodes, removed
        removed += drop
        nodes = keep


def _key(o):
    if isinstance(o, Ref):
        return ('r', o.vid)
    if isinstance(o, Const):
        return ('c', o.cid)
    if isinstance(o, (list, tuple)):
        return (type(o).__name__,) + tuple(_key(x) for x in o)
    if isinstance(o, dict):
        return ('d',) + tuple(sorted((k, _key(v)) for k, v in o.items()))
    if isinstance(o, slice):
        return ('s', _key(o.start), _key(o.stop), _key(o.step))
    try:
        hash(o)
        return ('v', type(o).__name__, o)
    except TypeError:
        return ('id', id(o))


def common_subexpression_elimination(prog, nodes):
    """Merge pure nodes with the same target and operands: uses of the duplicate's outputs are
    renamed to the first occurrence's; returns (nodes, merged count)."""
    seen = {}
    rename = {}
    out = []
    merged = 0

    def rn(o):
        if isinstance(o, Ref):
            return Ref(rename.get(o.vid, o.vid))
        if isinstance(o, tuple) and hasattr(o, '_fields'):
            return type(o)(*[rn(x) for x in o])
        if isinstance(o, (list, tuple)):
            return type(o)(rn(x) for x in o)
        if isinstance(o, dict):
            return {k: rn(v) for k, v in o.items()}
        if isinstance(o, slice):
            return slice(rn(o.start), rn(o.stop), rn(o.step))
        return o
    ext = IP._Graph(prog, nodes).external
    for n in nodes:
        if rename:
            n = Node(n.kind, n.target, rn(n.args), rn(n.kwargs), n.outs, n.meta)
        if _pure(n) and not n.meta.get('factory') and n.outs is not None:
            try:
                k = (n.target, _key(n.args), _key(n.kwargs))
                hash(k)
            except TypeError:
                k = None
            if k is not None:
                first = seen.get(k)
                a, b = IP._outs_of(first.outs, []) if first is not None else [], IP._outs_of(n.outs, [])
                if first is not None and len(a) == len(b) and not any(v in ext for v in b):
                    for x, y in zip(a, b):
                        rename[y] = x
                    merged += 1
                    continue
                seen[k] = n
        out.append(n)
    return out, merged


def _woq_linear(g, i):
    """Inference Linear with a 16-bit constant weight -> weight-only int8 (per-channel scales,
    quantised once at rewrite time) on the decode-shaped woq kernel (csrc/woq_gemm.hip)."""
    n = g.nodes[i]
    if _training(g.prog) or n.kind != 'torch' or n.kwargs:
        return None
    if n.target is TF.linear and len(n.args) >= 2:      # torch layout W [out, in]
        x, w = n.args[0], n.args[1]
        b = n.args[2] if len(n.args) > 2 else None
        tw = _const_t(g, w)
        tw = None if tw is None else tw.t()
    elif n.target is torch.addmm and len(n.args) == 3:  # paddle Linear: addmm(b, x, W[in, out])
        b, x, w = n.args
        tw = _const_t(g, w)
        if b is not None and not isinstance(b, Const):
            return None
    elif n.target in (torch.matmul, torch.mm) and len(n.args) == 2:
        x, w = n.args
        b, tw = None, _const_t(g, w)
    else:
        return None
    if not isinstance(x, Ref) or tw is None or tw.dim() != 2 or tw.dtype not in (torch.bfloat16, torch.float16):
        return None
    if tw.shape[0] % 64 or tw.shape[1] % 8:
        return None
    from ..nn.quant import weight_quantize
    from ..core.tensor import _wrap, _unwrap
    q, s = weight_quantize(_wrap(tw.contiguous()), algo='weight_only_int8')  # [out, in] int8, [out] scale
    node = Node('torch', woq_linear_static, [x, _new_const(g, _unwrap(q)), _new_const(g, _unwrap(s).to(tw.dtype)),
                                             b], {}, n.outs, dict(n.meta or {}, fused='fused_weight_only_linear_pass'))
    return [i], {i: node}


def woq_linear_static(x, q, scale, bias=None):
    from ..nn.quant import weight_only_linear
    from ..core.tensor import _wrap, _unwrap
    return _unwrap(weight_only_linear(_wrap(x), _wrap(q), None if bias is None else _wrap(bias), _wrap(scale), 'int8'))


# inplace_pass (reference: paddle/fluid/pir/transforms/general/inplace_pass.cc): in an inference
# program, an elementwise op whose first operand dies at it writes into that operand's buffer.
_FRESH = {  # producers whose output is a new buffer (never a view of an input)
    'addmm', 'mm', 'matmul', 'bmm', 'baddbmm', 'linear', 'conv1d', 'conv2d', 'conv3d', 'conv_transpose1d',
    'conv_transpose2d', 'conv_transpose3d', 'layer_norm', 'group_norm', 'batch_norm', 'instance_norm',
    'softmax', 'log_softmax', 'add', 'sub', 'mul', 'div', 'true_divide', 'tanh', 'sigmoid', 'gelu', 'relu',
    'silu', 'exp', 'erf', 'sqrt', 'rsqrt', 'pow', 'scaled_dot_product_attention', 'embedding', 'where',
}
_TF_INPLACE_KW = {TF.relu, TF.silu, TF.leaky_relu, TF.elu, TF.hardtanh, TF.relu6, TF.hardswish, TF.hardsigmoid}
_INPLACE = {torch.relu: torch.relu_, torch.tanh: torch.tanh_, torch.sigmoid: torch.sigmoid_, torch.exp: torch.exp_,
            torch.add: torch.Tensor.add_, torch.mul: torch.Tensor.mul_, torch.sub: torch.Tensor.sub_,
            torch.div: torch.Tensor.div_, torch.Tensor.add: torch.Tensor.add_, torch.Tensor.mul: torch.Tensor.mul_,
            torch.Tensor.sub: torch.Tensor.sub_, torch.Tensor.div: torch.Tensor.div_,
            torch.Tensor.__add__: torch.Tensor.add_, torch.Tensor.__mul__: torch.Tensor.mul_,
            torch.Tensor.__sub__: torch.Tensor.sub_, torch.Tensor.__truediv__: torch.Tensor.div_}


def inplace_pass(prog, nodes):
    """Rewrite dying-operand elementwise ops of inference programs to their in-place forms;
    returns (nodes, rewritten count).  The operand must be a fresh buffer (its producer allocates,
    see _FRESH), read only by non-aliasing ops, last read here, not fetched / fed, and of the
    result's shape and dtype (no broadcast growth, no type promotion)."""
    if _training(prog):
        return nodes, 0
    g = IP._Graph(prog, nodes)
    producers = {}
    for i, outs in enumerate(g.outs):
        for v in outs:
            producers.setdefault(v, []).append(i)
    out, cnt = [], 0
    for i, n in enumerate(nodes):
        tgt = n.target
        kw_form = n.kind == 'torch' and tgt in _TF_INPLACE_KW and not n.kwargs.get('inplace')
        if n.kind != 'torch' or not (kw_form or tgt in _INPLACE) or not n.args or not isinstance(n.args[0], Ref):
            out.append(n)
            continue
        x = n.args[0].vid
        outs = g.outs[i]
        prod = producers.get(x, [])
        ok = (len(outs) == 1 and outs[0] != x and x not in g.external and len(prod) == 1 and prod[0] < i
              and nodes[prod[0]].kind == 'torch' and _name(nodes[prod[0]]) in _FRESH
              and max(g.uses.get(x, {i})) == i
              and all(nodes[u].kind == 'torch' and (_name(nodes[u]) in _FRESH or nodes[u].target in _INPLACE
                                                    or nodes[u].target in _TF_INPLACE_KW) for u in g.uses.get(x, ()))
              and sum(1 for r in _refs(n.args) + _refs(n.kwargs) if r == x) == 1)
        mx, mo = g.meta.get(x), g.meta.get(outs[0]) if outs else None
        ok = ok and mx is not None and mo is not None and tuple(mx.shape) == tuple(mo.shape) and mx.dtype == mo.dtype
        if not ok:
            out.append(n)
            continue
        if kw_form:
            out.append(Node('torch', tgt, n.args, dict(n.kwargs, inplace=True), n.outs, dict(n.meta or {}, inplace=True)))
        else:
            out.append(Node('torch', _INPLACE[tgt], n.args, n.kwargs, n.outs, dict(n.meta or {}, inplace=True)))
        cnt += 1
    return out, cnt


# ------------------------------------------------------------------ round-6 general passes
def _ref1(n, k=0):
    a = n.args[k] if len(n.args) > k else None
    return a if isinstance(a, Ref) else None


def _scalar(v):
    return isinstance(v, (int, float)) and not isinstance(v, bool)


def rms_norm_static(x, weight, eps=1e-6):
    """x * rsqrt(mean(x^2, -1) + eps) * weight — csrc/norm.hip on the GPU, the composite elsewhere."""
    from . import ir_passes as _ip
    if _ip._hip(x) and weight is not None and weight.dim() == 1 and weight.numel() == x.shape[-1] and \
            x.dtype in (torch.bfloat16, torch.float16, torch.float32) and x.shape[-1] % 8 == 0 and weight.is_cuda:
        from ..ops import norm
        return norm.rms_norm(x, weight, float(eps))
    xf = x.float()
    y = (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)).to(x.dtype)
    return y * weight if weight is not None else y


def _rms_norm(g, i):
    """pow(x, 2) -> mean(-1, keepdim) -> + eps -> rsqrt -> x * r (-> cast) -> * weight: the composite
    RMSNorm a recorded program holds (reference pir/transforms/gpu/rms_norm_fuse_pass.cc)."""
    n = g.nodes[i]
    if n.kind != 'torch' or _name(n) not in ('mul', '__mul__', 'multiply') or len(n.args) != 2 or n.kwargs:
        return None
    a, b = n.args
    w, y = (b, a) if isinstance(b, Const) else ((a, b) if isinstance(a, Const) else (None, None))
    if not isinstance(y, Ref) or w is None:
        return None
    tw = _const_t(g, w)
    if tw is None or tw.dim() != 1:
        return None
    body = [i]
    j = g.producer(y.vid, i)
    m = g.node(j)
    if m is not None and _name(m) == 'to' and _ref1(m) is not None and IP._one_out(m) == _ref1(m).vid:
        j2 = g.producer(y.vid, j)  # the recorder's same-value cast: the product comes from before it
        body.append(j)
        j, m = j2, g.node(j2)
    if m is None or _name(m) not in ('mul', '__mul__', 'multiply') or len(m.args) != 2:
        return None
    body.append(j)
    x, r = m.args
    if not (isinstance(x, Ref) and isinstance(r, Ref)):
        return None
    for xx, rr in ((x, r), (r, x)):
        k = g.producer(rr.vid, j)
        rs = g.node(k)
        if rs is None or _name(rs) != 'rsqrt' or _ref1(rs) is None:
            continue
        k2 = g.producer(_ref1(rs).vid, k)
        ad = g.node(k2)
        if ad is None or _name(ad) not in ('add', '__add__') or len(ad.args) != 2 or not _scalar(ad.args[1]) or \
                _ref1(ad) is None:
            continue
        eps = float(ad.args[1])
        k3 = g.producer(_ref1(ad).vid, k2)
        mn = g.node(k3)
        if mn is None or _name(mn) != 'mean' or _ref1(mn) is None:
            continue
        dims = mn.args[1] if len(mn.args) > 1 else mn.kwargs.get('dim')
        if dims not in (-1, [-1], (-1,)) or not (mn.kwargs.get('keepdim') or (len(mn.args) > 2 and mn.args[2])):
            continue
        k4 = g.producer(_ref1(mn).vid, k3)
        pw = g.node(k4)
        if pw is None or _name(pw) not in ('pow', '__pow__') or _ref1(pw) is None or _ref1(pw).vid != xx.vid or \
                len(pw.args) < 2 or pw.args[1] != 2:
            continue
        chain = body + [k, k2, k3, k4]
        if not g.private(chain[1:], users=[i]):
            return None
        node = Node('torch', rms_norm_static, [xx, w], {'eps': eps}, n.outs, dict(n.meta or {}, fused='rms_norm_fuse_pass'))
        return chain, {i: node}
    return None


def _silu(g, i):
    """x * sigmoid(x) -> silu(x) (reference silu_fuse_pass)."""
    n = g.nodes[i]
    if n.kind != 'torch' or _name(n) not in ('mul', '__mul__', 'multiply') or len(n.args) != 2 or n.kwargs:
        return None
    a, b = n.args
    if not (isinstance(a, Ref) and isinstance(b, Ref)):
        return None
    for x, s_ in ((a, b), (b, a)):
        j = g.producer(s_.vid, i)
        m = g.node(j)
        if m is not None and _name(m) == 'sigmoid' and _ref1(m) is not None and _ref1(m).vid == x.vid and \
                len(m.args) == 1 and not m.kwargs and g.private([j], users=[i]):
            return [j, i], {i: Node('torch', TF.silu, [x], {}, n.outs, dict(n.meta or {}, fused='silu_fuse_pass'))}
    return None


def _perm_of(n):
    if _name(n) == 'permute':
        p = n.args[1:] if len(n.args) > 2 else (n.args[1] if len(n.args) > 1 else n.kwargs.get('dims'))
        return tuple(p) if isinstance(p, (list, tuple)) and all(isinstance(v, int) for v in p) else None
    return None


def identity_static(x):
    return x


def _transpose_pair(g, i):
    """permute(permute(x, p1), p2) -> one permute (or x itself) (reference
    remove_redundant_transpose_pass)."""
    n = g.nodes[i]
    if n.kind != 'torch':
        return None
    p2 = _perm_of(n)
    x = _ref1(n)
    if p2 is None or x is None:
        return None
    j = g.producer(x.vid, i)
    m = g.node(j)
    p1 = _perm_of(m) if m is not None and m.kind == 'torch' else None
    if p1 is None or len(p1) != len(p2) or _ref1(m) is None or not g.private([j], users=[i]):
        return None
    comp = tuple(p1[k] for k in p2)
    src = _ref1(m)
    if comp == tuple(range(len(comp))):
        node = Node('torch', identity_static, [src], {}, n.outs, dict(n.meta or {}, fused='remove_redundant_transpose_pass'))
    else:
        node = Node('torch', torch.permute, [src, list(comp)], {}, n.outs,
                    dict(n.meta or {}, fused='remove_redundant_transpose_pass'))
    return [j, i], {i: node}


def _matmul_scale(g, i):
    """Inference: (x @ W [+ b]) * c with a constant W -> x @ (c W) [+ c b] (reference
    matmul_scale_fuse_pass)."""
    n = g.nodes[i]
    if _training(g.prog) or n.kind != 'torch' or _name(n) not in ('mul', '__mul__', 'multiply') or \
            len(n.args) != 2 or n.kwargs:
        return None
    a, c = n.args
    if not (isinstance(a, Ref) and _scalar(c)):
        return None
    j = g.producer(a.vid, i)
    m = g.node(j)
    if m is None or m.kind != 'torch' or m.kwargs or not g.private([j], users=[i]):
        return None
    nm = _name(m)
    if nm == 'addmm' and len(m.args) == 3 and isinstance(m.args[2], Const) and isinstance(m.args[0], Const):
        tb, tw = _const_t(g, m.args[0]), _const_t(g, m.args[2])
        if tb is None or tw is None:
            return None
        with torch.no_grad():
            args = [_new_const(g, (tb * c).to(tb.dtype)), m.args[1], _new_const(g, (tw * c).to(tw.dtype))]
        return [j, i], {i: Node('torch', torch.addmm, args, {}, n.outs, dict(n.meta or {}, fused='matmul_scale_fuse_pass'))}
    if nm in ('mm', 'matmul') and len(m.args) == 2 and isinstance(m.args[1], Const):
        tw = _const_t(g, m.args[1])
        if tw is None:
            return None
        with torch.no_grad():
            args = [m.args[0], _new_const(g, (tw * c).to(tw.dtype))]
        return [j, i], {i: Node('torch', m.target, args, {}, n.outs, dict(n.meta or {}, fused='matmul_scale_fuse_pass'))}
    return None


def identity_op_clean(prog, nodes):
    """Drop identity nodes — a cast to the value's own dtype, a reshape to its own shape, x * 1,
    x + 0, x - 0, x / 1, dropout that is off, a same-order permute — renaming their outputs to
    their inputs (reference general/identity_op_clean_pass.cc); returns (nodes, dropped count)."""
    g = IP._Graph(prog, nodes)
    rename, out, cnt = {}, [], 0

    def rn(o):
        if isinstance(o, Ref):
            return Ref(rename.get(o.vid, o.vid))
        if isinstance(o, tuple) and hasattr(o, '_fields'):
            return type(o)(*[rn(x) for x in o])
        if isinstance(o, (list, tuple)):
            return type(o)(rn(x) for x in o)
        if isinstance(o, dict):
            return {k: rn(v) for k, v in o.items()}
        if isinstance(o, slice):
            return slice(rn(o.start), rn(o.stop), rn(o.step))
        return o

    for n in nodes:
        if rename:
            n = Node(n.kind, n.target, rn(n.args), rn(n.kwargs), n.outs, n.meta)
        src = _identity_src(g, n)
        outs = IP._outs_of(n.outs, [])
        if src is not None and len(outs) == 1 and outs[0] not in g.external and outs[0] != src:
            rename[outs[0]] = rename.get(src, src)
            cnt += 1
            continue
        out.append(n)
    return out, cnt


def _identity_src(g, n):
    if n.kind != 'torch' or not n.args or not isinstance(n.args[0], Ref):
        return None
    nm, x = _name(n), n.args[0].vid
    mx = g.meta.get(x)
    outs = IP._outs_of(n.outs, [])
    mo = g.meta.get(outs[0]) if len(outs) == 1 else None
    if mx is None or mo is None or tuple(mx.shape) != tuple(mo.shape) or mx.dtype != mo.dtype:
        return None
    if nm in ('to', 'type', 'type_as', 'float', 'reshape', 'view', 'flatten'):
        return x  # (contiguous / clone / detach change layout, aliasing or autograd: kept)
    if nm in ('mul', '__mul__', 'multiply', 'div', 'true_divide', '__truediv__') and len(n.args) == 2 and \
            _scalar(n.args[1]) and n.args[1] == 1 and not n.kwargs:
        return x
    if nm in ('add', '__add__', 'sub', '__sub__', 'subtract') and len(n.args) == 2 and _scalar(n.args[1]) and \
            n.args[1] == 0 and not n.kwargs:
        return x
    if nm == 'dropout':
        p = n.args[1] if len(n.args) > 1 else n.kwargs.get('p', 0.5)
        tr = n.args[2] if len(n.args) > 2 else n.kwargs.get('training', True)
        if p == 0 or not tr:
            return x
    if nm == 'permute':
        p = _perm_of(n)
        if p is not None and p == tuple(range(len(p))):
            return x
    return None


def _graph_pass(fn):
    """Adapt a whole-list rewrite (nodes -> nodes, count) to apply_passes' per-pass protocol."""
    fn._whole_list = True
    return fn


def register():
    IP._PASSES.update({
        'constant_folding_pass': _const_fold,
        'conv2d_bn_fuse_pass': _conv_bn,
        'fused_bn_add_act_pass': _bn_add_act,
        'conv2d_add_act_fuse_pass': _conv_add_act,
        'embedding_eltwise_layernorm_fuse_pass': _emb_ln,
        'fused_weight_only_linear_pass': _woq_linear,
        'dead_code_elimination_pass': _graph_pass(dead_code_elimination),
        'common_subexpression_elimination_pass': _graph_pass(common_subexpression_elimination),
        'inplace_pass': _graph_pass(inplace_pass),
        'identity_op_clean_pass': _graph_pass(identity_op_clean),
        'rms_norm_fuse_pass': _rms_norm,
        'silu_fuse_pass': _silu,
        'remove_redundant_transpose_pass': _transpose_pair,
        'matmul_scale_fuse_pass': _matmul_scale,
    })
