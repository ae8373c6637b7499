"""IR fusion passes over static Programs (recorded op lists and imported ProgramDesc / PIR programs).

Reference: the GPU inference pass list (paddle/fluid/inference/api/paddle_pass_builder.cc:192-204:
``multihead_matmul_fuse_pass_v2``, ``fc_fuse_pass``, ...) over the graph passes of
paddle/fluid/framework/ir/ (multihead_matmul_fuse_pass.cc, fc_fuse_pass.cc,
layer_norm_fuse_pass.cc, skip_layernorm_fuse_pass.cc, fused_dropout_add / fused bias-dropout-
residual-layernorm).  The reference rewrites ProgramDesc ops into fused PHI kernels; here a
Program is a node list (static/program.py) and a pass rewrites node sub-chains into ONE node whose
target is a fused entry point of this module.  The entry points run the hand-written HIP kernels
(csrc/flash_attn*.hip, csrc/norm.hip, csrc/act.hip, csrc/gemm8.hip) when their operands fit, and
otherwise the exact composite of the ops they replaced — so a fused program is correct on every
device and the passes are pure scheduling decisions.

Both node vocabularies are matched: torch-level nodes recorded from dygraph-style model code
(``torch.matmul`` / ``Tensor.masked_fill`` / ``F.layer_norm`` ...) and Paddle-operator nodes of
an imported ProgramDesc (``matmul_v2`` / ``scale`` / ``softmax`` / ``layer_norm`` ...).

Passes (names follow the reference where one exists; general and convolution passes in
static/ir_passes_ext.py: constant_folding_pass, common_subexpression_elimination_pass,
dead_code_elimination_pass, conv2d_bn_fuse_pass, conv2d_add_act_fuse_pass,
embedding_eltwise_layernorm_fuse_pass, fused_weight_only_linear_pass):
  multihead_matmul_fuse_pass_v2   q@k^T -> *scale -> (+mask | masked_fill) -> softmax -> (dropout)
                                  -> @v   ==>  flash attention (mask and dropout inside the kernel)
  fused_dropout_add_layernorm     dropout(x) + residual -> layer_norm  ==> one norm kernel each way
  skip_layernorm_fuse_pass        x + residual -> layer_norm           ==> fused add + norm kernel
  layer_norm_fuse_pass            layer_norm                           ==> csrc/norm.hip
  fuse_gemm_epilogue_pass         addmm -> gelu -> addmm (recorded FFN) ==> GELU and GELU' in the GEMM
                                  epilogues, forward and backward (training programs)
  fc_fuse_pass                    x @ W + b (-> relu / gelu)           ==> GEMM (+ bias + act kernel)
  softmax_fuse_pass               standalone last-dim softmax           ==> csrc/softmax_xent.hip
  quant_linear_fuse_pass          quantize_linear -> dequantize_linear (activation) + dequantize_linear
                                  (int8 weight) -> matmul_v2 (+ bias)  ==> the int8 MFMA GEMM

The Executor and the inference Predictor run programs through ``ir_nodes(program, device)``: the
rewritten node list is built once per program version and cached; ``program.nodes`` itself is never
modified (save / export still see the original ops).
"""
import math
import os

import torch
import torch.nn.functional as TF

from .program import Node, Ref, Const

# (CSE runs after the fusions: merging two equal subgraphs first would make them shared, and a
# fusion claims only private chains)
DEFAULT_PASSES = ('constant_folding_pass', 'identity_op_clean_pass', 'remove_redundant_transpose_pass',
                  'matmul_scale_fuse_pass', 'rms_norm_fuse_pass', 'silu_fuse_pass', 'conv2d_bn_fuse_pass',
                  'conv2d_add_act_fuse_pass', 'fused_bn_add_act_pass', 'embedding_eltwise_layernorm_fuse_pass',
                  'quant_linear_fuse_pass', 'multihead_matmul_fuse_pass_v2', 'fused_dropout_add_layernorm', 'skip_layernorm_fuse_pass',
                  'fuse_gemm_epilogue_pass', 'layer_norm_fuse_pass', 'fc_fuse_pass', 'softmax_fuse_pass',
                  'common_subexpression_elimination_pass', 'dead_code_elimination_pass', 'inplace_pass')
# opt-in (change numerics): 'fused_weight_only_linear_pass' (int8 weight-only Linears of inference programs)

# FLAGS_static_ir_fusion: 'auto' (default: GPU programs), '1' / 'always' (every device, used by the
# CPU tests of the rewrites), '0' (off)
_MODE = [os.environ.get('FLAGS_static_ir_fusion', 'auto')]


def set_mode(mode):
    old = _MODE[0]
    _MODE[0] = str(mode)
    return old


# ============================================================================ fused entry points
def _hip(t):
    from .. import ops
    return isinstance(t, torch.Tensor) and t.is_cuda and ops.enabled() and ops.use_hip(t)


def _attn_mask(mask, mode, fill, dtype):
    """The kernel's additive / bool mask from a recorded masking step."""
    if mask is None or mode is None:
        return None
    if mode == 'add':
        return mask
    keep = mask if mode == 'keep' else ~mask
    if fill == float('-inf'):
        return keep
    # masked_fill with a finite fill (-1e30 / -1e4): additive, so rows with every key masked keep
    # the composite's uniform distribution instead of the -inf form's zero row
    z = torch.zeros((), dtype=dtype, device=mask.device)
    return torch.where(keep, z, torch.full((), fill, dtype=dtype, device=mask.device))


def fused_attention(q, k, v, mask=None, scale=1.0, dropout=0.0, mask_mode=None, k_transposed=False, fill=-1e30):
    """softmax(q @ k^T * scale (+ mask)) (dropout) @ v on [B, H, S, D] operands.

    ``k_transposed``: ``k`` is already k^T ([B, H, D, Sk]).  mask_mode: 'keep' (bool, True keeps),
    'drop' (bool, True is filled with ``fill``), 'add' (additive) or None."""
    kk = k.transpose(-1, -2) if k_transposed else k
    if (q.dim() == 4 and kk.dim() == 4 and v.dim() == 4 and q.dtype in (torch.bfloat16, torch.float16)
            and kk.dtype == q.dtype and v.dtype == q.dtype and _hip(q)
            and (mask is None or (isinstance(mask, torch.Tensor) and mask.device == q.device and mask.dim() <= 4))):
        from ..ops import flash_attn as FA
        qb, kb, vb = q.transpose(1, 2), kk.transpose(1, 2), v.transpose(1, 2)
        if FA.supported_ex(qb, kb, vb) or FA.supported(qb, kb, vb):
            m = _attn_mask(mask, mask_mode, fill, q.dtype)
            if m is not None and m.dim() < 4:
                m = m.reshape((1,) * (4 - m.dim()) + tuple(m.shape))
            o = FA.flash_attention_ex(qb, kb, vb, scale=float(scale), mask=m, dropout=float(dropout))
            return o.transpose(1, 2)
    s = torch.matmul(q, kk.transpose(-1, -2)).float() * scale
    if mask is not None and mask_mode is not None:
        if mask_mode == 'add':
            s = s + mask.float()
        else:
            s = s.masked_fill(~mask if mask_mode == 'keep' else mask, fill)
    p = torch.softmax(s, -1)
    if dropout > 0.0:
        p = TF.dropout(p, dropout, True)
    return torch.matmul(p.to(v.dtype), v)


def fused_attention_packed(qkv, mask=None, scale=1.0, dropout=0.0, mask_mode=None, fill=-1e30):
    """The same attention with q / k / v the three [B, S, H, D] slices of one packed [B, S, 3, H, D]
    projection (dim 2): the packed flash path writes dQ / dK / dV straight into one packed gradient
    (no per-slice zero-filled gradient buffers and adds).  Returns [B, H, S, D]."""
    if (qkv.dim() == 5 and qkv.shape[2] == 3 and qkv.dtype in (torch.bfloat16, torch.float16) and _hip(qkv)
            and (mask is None or (isinstance(mask, torch.Tensor) and mask.device == qkv.device and mask.dim() <= 4))):
        from ..ops import flash_attn as FA
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        if FA.supported(q, k, v):
            m = _attn_mask(mask, mask_mode, fill, qkv.dtype)
            if m is not None and m.dim() < 4:
                m = m.reshape((1,) * (4 - m.dim()) + tuple(m.shape))
            o = FA.flash_attention_packed_ex(qkv, scale=float(scale), mask=m, dropout=float(dropout))
            return o.transpose(1, 2)
    q, k, v = (qkv[:, :, i].transpose(1, 2) for i in range(3))
    return fused_attention(q, k, v, mask, scale, dropout, mask_mode, False, fill)


def _norm_ok(x, w, b):
    C = x.shape[-1]
    return (_hip(x) and w is not None and b is not None and w.dim() == 1 and w.numel() == C and b.numel() == C
            and x.dtype in (torch.bfloat16, torch.float16, torch.float32) and C % 8 == 0 and C <= 8192
            and w.is_cuda)


def _ln_composite(x, weight, bias, eps, axis):
    ns = list(x.shape[axis:])
    w = None if weight is None else weight.reshape(ns)
    b = None if bias is None else bias.reshape(ns)
    return TF.layer_norm(x, ns, w, b, eps)


def _last_axis(x, axis):
    return axis is None or axis in (-1, x.dim() - 1)


def fused_layer_norm(x, weight=None, bias=None, eps=1e-5, begin_axis=None):
    """layer_norm over the last dim on csrc/norm.hip (composite otherwise); ``begin_axis``: an
    imported layer_norm's begin_norm_axis (normalises dims [begin_axis:])."""
    if not _last_axis(x, begin_axis):
        return _ln_composite(x, weight, bias, eps, begin_axis)
    if _norm_ok(x, weight, bias):
        from ..ops import norm
        return norm.layer_norm(x, weight, bias, float(eps))
    w = weight.to(x.dtype) if weight is not None and x.dtype != torch.float32 else weight
    b = bias.to(x.dtype) if bias is not None and x.dtype != torch.float32 else bias
    return TF.layer_norm(x, [x.shape[-1]], w, b, eps)


def fused_dropout_add_layer_norm(x, res, weight=None, bias=None, eps=1e-5, p=0.0, begin_axis=None):
    """[layer_norm(dropout(x, p) + res), dropout(x, p) + res] — one kernel each way on the GPU.
    Under AMP a float32 residual stream is carried in x's 16-bit dtype (the reference's O2)."""
    if not _last_axis(x, begin_axis):
        h = TF.dropout(x, p, True) if p > 0.0 else x
        s = h + res
        return [_ln_composite(s, weight, bias, eps, begin_axis), s]
    if (_norm_ok(x, weight, bias) and isinstance(res, torch.Tensor) and res.shape == x.shape
            and x.dtype in (torch.bfloat16, torch.float16)):
        from ..ops import norm, fused
        r = res if res.dtype == x.dtype else res.to(x.dtype)
        if p > 0.0 and fused.dropout_add_norm_ok(x, weight, p):
            y, s = fused.dropout_add_norm(x, None, r, weight, bias, float(eps), float(p))
            return [y, s]
        if p == 0.0:
            y, s = norm.add_layer_norm(x, r, weight, bias, float(eps))
            return [y, s]
    h = TF.dropout(x, p, True) if p > 0.0 else x
    s = h + res
    return [TF.layer_norm(s, [s.shape[-1]], weight, bias, eps), s]


_ACT = {None: None, 'relu': torch.relu, 'gelu': lambda t: TF.gelu(t), 'gelu_tanh': lambda t: TF.gelu(t, approximate='tanh'),
        'tanh': torch.tanh, 'sigmoid': torch.sigmoid}


def fused_linear(x, w, bias=None, act=None, trans_w=False):
    """act(x @ W + bias) (W [in, out], or [out, in] with ``trans_w``): the GEMM on the hand-written
    kernel (ops/matmul.py routing) with the bias in its epilogue; bf16 inputs of >= 1024 rows also
    take the activation in the epilogue (ops.gemm.mm_act), others run it as one pass over the
    output (csrc/act.hip); composite otherwise."""
    from ..ops import matmul as hm
    W = w.t() if trans_w else w
    if act in (None, 'relu', 'gelu', 'gelu_tanh') and _hip(x) and x.dtype in (torch.bfloat16, torch.float16) \
            and W.dtype == x.dtype and (bias is None or bias.dtype == x.dtype):
        from ..ops import act as A, gemm as G
        if act is None:
            return hm.linear(x, W, bias)
        x2 = x.reshape(-1, x.shape[-1])
        if (x.dtype == torch.bfloat16 and x2.shape[0] >= 1024 and not torch.is_grad_enabled()
                and G.epi_ok(x2, W, W.shape[1])):
            return G.mm_act(x2, W, bias, act).reshape(*x.shape[:-1], W.shape[1])
        y = hm.linear(x, W, None)
        if act == 'relu':
            return A.bias_relu(y, bias)
        return A.gelu(y, approximate=(act == 'gelu_tanh'), bias=bias)
    y = torch.matmul(x, W)
    if bias is not None:
        y = y + bias
    fn = _ACT[act]
    return fn(y) if fn is not None else y


def _replay_addmm(b, x, w):
    """torch.addmm as the Executor replays a recorded one (static.amp fp8 and GEMM substitutions)."""
    from .executor import _SUBS, _gemm_subs
    subs = _SUBS['map']
    fn = subs.get(torch.addmm, torch.addmm) if subs else torch.addmm
    fn = _gemm_subs().get(fn, fn)
    return fn(b, x, w)


def fused_ffn(x, w1, b1, w2, b2, approximate='none'):
    """gelu(x @ W1 + b1) @ W2 + b2 of a recorded feed-forward block (x 2-D).  Training on bf16 GPU
    operands: one autograd op with the GELU (and its derivative) in the GEMM epilogues
    (ops.matmul.ffn_gelu; under a static.amp fp8 replay the fp8 form, ops.fp8.fp8_ffn); inference: fc1's epilogue applies the GELU (fused_linear); otherwise
    exactly the recorded addmm -> gelu -> addmm (with the replay's fp8 / GEMM substitutions)."""
    from .executor import _SUBS
    if _SUBS['map'] is not None and _hip(x) and torch.is_grad_enabled():
        from ..ops import fp8 as F8
        if _SUBS['map'] is F8.STATIC_SUBS and F8.ffn_ok(x, w1, b1, w2, b2):  # static.amp fp8 replay
            return F8.fp8_ffn(x, w1, b1, w2, b2, approximate == 'tanh')
    if _SUBS['map'] is None and _hip(x):
        from ..ops import matmul as hm
        if torch.is_grad_enabled() and any(t.requires_grad for t in (x, w1, b1, w2, b2)):
            if hm.ffn_gelu_ok(x, w1, b1, w2, b2):
                return hm.ffn_gelu(x, w1, b1, w2, b2, approximate == 'tanh')
        elif x.dtype == w1.dtype == b1.dtype and x.dtype in (torch.bfloat16, torch.float16):
            act = 'gelu_tanh' if approximate == 'tanh' else 'gelu'
            return _replay_addmm(b2, fused_linear(x, w1, b1, act), w2)
    return _replay_addmm(b2, TF.gelu(_replay_addmm(b1, x, w1), approximate=approximate), w2)


def fused_softmax(x, dim=-1):
    if _hip(x) and x.dtype in (torch.bfloat16, torch.float16) and dim in (-1, x.dim() - 1) and x.shape[-1] % 8 == 0:
        from ..ops import softmax as S
        return S.softmax(x)
    return torch.softmax(x, dim)


FUSED_TARGETS = (fused_attention, fused_attention_packed, fused_layer_norm, fused_dropout_add_layer_norm, fused_linear,
                 fused_softmax, fused_ffn)


# ============================================================================ node vocabulary
_KINDS = {}


def _init_kinds():
    T = torch.Tensor
    table = {
        'matmul': [torch.matmul, T.matmul, T.__matmul__, torch.bmm, T.bmm],
        'transpose': [torch.transpose, T.transpose, torch.swapaxes, T.swapaxes],
        'cast': [T.float, T.to, T.half, T.bfloat16, T.contiguous, T.type_as],
        'mul': [torch.mul, T.mul, T.__mul__, T.__rmul__],
        'div': [torch.div, T.div, T.__truediv__],
        'add': [torch.add, T.add, T.__add__, T.__radd__],
        'masked_fill': [torch.masked_fill, T.masked_fill],
        'invert': [T.__invert__, torch.logical_not, T.logical_not, torch.bitwise_not, T.bitwise_not],
        'softmax': [torch.softmax, T.softmax, TF.softmax],
        'dropout': [TF.dropout],
        'layer_norm': [TF.layer_norm, torch.layer_norm],
        'addmm': [torch.addmm],
        'linear': [TF.linear],
        'reshape': [T.reshape, T.view, torch.reshape],
        'gelu': [TF.gelu],
        'relu': [torch.relu, TF.relu, T.relu],
        'getitem': [T.__getitem__],
    }
    for k, fs in table.items():
        for f in fs:
            try:
                _KINDS[f] = k
            except TypeError:
                pass


def _kind(n):
    if n is None or n.kind != 'torch':
        return None
    if not _KINDS:
        _init_kinds()
    t = n.target
    if type(t).__name__ == '_OpCall':
        return 'pd.' + t.type
    try:
        return _KINDS.get(t)
    except TypeError:
        return None


def _arg(n, i, name, default=None):
    if len(n.args) > i:
        return n.args[i]
    return n.kwargs.get(name, default)


def _num(v):
    return isinstance(v, (int, float)) and not isinstance(v, bool)


def _one_out(n):
    """The output of a single-output node as the executor binds it (imported operators keep a
    one-element list of vids)."""
    o = n.outs
    if isinstance(o, (list, tuple)) and len(o) == 1 and isinstance(o[0], int):
        return o[0]
    return o


def _pd_in(n, slot, i=0):
    """i-th argument of input slot ``slot`` of an imported-operator node (None if absent)."""
    pos = 0
    for s, cnt in n.target.slots:
        if s == slot:
            return n.args[pos + i] if i < cnt else None
        pos += cnt
    return None


def _pd_out(n, slot, i=0):
    pos = 0
    for s, cnt in n.target.out_slots:
        if s == slot:
            return n.outs[pos + i] if i < cnt else None
        pos += cnt
    return None


# ============================================================================ def-use view
def _refs_in(obj, out):
    if isinstance(obj, Ref):
        out.append(obj.vid)
    elif isinstance(obj, Node):
        _refs_in(obj.args, out)
        _refs_in(obj.kwargs, out)
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            _refs_in(o, out)
    elif isinstance(obj, dict):
        for o in obj.values():
            _refs_in(o, out)
    elif isinstance(obj, slice):
        _refs_in([obj.start, obj.stop, obj.step], out)


def _outs_of(o, acc):
    if o is None:
        return acc
    if isinstance(o, int):
        acc.append(o)
    else:
        for x in o:
            _outs_of(x, acc)
    return acc


class _Graph:
    def __init__(self, prog, nodes):
        self.prog, self.nodes = prog, nodes
        self.outs = [_outs_of(n.outs, []) for n in nodes]
        self.uses = {}
        for i, n in enumerate(nodes):
            r = []
            _refs_in(n.args, r)
            _refs_in(n.kwargs, r)
            for v in r:
                self.uses.setdefault(v, set()).add(i)
        ext = set()
        for var in getattr(prog, 'named_vars', {}).values():
            t = getattr(var, '_t', None)
            vid = prog._val.get(id(t)) if t is not None else None
            if vid is not None:
                ext.add(vid)
        for vid, _, _ in getattr(prog, 'feeds', {}).values():
            ext.add(vid)
        for vid in getattr(prog, '_fetch', []) or []:
            ext.add(vid)
        for vid in getattr(prog, '_ir_fetch', None) or ():
            ext.add(vid)
        self.external = ext
        self.meta = {}
        for m in getattr(prog, '_keep', []):
            vid = prog._val.get(id(m))
            if vid is not None:
                self.meta[vid] = m
        self.claimed = set()

    def producer(self, vid, before):
        for j in range(before - 1, -1, -1):
            if vid in self.outs[j]:
                return j
        return None

    def node(self, j):
        return None if j is None else self.nodes[j]

    def src(self, ref, before, chain):
        """Producer index of ``ref`` skipping pure casts (appended to ``chain``)."""
        if not isinstance(ref, Ref):
            return None
        j = self.producer(ref.vid, before)
        while j is not None:
            nj = self.nodes[j]
            k = _kind(nj)
            if k == 'cast' and self._pure_cast(nj):
                inner = nj.args[0]
            elif k in ('pd.cast', 'pd.assign') or (k == 'pd.dropout' and nj.target.attrs.get('is_test', False) and
                                                   nj.target.attrs.get('dropout_implementation') ==
                                                   'upscale_in_train'):
                inner = _pd_in(nj, 'X')
                if len(_outs_of(nj.outs, [])) != 1:
                    return None
            else:
                break
            chain.append(j)
            if not isinstance(inner, Ref):
                return None
            j = self.producer(inner.vid, j)
        return j

    @staticmethod
    def _pure_cast(n):
        """A dtype conversion / contiguous copy of one value (no device move, no other operand)."""
        if not n.args or not isinstance(n.args[0], Ref):
            return False
        for a in n.args[1:]:
            if not (isinstance(a, torch.dtype) or (n.target is torch.Tensor.type_as and isinstance(a, Ref))):
                return False
        for k, v in n.kwargs.items():
            if k in ('non_blocking', 'copy', 'memory_format') or (k == 'dtype' and isinstance(v, torch.dtype)):
                continue
            return False
        return True

    def private(self, idxs, keep=(), users=()):
        """Every output of the nodes ``idxs`` (except vids in ``keep``) is used only inside idxs
        (or by the nodes ``users``, e.g. the anchor a rewrite replaces)."""
        s = set(idxs) | set(users)
        for j in idxs:
            if j in self.claimed:
                return False
            for v in self.outs[j]:
                if v in keep:
                    continue
                if v in self.external or not self.uses.get(v, set()) <= s:
                    return False
        return True

    def rank(self, ref):
        m = self.meta.get(ref.vid) if isinstance(ref, Ref) else None
        return None if m is None else m.dim()


# ============================================================================ passes
def _scale_chain(g, j, chain):
    """Walks back over scalar mul / div (and casts) from node j; returns (j, scale)."""
    scale = 1.0
    while j is not None:
        n = g.nodes[j]
        k = _kind(n)
        if k == 'mul' and len(n.args) == 2:
            a, b = n.args
            if isinstance(a, Ref) and _num(b):
                scale *= float(b)
                x = a
            elif isinstance(b, Ref) and _num(a):
                scale *= float(a)
                x = b
            else:
                break
        elif k == 'div' and len(n.args) == 2 and isinstance(n.args[0], Ref) and _num(n.args[1]) and \
                not n.kwargs.get('rounding_mode'):
            scale /= float(n.args[1])
            x = n.args[0]
        elif k == 'pd.scale' and abs(n.target.attrs.get('bias', 0.0)) == 0.0:
            scale *= float(n.target.attrs.get('scale', 1.0))
            x = _pd_in(n, 'X')
        else:
            break
        chain.append(j)
        j = g.src(x, j, chain)
    return j, scale


def _attention(g, i):
    n = g.nodes[i]
    k = _kind(n)
    if k == 'matmul' and len(n.args) == 2 and not n.kwargs:
        p_ref, v_ref = n.args
    elif k in ('pd.matmul_v2', 'pd.matmul'):
        at = n.target.attrs
        if at.get('trans_x') or at.get('trans_y') or at.get('transpose_X') or at.get('transpose_Y') or \
                at.get('alpha', 1.0) != 1.0:
            return None
        p_ref, v_ref = _pd_in(n, 'X'), _pd_in(n, 'Y')
    else:
        return None
    if not isinstance(v_ref, Ref):
        return None
    chain = []
    j = g.src(p_ref, i, chain)
    drop = 0.0
    nj = g.node(j)
    if _kind(nj) == 'dropout':
        p = float(_arg(nj, 1, 'p', 0.5))
        if _arg(nj, 3, 'inplace', False):
            return None
        drop = p if _arg(nj, 2, 'training', True) else 0.0
        chain.append(j)
        j = g.src(nj.args[0], j, chain)
    elif _kind(nj) == 'pd.dropout':
        at = nj.target.attrs
        if not at.get('is_test', True) or at.get('dropout_implementation', 'downgrade_in_infer') != 'upscale_in_train':
            return None  # downgrade_in_infer scales the probabilities: keep the ops
        chain.append(j)
        j = g.src(_pd_in(nj, 'X'), j, chain)
    nj = g.node(j)
    if _kind(nj) == 'softmax':
        dim = _arg(nj, 1, 'dim', None)
        r = g.rank(nj.args[0])
        if dim is None or not (dim == -1 or (r is not None and dim == r - 1)) or nj.kwargs.get('dtype') is not None:
            return None
        s_ref = nj.args[0]
    elif _kind(nj) == 'pd.softmax':
        if nj.target.attrs.get('axis', -1) != -1:
            return None
        s_ref = _pd_in(nj, 'X')
    else:
        return None
    chain.append(j)
    j = g.src(s_ref, j, chain)
    mask, mode, fill = None, None, -1e30
    nj = g.node(j)
    kj = _kind(nj)
    if kj == 'masked_fill' and len(nj.args) == 3 and _num(nj.args[2]) and float(nj.args[2]) <= -1e4:
        x, m, fill = nj.args[0], nj.args[1], float(nj.args[2])
        if not isinstance(m, Ref):
            return None
        mj = g.producer(m.vid, j)
        if mj is not None and _kind(g.nodes[mj]) == 'invert' and isinstance(g.nodes[mj].args[0], Ref) and \
                m.vid not in g.external and g.uses.get(m.vid, set()) <= {j}:
            mask, mode = g.nodes[mj].args[0], 'keep'
            chain.append(mj)
        else:
            mask, mode = m, 'drop'
        chain.append(j)
        j = g.src(x, j, chain)
    elif kj == 'pd.where':
        cond, xv, yv = _pd_in(nj, 'Condition'), _pd_in(nj, 'X'), _pd_in(nj, 'Y')
        fj = g.producer(xv.vid, j) if isinstance(xv, Ref) else None
        fn = g.node(fj)
        if _kind(fn) != 'pd.fill_constant' or _pd_in(fn, 'ShapeTensor') is not None or \
                float(fn.target.attrs.get('value', 0.0)) > -1e4 or not isinstance(cond, Ref):
            return None
        fill = float(fn.target.attrs.get('value'))
        chain.append(fj)
        mj = g.producer(cond.vid, j)
        mn = g.node(mj)
        if _kind(mn) == 'pd.logical_not' and isinstance(_pd_in(mn, 'X'), Ref) and cond.vid not in g.external and \
                g.uses.get(cond.vid, set()) <= {j}:
            mask, mode = _pd_in(mn, 'X'), 'keep'
            chain.append(mj)
        else:
            mask, mode = cond, 'drop'
        chain.append(j)
        j = g.src(yv, j, chain)
    elif kj in ('add', 'pd.elementwise_add'):
        a, b = (nj.args[0], nj.args[1]) if kj == 'add' else (_pd_in(nj, 'X'), _pd_in(nj, 'Y'))
        if kj == 'add' and (len(nj.args) != 2 or nj.kwargs):
            return None
        if kj == 'pd.elementwise_add' and nj.target.attrs.get('axis', -1) not in (-1,):
            return None
        # the score operand leads back to the q @ k^T product; the other one is the additive mask
        picked = None
        for sc, mk in ((a, b), (b, a)):
            c2 = []
            t = g.src(sc, j, c2)
            t2, _ = _scale_chain(g, t, c2)
            if t2 is not None and _kind(g.nodes[t2]) in ('matmul', 'pd.matmul_v2', 'pd.matmul'):
                picked = (sc, mk)
                break
        if picked is None or not isinstance(picked[1], (Ref, Const)):
            return None
        mask, mode = picked[1], 'add'
        chain.append(j)
        j = g.src(picked[0], j, chain)
    j, scale = _scale_chain(g, j, chain)
    nj = g.node(j)
    kj = _kind(nj)
    if kj == 'matmul' and len(nj.args) == 2 and not nj.kwargs:
        q_ref, kt_ref = nj.args
        kt_given = True
    elif kj in ('pd.matmul_v2', 'pd.matmul'):
        at = nj.target.attrs
        if at.get('trans_x') or at.get('transpose_X'):
            return None
        q_ref, kt_ref = _pd_in(nj, 'X'), _pd_in(nj, 'Y')
        kt_given = not (at.get('trans_y') or at.get('transpose_Y'))
        scale *= float(at.get('alpha', 1.0))
    else:
        return None
    if not isinstance(q_ref, Ref) or not isinstance(kt_ref, Ref):
        return None
    chain.append(j)
    k_ref, k_transposed = kt_ref, kt_given
    if kt_given:
        tj = g.producer(kt_ref.vid, j)
        tn = g.node(tj)
        if _kind(tn) == 'transpose' and isinstance(tn.args[0], Ref) and len(tn.args) == 3:
            d0, d1 = tn.args[1], tn.args[2]
            r = g.rank(tn.args[0])
            last2 = {-1, -2} if r is None else {-1, -2, r - 1, r - 2}
            if d0 in last2 and d1 in last2 and d0 % 4 != d1 % 4 and kt_ref.vid not in g.external and \
                    g.uses.get(kt_ref.vid, set()) <= {j}:
                chain.append(tj)
                k_ref, k_transposed = tn.args[0], False
    for r_ in (q_ref, k_ref, v_ref):
        if g.rank(r_) not in (None, 4):
            return None
    # q / k / v as transposed slices 0 / 1 / 2 of one packed [B, S, 3, H, D] projection
    packed = None
    if not k_transposed:
        srcs = [_packed_slice(g, r_, idx, i) for idx, r_ in enumerate((q_ref, k_ref, v_ref))]
        if all(sr is not None for sr in srcs) and len({sr[0].vid for sr in srcs}) == 1 and \
                g.rank(srcs[0][0]) in (None, 5):
            body = sorted(set(chain + [j_ for sr in srcs for j_ in sr[1]]))
            if g.private(body, users=(i,)):
                packed = srcs[0][0]
    if packed is not None:
        node = Node('torch', fused_attention_packed, [packed, mask],
                    {'scale': scale, 'dropout': drop, 'mask_mode': mode, 'fill': fill},
                    _one_out(n), dict(n.meta or {}, fused='multihead_matmul_fuse_pass_v2'))
        return body + [i], {i: node}
    body = sorted(set(chain))
    if not g.private(body, users=(i,)):
        return None
    node = Node('torch', fused_attention, [q_ref, k_ref, v_ref, mask],
                {'scale': scale, 'dropout': drop, 'mask_mode': mode, 'k_transposed': k_transposed, 'fill': fill},
                _one_out(n), dict(n.meta or {}, fused='multihead_matmul_fuse_pass_v2'))
    return body + [i], {i: node}


def _packed_slice(g, ref, idx, before):
    """(P, [node indices]) when ``ref`` = P[:, :, idx].transpose(1, 2), else None."""
    tj = g.producer(ref.vid, before)
    tn = g.node(tj)
    if _kind(tn) != 'transpose' or len(tn.args) != 3 or not isinstance(tn.args[0], Ref) or \
            {tn.args[1], tn.args[2]} != {1, 2}:
        return None
    gj = g.producer(tn.args[0].vid, tj)
    gn = g.node(gj)
    if _kind(gn) != 'getitem' or len(gn.args) != 2 or not isinstance(gn.args[0], Ref):
        return None
    key = gn.args[1]
    full = slice(None, None, None)
    if not (isinstance(key, tuple) and len(key) == 3 and key[0] == full and key[1] == full and key[2] == idx):
        return None
    return gn.args[0], [tj, gj]


def _ln_args(n):
    """(x, weight, bias, eps) of a last-dim layer_norm node, else None."""
    k = _kind(n)
    if k == 'layer_norm':
        x = n.args[0]
        ns = _arg(n, 1, 'normalized_shape')
        w, b = _arg(n, 2, 'weight'), _arg(n, 3, 'bias')
        eps = _arg(n, 4, 'eps', 1e-5)
        if not isinstance(ns, (list, tuple, torch.Size)) or len(ns) != 1 or not isinstance(x, Ref):
            return None
        if n.kwargs.get('cudnn_enable') is not None:
            return None
        return x, w, b, float(eps)
    if k == 'pd.layer_norm':
        x = _pd_in(n, 'X')
        return (x, _pd_in(n, 'Scale'), _pd_in(n, 'Bias'), float(n.target.attrs.get('epsilon', 1e-5))) \
            if isinstance(x, Ref) else None
    return None


def _ln_rank_ok(g, n, x):
    """An imported layer_norm whose rank is known must normalise the last dim; with the rank
    unknown (ProgramDesc values carry no shapes here) the fused node checks begin_norm_axis at run
    time and takes the composite otherwise."""
    if _kind(n) == 'pd.layer_norm':
        r = g.rank(x)
        ax = n.target.attrs.get('begin_norm_axis', 1)
        return r is None or ax in (-1, r - 1)
    return True


def _ln_axis(n):
    return n.target.attrs.get('begin_norm_axis', 1) if _kind(n) == 'pd.layer_norm' else None


def _ln_out(n):
    if _kind(n) == 'pd.layer_norm':
        return _pd_out(n, 'Y')
    return n.outs


def _ln_extra_outs(n):
    """Mean / Variance outputs of an imported layer_norm (must be unused for a rewrite)."""
    if _kind(n) == 'pd.layer_norm':
        return [v for v in (_pd_out(n, 'Mean'), _pd_out(n, 'Variance')) if v is not None]
    return []


def _add_ln(g, i, with_dropout):
    n = g.nodes[i]
    la = _ln_args(n)
    if la is None or not _ln_rank_ok(g, n, la[0]):
        return None
    x, w, b, eps = la
    extra = _ln_extra_outs(n)
    if any(v in g.external or g.uses.get(v) for v in extra):
        return None
    aj = g.producer(x.vid, i)
    an = g.node(aj)
    ka = _kind(an)
    if ka == 'add' and len(an.args) == 2 and not an.kwargs:
        a, r = an.args
    elif ka == 'pd.elementwise_add' and an.target.attrs.get('axis', -1) == -1:
        a, r = _pd_in(an, 'X'), _pd_in(an, 'Y')
    else:
        return None
    if not isinstance(a, Ref) or not isinstance(r, (Ref, Const)):
        return None
    add_out = _outs_of(an.outs, [])
    if len(add_out) != 1:
        return None
    for xin, res in ((a, r), (r, a)):
        if not isinstance(xin, Ref):
            continue
        dj = g.producer(xin.vid, aj)
        dn = g.node(dj)
        if with_dropout:
            if _kind(dn) != 'dropout' or _arg(dn, 3, 'inplace', False) or not isinstance(dn.args[0], Ref):
                continue
            p = float(_arg(dn, 1, 'p', 0.5)) if _arg(dn, 2, 'training', True) else 0.0
            body = [dj, aj]
            if xin.vid in g.external or not g.uses.get(xin.vid, set()) <= {aj}:
                continue
            src = dn.args[0]
        else:
            p, body, src = 0.0, [aj], xin
        if not g.private(body, keep=set(add_out), users=(i,)) or i in g.claimed:
            return None
        # the fused node takes the add's place: norm parameters computed between the two are not
        # available there
        if any(isinstance(t, Ref) and (g.producer(t.vid, i) or -1) > aj for t in (w, b)):
            return None
        ln_out = _ln_out(n)
        node = Node('torch', fused_dropout_add_layer_norm, [src, res, w, b], {'eps': eps, 'p': p,
                                                                            'begin_axis': _ln_axis(n)},
                    [ln_out, add_out[0]], dict(n.meta or {},
                                               fused='fused_dropout_add_layernorm' if with_dropout else
                                               'skip_layernorm_fuse_pass'))
        # the fused node sits where the add was (its inputs are defined there); the norm node goes
        return body + [i], {aj: node}
    return None


def _layer_norm(g, i):
    n = g.nodes[i]
    la = _ln_args(n)
    if la is None or not _ln_rank_ok(g, n, la[0]):
        return None
    extra = _ln_extra_outs(n)
    if any(v in g.external or g.uses.get(v) for v in extra):
        return None
    x, w, b, eps = la
    node = Node('torch', fused_layer_norm, [x, w, b], {'eps': eps, 'begin_axis': _ln_axis(n)}, _ln_out(n),
                dict(n.meta or {}, fused='layer_norm_fuse_pass'))
    return [i], {i: node}


def _fc(g, i):
    """Imported ``matmul_v2`` / ``matmul`` / ``mul`` (x @ W) -> ``elementwise_add`` (bias) (-> relu /
    gelu) chains as one node: the bias in the GEMM epilogue, the activation in one pass (the
    recorded torch form already gets the bias from ``addmm``'s epilogue)."""
    n = g.nodes[i]
    k = _kind(n)
    if k not in ('pd.matmul_v2', 'pd.matmul', 'pd.mul'):
        return None
    at = n.target.attrs
    if at.get('trans_x') or at.get('transpose_X') or at.get('alpha', 1.0) != 1.0:
        return None
    x, w = _pd_in(n, 'X'), _pd_in(n, 'Y')
    if k == 'pd.mul':
        r = g.rank(x)
        if r is None or at.get('y_num_col_dims', 1) != 1 or at.get('x_num_col_dims', 1) != r - 1:
            return None
    trans = bool(at.get('trans_y') or at.get('transpose_Y'))
    if not isinstance(x, Ref) or not isinstance(w, Const):
        return None
    outs = _outs_of(n.outs, [])
    if len(outs) != 1:
        return None
    body, out_v, bias, tail = [i], outs, None, i
    uj = list(g.uses.get(outs[0], ()))
    if len(uj) == 1 and outs[0] not in g.external:
        an = g.nodes[uj[0]]
        if _kind(an) == 'pd.elementwise_add' and getattr(_pd_in(an, 'X'), 'vid', None) == outs[0] and \
                isinstance(_pd_in(an, 'Y'), Const) and an.target.attrs.get('axis', -1) in (-1, g.rank(x) - 1 if
                                                                                          g.rank(x) else -1):
            bias, tail = _pd_in(an, 'Y'), uj[0]
            body.append(uj[0])
            out_v = _outs_of(an.outs, [])
    act = None
    view = None  # a reshape2 between the bias add and the activation (the 3-D Linear export)
    if len(out_v) == 1:
        uj = list(g.uses.get(out_v[0], ()))
        if len(uj) == 1 and out_v[0] not in g.external and _kind(g.nodes[uj[0]]) == 'pd.reshape2':
            rn = g.nodes[uj[0]]
            r_out = rn.outs[0] if isinstance(rn.outs, list) and rn.outs else None
            xs = rn.outs[1] if isinstance(rn.outs, list) and len(rn.outs) > 1 else None
            uk = list(g.uses.get(r_out, ())) if r_out is not None else []
            if (r_out is not None and r_out not in g.external and len(uk) == 1 and
                    (xs is None or not g.uses.get(xs)) and _kind(g.nodes[uk[0]]) in ('pd.relu', 'pd.gelu')):
                view = uj[0]
                uj = uk
        if len(uj) == 1 and (view is not None or out_v[0] not in g.external):
            cn = g.nodes[uj[0]]
            kc = _kind(cn)
            if kc == 'pd.relu':
                act = 'relu'
            elif kc == 'pd.gelu':
                act = 'gelu_tanh' if cn.target.attrs.get('approximate', False) else 'gelu'
            if act is not None:
                if view is not None:
                    body.append(view)
                body.append(uj[0])
                tail = uj[0]
                act_out = _outs_of(cn.outs, [])
                if view is None:
                    out_v = act_out
            elif view is not None:
                view = None
    if len(body) == 1 or len(out_v) != 1 or not g.private(body[:-1], users=body[-1:]):
        return None  # a bare matmul already runs on the hand-written GEMM
    if view is not None:
        # act(x @ W + b) on the 2-D product, then the reshape re-targeted to the activation's output
        if len(act_out) != 1:
            return None
        rn = g.nodes[view]
        lin = Node('torch', fused_linear, [x, w, bias], {'act': act, 'trans_w': trans}, out_v[0],
                   dict(n.meta or {}, fused='fc_fuse_pass'))
        rs = Node(rn.kind, rn.target, list(rn.args), dict(rn.kwargs),
                  [act_out[0]] + [None] * (len(rn.outs) - 1), dict(rn.meta or {}))
        return body, {body[1]: lin, tail: rs}
    node = Node('torch', fused_linear, [x, w, bias], {'act': act, 'trans_w': trans}, out_v[0],
                dict(n.meta or {}, fused='fc_fuse_pass'))
    return body, {tail: node}


def _sole_user(g, vid, body):
    """Index of the single user of ``vid`` (a value private to the chain), else None."""
    if vid is None or isinstance(vid, (list, tuple)) or vid in g.external:
        return None
    uj = list(g.uses.get(vid, ()))
    return uj[0] if len(uj) == 1 and uj[0] not in body else None


def _ffn(g, i):
    """Recorded feed-forward blocks addmm(b1, x, W1) -> (reshape) -> gelu -> (reshape) ->
    addmm(b2, ., W2) (nn.Linear -> F.gelu -> nn.Linear) as one fused_ffn node — the reference's
    training-side fuse_gemm_epilogue_pass (linear + gelu forward, linear_grad + gelu_grad backward)."""
    n = g.nodes[i]
    if _kind(n) != 'addmm' or n.kwargs or len(n.args) != 3:
        return None
    b1, x, w1 = n.args
    if not isinstance(x, Ref) or not isinstance(w1, Const) or not isinstance(b1, Const):
        return None
    body, cur, approx = [i], _one_out(n), None
    while True:  # reshapes, then the gelu, then reshapes, then fc2
        j = _sole_user(g, cur, body)
        if j is None:
            return None
        m = g.nodes[j]
        k = _kind(m)
        if not m.args or not isinstance(m.args[0], Ref) or m.args[0].vid != cur:
            if k == 'addmm' and approx is not None and len(m.args) == 3 and isinstance(m.args[1], Ref) and \
                    m.args[1].vid == cur and not m.kwargs:
                break
            return None
        if k == 'reshape':
            pass
        elif k == 'gelu' and approx is None and m.target is TF.gelu and len(m.args) <= 2:
            approx = m.args[1] if len(m.args) == 2 else m.kwargs.get('approximate', 'none')
            if set(m.kwargs) - {'approximate'} or approx not in ('none', 'tanh'):
                return None
        else:
            return None
        body.append(j)
        cur = _one_out(m)
    b2, _, w2 = m.args
    if not isinstance(w2, Const) or not isinstance(b2, Const):
        return None
    body.append(j)
    if not g.private(body[:-1], users=body[-1:]):
        return None
    node = Node('torch', fused_ffn, [x, w1, b1, w2, b2], {'approximate': approx}, _one_out(m),
                dict(n.meta or {}, fused='fuse_gemm_epilogue_pass'))
    return body, {j: node}


def _softmax(g, i):
    n = g.nodes[i]
    k = _kind(n)
    # imported (inference) programs only: a recorded torch softmax runs in fp32 under autocast and
    # may feed a loss, the 16-bit kernel would change what it computes
    if k == 'pd.softmax':
        if n.target.attrs.get('axis', -1) != -1:
            return None
        x = _pd_in(n, 'X')
    else:
        return None
    return [i], {i: Node('torch', fused_softmax, [x], {}, _one_out(n), dict(n.meta or {}, fused='softmax_fuse_pass'))}


def _quant_linear(g, i):
    """An imported onnx-format int8 GEMM (the reference's quantised inference models and this
    framework's saved PTQ / QAT models) as one paddle.ops.int8.quant_linear node."""
    n = g.nodes[i]
    if _kind(n) != 'pd.matmul_v2' or n.target.attrs.get('trans_x'):
        return None
    xd, wd = _pd_in(n, 'X'), _pd_in(n, 'Y')
    if not isinstance(xd, Ref) or not isinstance(wd, Ref):
        return None
    dj, wj = g.producer(xd.vid, i), g.producer(wd.vid, i)
    dn, wn = g.node(dj), g.node(wj)
    if _kind(dn) != 'pd.dequantize_linear' or _kind(wn) != 'pd.dequantize_linear':
        return None
    qv = _pd_in(dn, 'X')
    qj = g.producer(qv.vid, dj) if isinstance(qv, Ref) else None
    qn = g.node(qj)
    if _kind(qn) != 'pd.quantize_linear' or qn.target.attrs.get('quant_axis', -1) not in (-1, None) or \
            dn.target.attrs.get('quant_axis', -1) not in (-1, None):
        return None
    x, acs = _pd_in(qn, 'X'), _pd_in(qn, 'Scale')
    wq, ws = _pd_in(wn, 'X'), _pd_in(wn, 'Scale')
    if not isinstance(x, Ref) or not isinstance(wq, Const) or not isinstance(ws, Const) or acs is None:
        return None
    trans = bool(n.target.attrs.get('trans_y'))
    if wn.target.attrs.get('quant_axis', 0) != (0 if trans else 1):
        return None
    body, tail, bias = [qj, dj, wj, i], i, None
    out_v = _outs_of(n.outs, [])
    uj = list(g.uses.get(out_v[0], ()))
    if len(uj) == 1 and out_v[0] not in g.external:
        an = g.nodes[uj[0]]
        if _kind(an) == 'pd.elementwise_add' and getattr(_pd_in(an, 'X'), 'vid', None) == out_v[0] and \
                isinstance(_pd_in(an, 'Y'), Const):
            bias, tail = _pd_in(an, 'Y'), uj[0]
            body.append(uj[0])
            out_v = _outs_of(an.outs, [])
    if not trans or len(out_v) != 1 or not g.private(body[:-1] if tail != i else [qj, dj, wj], users=(i, tail)):
        return None
    from ..ops.int8 import quant_linear
    node = Node('torch', quant_linear, [x, wq, ws, acs, bias], {'bits': qn.target.attrs.get('bit_length', 8),
                                                                 'weight_bits': wn.target.attrs.get('bit_length', 8)},
                out_v[0], dict(n.meta or {}, fused='quant_linear_fuse_pass'))
    return body, {tail: node}


_PASSES = {
    'quant_linear_fuse_pass': _quant_linear,
    'multihead_matmul_fuse_pass_v2': _attention,
    'fused_dropout_add_layernorm': lambda g, i: _add_ln(g, i, True),
    'skip_layernorm_fuse_pass': lambda g, i: _add_ln(g, i, False),
    'fuse_gemm_epilogue_pass': _ffn,
    'layer_norm_fuse_pass': _layer_norm,
    'fc_fuse_pass': _fc,
    'softmax_fuse_pass': _softmax,
}


from . import ir_passes_ext as _ext  # noqa: E402
_ext.register()


def pass_names():
    return list(_PASSES)


def apply_passes(prog, nodes=None, passes=None, fetch=None):
    """The node list of ``prog`` with every match of ``passes`` (default DEFAULT_PASSES, in order)
    rewritten; returns (nodes, {pass name: match count}).  ``fetch``: value ids read after the run
    (a loaded program knows its own); without them the whole-list passes (dead-code and common-
    subexpression elimination), which must know what is read, are skipped."""
    nodes = list(prog.nodes if nodes is None else nodes)
    stats = {}
    if fetch is None and getattr(prog, '_fetch', None):
        fetch = tuple(prog._fetch)
    prev_fetch = getattr(prog, '_ir_fetch', None)
    prog._ir_fetch = fetch
    try:
        return _apply(prog, nodes, passes, fetch, stats)
    finally:
        prog._ir_fetch = prev_fetch


def _apply(prog, nodes, passes, fetch, stats):
    for name in (passes if passes is not None else DEFAULT_PASSES):
        fn = _PASSES[name]
        if getattr(fn, '_whole_list', False):  # DCE / CSE: whole-list rewrites
            if fetch is None:
                continue
            nodes, cnt = fn(prog, nodes)
            if cnt:
                stats[name] = stats.get(name, 0) + cnt
            continue
        g = _Graph(prog, nodes)
        remove, replace = set(), {}
        for i in range(len(nodes)):
            if i in g.claimed:
                continue
            r = fn(g, i)
            if r is None:
                continue
            body, rep = r
            if any(j in g.claimed for j in body):
                continue
            g.claimed.update(body)
            remove.update(body)
            replace.update(rep)
            stats[name] = stats.get(name, 0) + 1
        if replace:
            nodes = [replace[i] if i in replace else n for i, n in enumerate(nodes)
                     if i in replace or i not in remove]
    return nodes, stats


def _enabled(prog, dev):
    mode = _MODE[0]
    if getattr(prog, '_ir_optim', None) is False or mode in ('0', 'off', 'false'):
        return False
    if mode in ('1', 'always', 'true'):
        return True
    return dev is not None and torch.device(dev).type == 'cuda'


def ir_nodes(prog, dev, fetch=None):
    """The node list the Executor / Predictor runs: the fused rewrite of prog.nodes (cached per
    program version, pass list and fetch set), or prog.nodes itself when fusion is off."""
    if not _enabled(prog, dev) or not prog.nodes:
        return prog.nodes
    passes = getattr(prog, '_ir_passes', None)
    passes = tuple(DEFAULT_PASSES if passes is None else passes)
    key = (len(prog.nodes), id(prog.nodes[-1]), passes, fetch)
    c = getattr(prog, '_ir_cache', None)
    if c is not None and c[0] == key:
        return c[1]
    nodes, stats = apply_passes(prog, passes=passes, fetch=fetch)
    prog._ir_cache = (key, nodes)
    prog._ir_stats = stats
    return nodes


def fusion_stats(prog):
    """{pass name: number of rewrites} of the program's last fused version."""
    return dict(getattr(prog, '_ir_stats', {}) or {})


_ = math
