"""The reference's PIR program format: ``<prefix>.json`` written by ``save_pir`` / jit.save under
FLAGS_enable_pir_api (python/paddle/static/pir_io.py:527 save_pir, :610 load_pir) with the schema
of paddle/fluid/pir/serialize_deserialize (include/schema.h keys, ir_serialize.cc / ir_deserialize.cc
layout):

  {"base_code": {"magic": "pir", "version": V, "trainable": false},
   "program": {"regions": [{"#": "region_0", "blocks": [{"#": "block_0", "args": [], "ops": [...]}]}]}}

  op        {"#": "<dialect id>.<op>", "I": [{"%": value id}], "O": [{"%": id, "TT": type}],
             "A": [{"N": attr name, "AT": {"#": "<dialect>.<attr kind>", "D": data}}]}
  parameter {"#": "p", "O": {"%": id, "TT": type}, "A": [is_distributed, is_parameter, need_clip, name]}
  type      {"#": "0.t_dtensor", "D": [{"#": "0.t_f32"}, dims, "NCHW", lod, offset]}
  dialects  0 = builtin, 1 = pd_op, 2 = cf

Values are numbered from 1 in definition order (0 = null operand).  Mutable attributes (IntArray /
Scalar arguments of ops.yaml such as reshape's shape or pool2d's kernel_size) are operands produced
by pd_op.full_int_array / pd_op.full; vector operands by builtin.combine.

Export lowers a recorded Program through the same operator lowering as the ProgramDesc exporter
(static/pdmodel.py) and translates each legacy operator to its PIR form (ops.yaml argument order
and names); import translates each pd_op operation back to the legacy operator implementations of
pdmodel.OPS, folding full / full_int_array operands into attributes, so the loaded program runs on
the same op implementations (and the hand-written GEMM for matmul) as an imported ProgramDesc.
Parameters travel in the .pdiparams combine stream (sorted names), as in the reference.
"""
import json

import torch

from . import proto as P
from . import pdmodel as PM
from .program import Ref, Const, Node

PIR_VERSION = 1
_DIALECT = {'builtin': '0', 'pd_op': '1', 'cf': '2', 'custom_op': '3'}
_DIALECT_R = {v: k for k, v in _DIALECT.items()}

_TYPE_OF = {torch.float32: 't_f32', torch.float16: 't_f16', torch.bfloat16: 't_bf16', torch.float64: 't_f64',
            torch.int8: 't_i8', torch.uint8: 't_ui8', torch.int16: 't_i16', torch.int32: 't_i32',
            torch.int64: 't_i64', torch.bool: 't_bool', torch.complex64: 't_c64', torch.complex128: 't_c128'}
_TORCH_OF_TYPE = {v: k for k, v in _TYPE_OF.items()}
_DTYPE_STR = {torch.float32: 'float32', torch.float16: 'float16', torch.bfloat16: 'bfloat16',
              torch.float64: 'float64', torch.int8: 'int8', torch.uint8: 'uint8', torch.int16: 'int16',
              torch.int32: 'int32', torch.int64: 'int64', torch.bool: 'bool', torch.complex64: 'complex64',
              torch.complex128: 'complex128'}
_TORCH_OF_STR = {v: k for k, v in _DTYPE_STR.items()}

# ------------------------------------------------------------------------------------------------
# legacy operator <-> PIR operation (ops.yaml argument order).  'ins': tensor slot names of the legacy
# op in operand order; '*S' = a vector operand (builtin.combine) of slot S; '@a' = a mutable-attribute
# operand holding legacy attribute a (full_int_array for int lists, full for scalars); None = an
# optional operand the legacy op does not have.  'outs': legacy output slots in result order (None =
# a result the legacy op lacks).  'attrs': PIR attribute -> (legacy attribute, kind).
# ------------------------------------------------------------------------------------------------
_B, _I32, _I64, _F32, _STR = 'bool', 'i32', 'i64', 'f32', 'str'
_I32S, _I64S, _IA, _DT = 'i32s', 'i64s', 'intarray', 'dtype'


SPEC = {
    'conv2d': dict(leg='conv2d', ins=['Input', 'Filter'], outs=['Output'],
                   attrs={'strides': ('strides', _I32S), 'paddings': ('paddings', _I32S),
                          'padding_algorithm': ('padding_algorithm', _STR), 'dilations': ('dilations', _I32S),
                          'groups': ('groups', _I32), 'data_format': ('data_format', _STR)}),
    'depthwise_conv2d': dict(leg='depthwise_conv2d', ins=['Input', 'Filter'], outs=['Output'],
                             attrs={'strides': ('strides', _I32S), 'paddings': ('paddings', _I32S),
                                    'padding_algorithm': ('padding_algorithm', _STR), 'groups': ('groups', _I32),
                                    'dilations': ('dilations', _I32S), 'data_format': ('data_format', _STR)}),
    'conv2d_transpose': dict(leg='conv2d_transpose', ins=['Input', 'Filter', '@output_size'], outs=['Output'],
                             attrs={'strides': ('strides', _I32S), 'paddings': ('paddings', _I32S),
                                    'output_padding': ('output_padding', _I32S),
                                    'padding_algorithm': ('padding_algorithm', _STR), 'groups': ('groups', _I32),
                                    'dilations': ('dilations', _I32S), 'data_format': ('data_format', _STR)}),
    'pool2d': dict(leg='pool2d', ins=['X', '@ksize'], outs=['Out'],
                   attrs={'strides': ('strides', _I32S), 'paddings': ('paddings', _I32S),
                          'ceil_mode': ('ceil_mode', _B), 'exclusive': ('exclusive', _B),
                          'data_format': ('data_format', _STR), 'pooling_type': ('pooling_type', _STR),
                          'global_pooling': ('global_pooling', _B), 'adaptive': ('adaptive', _B),
                          'padding_algorithm': ('padding_algorithm', _STR)}),
    'batch_norm': dict(leg='batch_norm', ins=['X', 'Mean', 'Variance', 'Scale', 'Bias'],
                       outs=['Y', 'MeanOut', 'VarianceOut', 'SavedMean', 'SavedVariance', None],
                       attrs={'is_test': ('is_test', _B), 'momentum': ('momentum', _F32), 'epsilon': ('epsilon', _F32),
                              'data_format': ('data_layout', _STR), 'use_global_stats': ('use_global_stats', _B),
                              'trainable_statistics': ('trainable_statistics', _B)}),
    'layer_norm': dict(leg='layer_norm', ins=['X', 'Scale', 'Bias'], outs=['Y', 'Mean', 'Variance'],
                       attrs={'epsilon': ('epsilon', _F32), 'begin_norm_axis': ('begin_norm_axis', _I32)}),
    'group_norm': dict(leg='group_norm', ins=['X', 'Scale', 'Bias'], outs=['Y', 'Mean', 'Variance'],
                       attrs={'epsilon': ('epsilon', _F32), 'groups': ('groups', _I32),
                              'data_format': ('data_layout', _STR)}),
    'instance_norm': dict(leg='instance_norm', ins=['X', 'Scale', 'Bias'], outs=['Y', 'SavedMean', 'SavedVariance'],
                          attrs={'epsilon': ('epsilon', _F32)}),
    'matmul': dict(leg='matmul_v2', ins=['X', 'Y'], outs=['Out'],
                   attrs={'transpose_x': ('trans_x', _B), 'transpose_y': ('trans_y', _B)}),
    'bmm': dict(leg='bmm', ins=['X', 'Y'], outs=['Out'], attrs={}),
    'fc': dict(leg='fc', ins=['Input', 'W', 'Bias'], outs=['Out'],
               attrs={'in_num_col_dims': ('in_num_col_dims', _I32), 'activation_type': ('activation_type', _STR)}),
    'add': dict(leg='elementwise_add', ins=['X', 'Y'], outs=['Out'], attrs={}),
    'subtract': dict(leg='elementwise_sub', ins=['X', 'Y'], outs=['Out'], attrs={}),
    'multiply': dict(leg='elementwise_mul', ins=['X', 'Y'], outs=['Out'], attrs={}),
    'divide': dict(leg='elementwise_div', ins=['X', 'Y'], outs=['Out'], attrs={}),
    'maximum': dict(leg='elementwise_max', ins=['X', 'Y'], outs=['Out'], attrs={}),
    'minimum': dict(leg='elementwise_min', ins=['X', 'Y'], outs=['Out'], attrs={}),
    'elementwise_pow': dict(leg='elementwise_pow', ins=['X', 'Y'], outs=['Out'], attrs={}),
    'floor_divide': dict(leg='elementwise_floordiv', ins=['X', 'Y'], outs=['Out'], attrs={}),
    'remainder': dict(leg='elementwise_mod', ins=['X', 'Y'], outs=['Out'], attrs={}),
    'gelu': dict(leg='gelu', ins=['X'], outs=['Out'], attrs={'approximate': ('approximate', _B)}),
    'softmax': dict(leg='softmax', ins=['X'], outs=['Out'], attrs={'axis': ('axis', _I32)}),
    'log_softmax': dict(leg='log_softmax', ins=['X'], outs=['Out'], attrs={'axis': ('axis', _I32)}),
    'leaky_relu': dict(leg='leaky_relu', ins=['X'], outs=['Out'], attrs={'negative_slope': ('alpha', _F32)}),
    'hardsigmoid': dict(leg='hard_sigmoid', ins=['X'], outs=['Out'],
                        attrs={'slope': ('slope', _F32), 'offset': ('offset', _F32)}),
    'softplus': dict(leg='softplus', ins=['X'], outs=['Out'],
                     attrs={'beta': ('beta', _F32), 'threshold': ('threshold', _F32)}),
    'elu': dict(leg='elu', ins=['X'], outs=['Out'], attrs={'alpha': ('alpha', _F32)}),
    'celu': dict(leg='celu', ins=['X'], outs=['Out'], attrs={'alpha': ('alpha', _F32)}),
    'pow': dict(leg='pow', ins=['X'], outs=['Out'], attrs={'y': ('factor', _F32)}),
    'scale': dict(leg='scale', ins=['X', '@scale'], outs=['Out'],
                  attrs={'bias': ('bias', _F32), 'bias_after_scale': ('bias_after_scale', _B)}),
    'reshape': dict(leg='reshape2', ins=['X', '@shape'], outs=['Out', 'XShape'], attrs={}),
    'transpose': dict(leg='transpose2', ins=['X'], outs=['Out'], attrs={'perm': ('axis', _I32S)}),
    'flatten': dict(leg='flatten_contiguous_range', ins=['X'], outs=['Out', 'XShape'],
                    attrs={'start_axis': ('start_axis', _I32), 'stop_axis': ('stop_axis', _I32)}),
    'concat': dict(leg='concat', ins=['*X', '@axis'], outs=['Out'], attrs={}),
    'stack': dict(leg='stack', ins=['*X'], outs=['Y'], attrs={'axis': ('axis', _I32)}),
    'unsqueeze': dict(leg='unsqueeze2', ins=['X', '@axes'], outs=['Out', 'XShape'], attrs={}),
    'squeeze': dict(leg='squeeze2', ins=['X', '@axes'], outs=['Out', 'XShape'], attrs={}),
    'mean': dict(leg='reduce_mean', ins=['X'], outs=['Out'], attrs={'axis': ('dim', _IA), 'keepdim': ('keep_dim', _B)}),
    'sum': dict(leg='reduce_sum', ins=['X', '@dim'], outs=['Out'], attrs={'keepdim': ('keep_dim', _B)}),
    'max': dict(leg='reduce_max', ins=['X', '@dim'], outs=['Out'], attrs={'keepdim': ('keep_dim', _B)}),
    'min': dict(leg='reduce_min', ins=['X', '@dim'], outs=['Out'], attrs={'keepdim': ('keep_dim', _B)}),
    'prod': dict(leg='reduce_prod', ins=['X', '@dim'], outs=['Out'],
                 attrs={'keepdim': ('keep_dim', _B), 'reduce_all': ('reduce_all', _B)}),
    'embedding': dict(leg='lookup_table_v2', ins=['Ids', 'W'], outs=['Out'],
                      attrs={'padding_idx': ('padding_idx', _I64), 'sparse': ('is_sparse', _B)}),
    'assign': dict(leg='assign', ins=['X'], outs=['Out'], attrs={}),
    'cast': dict(leg='cast', ins=['X'], outs=['Out'], attrs={'dtype': ('out_dtype', _DT)}),
    'clip': dict(leg='clip', ins=['X', '@min', '@max'], outs=['Out'], attrs={}),
    'slice': dict(leg='slice', ins=['Input', '@starts', '@ends'], outs=['Out'],
                  attrs={'axes': ('axes', _I64S), 'infer_flags': ('infer_flags', _I64S),
                         'decrease_axis': ('decrease_axis', _I64S)}),
    'argmax': dict(leg='arg_max', ins=['X', '@axis'], outs=['Out'],
                   attrs={'keepdims': ('keepdims', _B), 'flatten': ('flatten', _B)}),
    'argmin': dict(leg='arg_min', ins=['X', '@axis'], outs=['Out'],
                   attrs={'keepdims': ('keepdims', _B), 'flatten': ('flatten', _B)}),
    'dropout': dict(leg='dropout', ins=['X', None, '@dropout_prob'], outs=['Out', 'Mask'],
                    attrs={'is_test': ('is_test', _B), 'mode': ('dropout_implementation', _STR)}),
    'shape': dict(leg='shape', ins=['Input'], outs=['Out'], attrs={}),
    'gather': dict(leg='gather', ins=['X', 'Index', '@axis'], outs=['Out'], attrs={}),
    'where': dict(leg='where', ins=['Condition', 'X', 'Y'], outs=['Out'], attrs={}),
    'tril': dict(leg='tril_triu', ins=['X'], outs=['Out'], attrs={'diagonal': ('diagonal', _I32)}, fixed={'lower': True}),
    'triu': dict(leg='tril_triu', ins=['X'], outs=['Out'], attrs={'diagonal': ('diagonal', _I32)},
                 fixed={'lower': False}),
    'expand': dict(leg='expand_v2', ins=['X', '@shape'], outs=['Out'], attrs={}),
    'tile': dict(leg='tile', ins=['X', '@repeat_times'], outs=['Out'], attrs={}),
    'cumsum': dict(leg='cumsum', ins=['X', '@axis'], outs=['Out'],
                   attrs={'flatten': ('flatten', _B), 'exclusive': ('exclusive', _B), 'reverse': ('reverse', _B)}),
    'topk': dict(leg='top_k_v2', ins=['X', '@k'], outs=['Out', 'Indices'],
                 attrs={'axis': ('axis', _I32), 'largest': ('largest', _B), 'sorted': ('sorted', _B)}),
    'one_hot': dict(leg='one_hot_v2', ins=['X', '@depth'], outs=['Out'], attrs={}),
    'index_select': dict(leg='index_select', ins=['X', 'Index'], outs=['Out'], attrs={'axis': ('dim', _I32)}),
    'p_norm': dict(leg='p_norm', ins=['X'], outs=['Out'],
                   attrs={'porder': ('porder', _F32), 'axis': ('axis', _I32), 'epsilon': ('epsilon', _F32),
                          'keepdim': ('keepdim', _B), 'asvector': ('asvector', _B)}),
    'pad3d': dict(leg='pad3d', ins=['X', '@paddings'], outs=['Out'],
                  attrs={'mode': ('mode', _STR), 'pad_value': ('value', _F32), 'data_format': ('data_format', _STR)}),
    'prelu': dict(leg='prelu', ins=['X', 'Alpha'], outs=['Out'],
                  attrs={'data_format': ('data_format', _STR), 'mode': ('mode', _STR)}),
    'argsort': dict(leg='argsort', ins=['X'], outs=['Out', 'Indices'],
                    attrs={'axis': ('axis', _I32), 'descending': ('descending', _B)}),
    'flip': dict(leg='flip', ins=['X'], outs=['Out'], attrs={'axis': ('axis', _I32S)}),
    'roll': dict(leg='roll', ins=['X', '@shifts'], outs=['Out'], attrs={'axis': ('axis', _I64S)}),
    'add_n': dict(leg='sum', ins=['*X'], outs=['Out'], attrs={}),
    'split': dict(leg='split', ins=['X', '@sections', '@axis'], outs=['*Out'], attrs={}),
    'split_with_num': dict(leg='split', ins=['X', '@axis'], outs=['*Out'], attrs={'num': ('num', _I32)}),
    'unstack': dict(leg='unstack', ins=['X'], outs=['*Y'], attrs={'axis': ('axis', _I32), 'num': ('num', _I32)}),
    'bilinear_interp': dict(leg='bilinear_interp_v2', ins=['X', 'OutSize', None, None], outs=['Out'],
                            attrs={'data_format': ('data_layout', _STR), 'out_h': ('out_h', _I32),
                                   'out_w': ('out_w', _I32), 'scale': ('scale', 'f32s'),
                                   'interp_method': ('interp_method', _STR),
                                   'align_corners': ('align_corners', _B), 'align_mode': ('align_mode', _I32)}),
    'nearest_interp': dict(leg='nearest_interp_v2', ins=['X', 'OutSize', None, None], outs=['Out'],
                           attrs={'data_format': ('data_layout', _STR), 'out_h': ('out_h', _I32),
                                  'out_w': ('out_w', _I32), 'scale': ('scale', 'f32s'),
                                  'interp_method': ('interp_method', _STR),
                                  'align_corners': ('align_corners', _B), 'align_mode': ('align_mode', _I32)}),
    'full_like': dict(leg='fill_any_like', ins=['X', '@value'], outs=['Out'], attrs={'dtype': ('dtype', _DT)}),
    'equal': dict(leg='equal', ins=['X', 'Y'], outs=['Out'], attrs={}),
    'not_equal': dict(leg='not_equal', ins=['X', 'Y'], outs=['Out'], attrs={}),
    'less_than': dict(leg='less_than', ins=['X', 'Y'], outs=['Out'], attrs={}),
    'less_equal': dict(leg='less_equal', ins=['X', 'Y'], outs=['Out'], attrs={}),
    'greater_than': dict(leg='greater_than', ins=['X', 'Y'], outs=['Out'], attrs={}),
    'greater_equal': dict(leg='greater_equal', ins=['X', 'Y'], outs=['Out'], attrs={}),
    'logical_and': dict(leg='logical_and', ins=['X', 'Y'], outs=['Out'], attrs={}),
    'logical_or': dict(leg='logical_or', ins=['X', 'Y'], outs=['Out'], attrs={}),
    'logical_xor': dict(leg='logical_xor', ins=['X', 'Y'], outs=['Out'], attrs={}),
    'logical_not': dict(leg='logical_not', ins=['X'], outs=['Out'], attrs={}),
}
for _n in ('relu', 'tanh', 'sigmoid', 'silu', 'exp', 'sqrt', 'rsqrt', 'abs', 'relu6', 'sin', 'cos', 'log', 'square',
           'sign', 'floor', 'ceil', 'round', 'reciprocal', 'erf', 'mish', 'selu', 'swish'):
    SPEC[_n] = dict(leg=_n, ins=['X'], outs=['Out'], attrs={})
SPEC['hardswish'] = dict(leg='hard_swish', ins=['X'], outs=['Out'], attrs={})

# legacy type -> PIR name (the first spec naming it; tril_triu / split pick by attributes)
_LEG2PIR = {}
for _k, _v in SPEC.items():
    _LEG2PIR.setdefault(_v['leg'], _k)
_LEG2PIR['elementwise_add'] = 'add'


# ============================================================================ JSON helpers
def _dt_type(dt):
    return {'#': '0.' + _TYPE_OF[dt]}


def _tensor_type(dt, shape, layout='NCHW'):
    return {'#': '0.t_dtensor', 'D': [_dt_type(dt), [int(s) for s in shape], layout, [], 0]}


def _attr(kind, v):
    if kind == _B:
        return {'#': '0.a_bool', 'D': bool(v)}
    if kind == _I32:
        return {'#': '0.a_i32', 'D': int(v)}
    if kind == _I64:
        return {'#': '0.a_i64', 'D': int(v)}
    if kind == _F32:
        return {'#': '0.a_f32', 'D': float(v)}
    if kind == 'f64':
        return {'#': '0.a_f64', 'D': float(v)}
    if kind == _STR:
        return {'#': '0.a_str', 'D': str(v)}
    if kind == _I32S:
        return {'#': '0.a_array', 'D': [_attr(_I32, x) for x in (v or [])]}
    if kind == _I64S:
        return {'#': '0.a_array', 'D': [_attr(_I64, x) for x in (v or [])]}
    if kind == 'f32s':
        return {'#': '0.a_array', 'D': [_attr(_F32, x) for x in (v or [])]}
    if kind == _IA:
        return {'#': '1.a_intarray', 'D': [int(x) for x in (v if isinstance(v, (list, tuple)) else [v])]}
    if kind == _DT:
        dt = v if isinstance(v, torch.dtype) else P.torch_dtype(int(v))
        return {'#': '1.a_dtype', 'D': _DTYPE_STR[dt]}
    if kind == 'place':
        return {'#': '1.a_place', 'D': [1, 0, '']}  # phi::AllocationType::CPU, device 0
    if kind == 'scalar':
        return {'#': '1.a_scalar', 'D': ['float32', float(v)]}
    raise PM.Unsupported(f"PIR attribute kind {kind}")


def _attr_value(a):
    """Decode one attribute JSON object to a Python value (ints / floats / str / lists / dtypes)."""
    kind = a['#'].split('.', 1)[1]
    d = a.get('D')
    if kind == 'a_array':
        return [_attr_value(x) for x in d]
    if kind == 'a_dtype':
        return _TORCH_OF_STR.get(d, torch.float32)
    if kind == 'a_scalar':
        return d[1] if isinstance(d, list) and len(d) > 1 else d
    if kind in ('a_place', 'a_layout', 'a_pointer', 'a_type'):
        return d
    return d


def _type_info(tt):
    """(dtype, shape) of a value type JSON (dtensor), or (None, None)."""
    if not tt or tt.get('#') != '0.t_dtensor':
        return None, None
    d = tt['D']
    return _TORCH_OF_TYPE.get(d[0]['#'].split('.', 1)[1], torch.float32), [int(s) for s in d[1]]


# ============================================================================ export
class _Collector(PM._Exporter):
    """pdmodel's lowering with the ProgramDesc writer replaced by an op list."""

    def __init__(self, prog):
        super().__init__(prog)
        self.ops = []
        self.vmeta = {}

    def _var(self, name, dt=None, shape=None, persistable=False):
        if name not in self.vmeta:
            self.vmeta[name] = (dt, list(shape or []), persistable)
        self.vars[name] = True
        return name

    def _special(self, name, typ):
        self.vars[name] = True

    def op(self, typ, inputs, outputs, **attrs):
        self.ops.append((typ, {k: (v if isinstance(v, list) else [v]) for k, v in inputs.items()},
                         {k: (v if isinstance(v, list) else [v]) for k, v in outputs.items()}, attrs))


class _Writer:
    def __init__(self):
        self.ops = []
        self.next_id = 1
        self.ids = {}    # legacy var name -> value id
        self.types = {}  # value id -> type json

    def value(self, tt):
        vid = self.next_id
        self.next_id += 1
        self.types[vid] = tt
        return vid

    def emit(self, name, operands, results_tt, attrs):
        outs = [self.value(tt) for tt in results_tt]
        self.ops.append({'#': name, 'I': [{'%': i} for i in operands],
                         'O': [{'%': o, 'TT': self.types[o]} for o in outs],
                         'A': [{'N': k, 'AT': v} for k, v in attrs]})
        return outs


def _legacy_to_pir(w, coll, typ, ins, outs, at):
    if typ in ('feed', 'fetch'):
        return
    pname = _LEG2PIR.get(typ)
    if typ == 'tril_triu':
        pname = 'tril' if at.get('lower', True) else 'triu'
    if pname is None:
        raise PM.Unsupported(f"no PIR form for legacy op {typ}")
    spec = SPEC[pname]

    def vt(name):
        dt, shape, _ = coll.vmeta.get(name, (torch.float32, [], False))
        return _tensor_type(dt or torch.float32, shape)
    operands = []
    if typ.startswith('elementwise_') and at.get('axis', -1) not in (-1, None):
        # PIR's binary ops broadcast numpy-style: the legacy 'axis' alignment becomes a reshape of Y
        # to [1]*axis + Y.shape + [1]*rest (as the reference's program translator does)
        xr = max(len(coll.vmeta.get(ins['X'][0], (None, [], False))[1]),
                 len(coll.vmeta.get((outs.get('Out') or [''])[0], (None, [], False))[1]))
        yd, ys, _ = coll.vmeta.get(ins['Y'][0], (torch.float32, [], False))
        ax = int(at['axis'])
        if xr and len(ys) < xr and ax >= 0:
            shape = [1] * ax + list(ys) + [1] * (xr - ax - len(ys))
            sh = w.emit('1.full_int_array', [], [_tensor_type(torch.int64, [len(shape)])],
                        [('value', _attr(_I64S, shape)), ('dtype', _attr(_DT, torch.int64)),
                         ('place', _attr('place', None))])
            yr = w.emit('1.reshape', [w.ids[ins['Y'][0]]] + sh,
                        [_tensor_type(yd or torch.float32, shape), _tensor_type(yd or torch.float32, [])], [])
            ins = dict(ins)
            ins['Y'] = ['__bcast_y__']
            w.ids['__bcast_y__'] = yr[0]
    for slot in spec['ins']:
        if slot is None:
            operands.append(0)
        elif slot.startswith('*'):
            names = ins.get(slot[1:], [])
            vec_tt = {'#': '0.t_vec', 'D': [w.types[w.ids[n]] for n in names]}
            operands.extend(w.emit('0.combine', [w.ids[n] for n in names], [vec_tt], []))
        elif slot.startswith('@'):
            val = at.get(slot[1:])
            if isinstance(val, (list, tuple)):
                operands.extend(w.emit('1.full_int_array', [], [_tensor_type(torch.int64, [len(val)])],
                                       [('value', _attr(_I64S, val)), ('dtype', _attr(_DT, torch.int64)),
                                        ('place', _attr('place', None))]))
            elif val is None:
                operands.append(0)
            else:
                operands.extend(w.emit('1.full', [], [_tensor_type(torch.float32, [1])],
                                       [('shape', _attr(_IA, [1])), ('value', _attr('f64', float(val))),
                                        ('dtype', _attr(_DT, torch.float32)), ('place', _attr('place', None))]))
        else:
            names = ins.get(slot, [])
            operands.append(w.ids[names[0]] if names else 0)
    attrs = []
    for pa, (la, kind) in spec['attrs'].items():
        if la in at:
            attrs.append((pa, _attr(kind, at[la])))
    res_tt, res_names = [], []
    for slot in spec['outs']:
        names = outs.get(slot, []) if slot else []
        n = names[0] if names else None
        res_names.append(n)
        res_tt.append(vt(n) if n else _tensor_type(torch.float32, []))
    rids = w.emit('1.' + pname, operands, res_tt, attrs)
    for n, r in zip(res_names, rids):
        if n:
            w.ids[n] = r


def export(prog, feed_names, fetch_vids, trainable=False):
    """Recorded Program -> (PIR JSON bytes, [(param name, tensor)]).  Raises pdmodel.Unsupported
    for operators outside the lowered set (as the ProgramDesc exporter does)."""
    coll = _Collector(prog)
    feed_vid = {prog.feeds[n][0]: n for n in feed_names}
    orig = coll.name_of

    def name_of(a):
        if isinstance(a, Ref) and a.vid in feed_vid:
            return feed_vid[a.vid]
        return orig(a)
    coll.name_of = name_of
    for n in prog.nodes:
        if n.kind != 'torch':
            raise PM.Unsupported(f"node kind {n.kind}")
        if not isinstance(n.outs, int):
            raise PM.Unsupported("multi-output node")
        PM._emit(coll, n)
    w = _Writer()
    # parameters first (builtin.parameter, compressed "p"), in sorted-name order like .pdiparams
    for name, t in sorted(coll.params.items()):
        vid = w.value(_tensor_type(t.dtype, list(t.shape)))
        w.ids[name] = vid
        w.ops.append({'#': 'p', 'O': {'%': vid, 'TT': w.types[vid]}, 'A': [0, 1, 1, name]})
    for i, name in enumerate(feed_names):
        vid_, shape, dt = prog.feeds[name]
        shp = [-1 if s in PM._SENT else int(s) for s in shape]
        (r,) = w.emit('1.data', [], [_tensor_type(dt, shp)],
                      [('name', _attr(_STR, name)), ('shape', _attr(_IA, shp)), ('dtype', _attr(_DT, dt)),
                       ('place', _attr('place', None))])
        w.ids[name] = r
    for typ, ins, outs, at in coll.ops:
        _legacy_to_pir(w, coll, typ, ins, outs, at)
    for i, vid in enumerate(fetch_vids):
        nm = coll.name_of(Ref(vid))
        src = w.ids[nm]
        w.emit('1.fetch', [src], [w.types[src]], [('name', _attr(_STR, f'fetch_name_{i}')), ('col', _attr(_I32, i))])
    doc = {'base_code': {'magic': 'pir', 'version': PIR_VERSION, 'trainable': bool(trainable)},
           'program': {'regions': [{'#': 'region_0', 'blocks': [{'#': 'block_0', 'args': [], 'ops': w.ops}]}]}}
    return json.dumps(doc).encode(), sorted(coll.params.items())


# ============================================================================ import
def is_pir_json(data):
    head = bytes(data[:4096]) if isinstance(data, (bytes, bytearray)) else str(data[:4096]).encode()
    return head.lstrip()[:1] == b'{' and b'"base_code"' in head


def _dialect_op(name):
    if name == 'p':
        return 'builtin', 'parameter'
    d, _, op = name.partition('.')
    return _DIALECT_R.get(d, d), op


def load(data):
    """PIR JSON bytes -> LoadedProgram whose nodes run pdmodel.OPS implementations."""
    from .io import LoadedProgram
    from ..core.tensor import _wrap
    doc = json.loads(data.decode() if isinstance(data, (bytes, bytearray)) else data)
    base = doc.get('base_code', {})
    if base.get('magic') != 'pir':
        raise ValueError("not a PIR program file (base_code.magic != 'pir')")
    regions = doc['program']['regions']
    blocks = regions[0]['blocks']
    ops = blocks[0]['ops']
    prog = LoadedProgram()
    prog._const_names = {}
    env = {}      # value id -> Ref | Const | ('const', python value) | ('vec', [ids])
    vtypes = {}
    feeds, fetch = [], []
    pending_vec = {}  # vector value id -> (node builder) for ops with vector results

    def new_ref():
        return Ref(next(prog._vid))

    def const_tensor(val, dt=torch.float32, shape=None):
        """A full / full_int_array result used as a tensor operand (moved to the device with the
        parameters, pdmodel.load_params)."""
        cid = len(prog.consts)
        if isinstance(val, (list, tuple)):
            t = torch.tensor(list(val), dtype=dt)
        else:
            t = torch.full([int(s) for s in (shape or [])], val, dtype=dt)
        prog.consts[cid] = t
        return Const(cid)

    def operand(i):
        if i == 0:
            return None
        v = env[i]
        if isinstance(v, tuple) and v[0] == 'const':
            val, dt, shape = v[1], v[2], v[3]
            c = const_tensor(val, dt, shape)
            env[i] = c
            return c
        return v

    def const_value(i):
        v = env.get(i)
        if isinstance(v, tuple) and v[0] == 'const':
            return v[1]
        raise PM.Unsupported("a mutable-attribute operand that is not a full / full_int_array constant")

    for op in ops:
        dialect, name = _dialect_op(op['#'])
        if op['#'] == 'p':
            o = op['O']
            pname = op['A'][3]
            cid = len(prog.consts)
            prog.consts[cid] = None
            prog._const_names[cid] = pname
            env[o['%']] = Const(cid)
            vtypes[o['%']] = o.get('TT')
            continue
        attrs = {a['N']: _attr_value(a['AT']) for a in op.get('A', [])}
        ins = [x['%'] for x in op.get('I', [])]
        outs = op.get('O', [])
        for o in outs:
            vtypes[o['%']] = o.get('TT')
        if dialect == 'pd_op' and name == 'data':
            r = new_ref()
            env[outs[0]['%']] = r
            dt, shape = _type_info(outs[0].get('TT'))
            feeds.append((attrs['name'], r.vid, attrs.get('shape', shape), attrs.get('dtype', dt)))
            continue
        if dialect == 'pd_op' and name == 'fetch':
            fetch.append((attrs.get('col', len(fetch)), ins[0]))
            continue
        if dialect == 'pd_op' and name == 'full_int_array':
            env[outs[0]['%']] = ('const', [int(x) for x in attrs['value']], torch.int64, None)
            continue
        if dialect == 'pd_op' and name == 'full':
            dt = attrs.get('dtype', torch.float32)
            dt = dt if isinstance(dt, torch.dtype) else torch.float32
            shape = attrs.get('shape', [1])
            val = attrs.get('value', 0.0)
            if not dt.is_floating_point and not dt.is_complex:
                val = bool(val) if dt == torch.bool else int(val)
            env[outs[0]['%']] = ('const', val, dt, shape)
            continue
        if dialect == 'builtin' and name == 'combine':
            env[outs[0]['%']] = ('vec', ins)
            continue
        if dialect == 'builtin' and name in ('split', 'slice'):
            src = ins[0]
            if src in pending_vec:
                pending_vec.pop(src)([o['%'] for o in outs] if name == 'split' else None, attrs)
            if name == 'slice':
                raise PM.Unsupported("builtin.slice of a vector")
            continue
        if dialect == 'builtin' and name in ('shadow_output', 'set_parameter'):
            if name == 'shadow_output' and outs:
                env[outs[0]['%']] = env.get(ins[0])
            continue
        if dialect != 'pd_op':
            raise NotImplementedError(f"PIR operation {op['#']} is not supported by this runtime")
        base = name[:-1] if name.endswith('_') and name[:-1] in SPEC else name  # inplace variants
        spec = SPEC.get(base)
        if spec is None:
            raise NotImplementedError(f"PIR operation pd_op.{name} is not supported by this runtime")
        leg_at = dict(spec.get('fixed', {}))
        for pa, (la, kind) in spec['attrs'].items():
            if pa in attrs:
                v = attrs[pa]
                if kind == _DT and isinstance(v, torch.dtype):
                    v = P.dtype_code(v)
                leg_at[la] = v
        slots, args = [], []
        for slot, i in zip(spec['ins'], ins + [0] * (len(spec['ins']) - len(ins))):
            if slot is None or i == 0:
                continue
            if slot.startswith('@'):
                leg_at[slot[1:]] = const_value(i)
            elif slot.startswith('*'):
                vec = env[i]
                ids = vec[1] if isinstance(vec, tuple) and vec[0] == 'vec' else [i]
                vals = [operand(j) for j in ids]
                slots.append((slot[1:], len(vals)))
                args.extend(vals)
            else:
                slots.append((slot, 1))
                args.append(operand(i))
        if spec['leg'] in ('reduce_mean', 'reduce_sum', 'reduce_max', 'reduce_min', 'reduce_prod'):
            d = leg_at.get('dim', [])
            d = [d] if isinstance(d, int) else list(d)
            leg_at['dim'] = d
            leg_at.setdefault('reduce_all', not d)
        if spec['leg'] == 'pool2d' and isinstance(leg_at.get('ksize'), int):
            leg_at['ksize'] = [leg_at['ksize']] * 2
        vec_out = spec['outs'] and spec['outs'][0] is not None and spec['outs'][0].startswith('*')

        def build(out_ids, _a=None, spec=spec, slots=slots, args=args, leg_at=leg_at):
            if vec_out:
                oslot = spec['outs'][0][1:]
                out_slots = [(oslot, len(out_ids))]
                refs = []
                for oid in out_ids:
                    r = new_ref()
                    env[oid] = r
                    refs.append(r.vid)
                prog.nodes.append(Node('torch', PM._OpCall(spec['leg'], slots, out_slots, leg_at), args, {}, refs))
                return
            out_slots = []
            refs = []
            for slot, oid in zip(spec['outs'], out_ids):
                if slot is None:
                    continue
                r = new_ref()
                env[oid] = r
                out_slots.append((slot, 1))
                refs.append(r.vid)
            prog.nodes.append(Node('torch', PM._OpCall(spec['leg'], slots, out_slots, leg_at), args, {}, refs))
        if vec_out:
            pending_vec[outs[0]['%']] = build
        else:
            build([o['%'] for o in outs])
    for name, vid, shape, dt in feeds:
        shape = [int(s) for s in (shape or [])]
        dt = dt if isinstance(dt, torch.dtype) else torch.float32
        prog.feeds[name] = (vid, shape, dt)
        m = torch.empty([max(s, 1) for s in shape], dtype=dt, device='meta')
        prog._val[id(m)] = vid
        prog._keep.append(m)
        var = _wrap(m)
        var._name = name
        prog.named_vars[name] = var
    prog._fetch = []
    for _, vid in sorted(fetch):
        v = env[vid]
        if isinstance(v, Const):  # a parameter fetched directly: route through an identity node
            r = new_ref()
            prog.nodes.append(Node('torch', PM._OpCall('assign', [('X', 1)], [('Out', 1)], {}), [v], {}, [r.vid]))
            v = r
        prog._fetch.append(v.vid)
    prog._fetch_vars = []
    for vid in prog._fetch:
        m = torch.empty(0, device='meta')
        prog._val[id(m)] = vid
        prog._keep.append(m)
        prog._fetch_vars.append(_wrap(m))
    prog._pdmodel = True
    prog._pir = True
    return prog
