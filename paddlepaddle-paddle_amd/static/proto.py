"""The reference's on-disk program / tensor formats, without protoc or any reference binary.

* ``ProgramDesc`` & friends: the message set of paddle/fluid/framework/framework.proto
  (package ``paddle.framework.proto``: ProgramDesc:264, BlockDesc, VarDesc, VarType,
  OpDesc, Version, OpVersionMap), declared here as a FileDescriptorProto and materialised with
  google.protobuf's descriptor pool, so ``.pdmodel`` files parse and serialise byte-compatibly.
* LoDTensor streams (paddle/fluid/framework/lod_tensor.cc:205 SerializeToStream,
  tensor_util.cc:455 TensorToStream): ``uint32 version=0 | uint64 lod_level | per level
  (uint64 bytes, size_t offsets) | uint32 version=0 | int32 desc_size | TensorDesc | raw data``.
  A ``.pdiparams`` file is the concatenation of these for every persistable variable in
  sorted-name order (the save_combine op); a per-variable file holds one.
"""
import io
import struct

import numpy as np
import torch
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_F = descriptor_pb2.FieldDescriptorProto
_OPT, _REQ, _REP = _F.LABEL_OPTIONAL, _F.LABEL_REQUIRED, _F.LABEL_REPEATED
_T = {'int32': _F.TYPE_INT32, 'int64': _F.TYPE_INT64, 'float': _F.TYPE_FLOAT, 'double': _F.TYPE_DOUBLE,
      'string': _F.TYPE_STRING, 'bool': _F.TYPE_BOOL}

ATTR_TYPES = ['INT', 'FLOAT', 'STRING', 'INTS', 'FLOATS', 'STRINGS', 'BOOLEAN', 'BOOLEANS', 'BLOCK', 'LONG',
              'BLOCKS', 'LONGS', 'FLOAT64S', 'VAR', 'VARS', 'FLOAT64', 'SCALAR', 'SCALARS']
VAR_TYPES = {'BOOL': 0, 'INT16': 1, 'INT32': 2, 'INT64': 3, 'FP16': 4, 'FP32': 5, 'FP64': 6, 'LOD_TENSOR': 7,
             'SELECTED_ROWS': 8, 'FEED_MINIBATCH': 9, 'FETCH_LIST': 10, 'STEP_SCOPES': 11, 'LOD_RANK_TABLE': 12,
             'LOD_TENSOR_ARRAY': 13, 'PLACE_LIST': 14, 'READER': 15, 'RAW': 17, 'TUPLE': 18, 'SIZE_T': 19,
             'UINT8': 20, 'INT8': 21, 'BF16': 22, 'COMPLEX64': 23, 'COMPLEX128': 24, 'STRING': 25, 'STRINGS': 26,
             'VOCAB': 27, 'FEED_LIST': 28, 'PSTRING': 29, 'SPARSE_COO': 30, 'SPARSE_CSR': 31}


def _msg(parent, name, fields, enums=None, nested=None):
    m = parent.add()
    m.name = name
    for num, (fname, label, ftype, default) in fields.items():
        f = m.field.add()
        f.name, f.number, f.label = fname, num, label
        if ftype in _T:
            f.type = _T[ftype]
        elif ftype.startswith('enum:'):
            f.type = _F.TYPE_ENUM
            f.type_name = ftype[5:]
        else:
            f.type = _F.TYPE_MESSAGE
            f.type_name = ftype
        if default is not None:
            f.default_value = default
    for ename, vals in (enums or {}).items():
        e = m.enum_type.add()
        e.name = ename
        for k, v in vals.items():
            ev = e.value.add()
            ev.name, ev.number = k, v
    for fn in nested or ():
        fn(m.nested_type)
    return m


def _build():
    fd = descriptor_pb2.FileDescriptorProto()
    fd.name = 'paddle_amd/framework.proto'
    fd.package = 'paddle.framework.proto'
    fd.syntax = 'proto2'
    P = '.paddle.framework.proto.'
    e = fd.enum_type.add()
    e.name = 'AttrType'
    for i, n in enumerate(ATTR_TYPES):
        v = e.value.add()
        v.name, v.number = n, i
    _msg(fd.message_type, 'Version', {1: ('version', _OPT, 'int64', '0')})
    _msg(fd.message_type, 'Complex', {1: ('r', _REQ, 'double', None), 2: ('i', _REQ, 'double', None)})
    _msg(fd.message_type, 'Scalar', {1: ('type', _REQ, 'enum:' + P + 'Scalar.Type', None),
                                     2: ('b', _OPT, 'bool', None), 3: ('i', _OPT, 'int64', None),
                                     4: ('r', _OPT, 'double', None), 5: ('c', _OPT, P + 'Complex', None)},
         enums={'Type': {'BOOLEAN': 1, 'LONG': 2, 'FLOAT64': 3, 'COMPLEX128': 4}})

    def op_attr(nt):
        _msg(nt, 'Attr', {1: ('name', _REQ, 'string', None), 2: ('type', _REQ, 'enum:' + P + 'AttrType', None),
                          3: ('i', _OPT, 'int32', None), 4: ('f', _OPT, 'float', None),
                          5: ('s', _OPT, 'string', None), 6: ('ints', _REP, 'int32', None),
                          7: ('floats', _REP, 'float', None), 8: ('strings', _REP, 'string', None),
                          10: ('b', _OPT, 'bool', None), 11: ('bools', _REP, 'bool', None),
                          12: ('block_idx', _OPT, 'int32', None), 13: ('l', _OPT, 'int64', None),
                          14: ('blocks_idx', _REP, 'int32', None), 15: ('longs', _REP, 'int64', None),
                          16: ('float64s', _REP, 'double', None), 17: ('var_name', _OPT, 'string', None),
                          18: ('vars_name', _REP, 'string', None), 19: ('float64', _OPT, 'double', None),
                          20: ('scalar', _OPT, P + 'Scalar', None), 21: ('scalars', _REP, P + 'Scalar', None)})

    def op_var(nt):
        _msg(nt, 'Var', {1: ('parameter', _REQ, 'string', None), 2: ('arguments', _REP, 'string', None)})

    _msg(fd.message_type, 'OpDesc', {3: ('type', _REQ, 'string', None), 1: ('inputs', _REP, P + 'OpDesc.Var', None),
                                     2: ('outputs', _REP, P + 'OpDesc.Var', None),
                                     4: ('attrs', _REP, P + 'OpDesc.Attr', None),
                                     5: ('is_target', _OPT, 'bool', 'false')}, nested=[op_attr, op_var])
    VT = P + 'VarType.Type'

    def tdesc(nt):
        _msg(nt, 'TensorDesc', {1: ('data_type', _REQ, 'enum:' + VT, None), 2: ('dims', _REP, 'int64', None)})

    def lodt(nt):
        _msg(nt, 'LoDTensorDesc', {1: ('tensor', _REQ, P + 'VarType.TensorDesc', None),
                                   2: ('lod_level', _OPT, 'int32', '0')})

    def lodta(nt):
        _msg(nt, 'LoDTensorArrayDesc', {1: ('tensor', _REQ, P + 'VarType.TensorDesc', None),
                                        2: ('lod_level', _OPT, 'int32', '0')})

    def reader(nt):
        _msg(nt, 'ReaderDesc', {1: ('lod_tensor', _REP, P + 'VarType.LoDTensorDesc', None)})

    def tup(nt):
        _msg(nt, 'Tuple', {1: ('element_type', _REP, 'enum:' + VT, None)})

    TD = P + 'VarType.TensorDesc'
    _msg(fd.message_type, 'VarType', {1: ('type', _REQ, 'enum:' + VT, None), 2: ('selected_rows', _OPT, TD, None),
                                      3: ('lod_tensor', _OPT, P + 'VarType.LoDTensorDesc', None),
                                      4: ('tensor_array', _OPT, P + 'VarType.LoDTensorArrayDesc', None),
                                      5: ('reader', _OPT, P + 'VarType.ReaderDesc', None),
                                      7: ('tuple', _OPT, P + 'VarType.Tuple', None), 8: ('string', _OPT, TD, None),
                                      9: ('strings', _OPT, TD, None), 10: ('vocab', _OPT, TD, None),
                                      11: ('sparse_coo', _OPT, TD, None), 12: ('sparse_csr', _OPT, TD, None)},
         enums={'Type': VAR_TYPES}, nested=[tdesc, lodt, lodta, reader, tup])

    def var_attr(nt):
        _msg(nt, 'Attr', {1: ('name', _REQ, 'string', None), 2: ('type', _REQ, 'enum:' + P + 'AttrType', None),
                          3: ('i', _OPT, 'int32', None), 4: ('s', _OPT, 'string', None),
                          5: ('ints', _REP, 'int32', None)})

    _msg(fd.message_type, 'VarDesc', {1: ('name', _REQ, 'string', None), 2: ('type', _REQ, P + 'VarType', None),
                                      3: ('persistable', _OPT, 'bool', 'false'),
                                      4: ('need_check_feed', _OPT, 'bool', 'false'),
                                      5: ('is_parameter', _OPT, 'bool', 'false'),
                                      6: ('stop_gradient', _OPT, 'bool', 'false'),
                                      7: ('attrs', _REP, P + 'VarDesc.Attr', None)}, nested=[var_attr])
    _msg(fd.message_type, 'BlockDesc', {1: ('idx', _REQ, 'int32', None), 2: ('parent_idx', _REQ, 'int32', None),
                                        3: ('vars', _REP, P + 'VarDesc', None), 4: ('ops', _REP, P + 'OpDesc', None),
                                        5: ('forward_block_idx', _OPT, 'int32', '-1')})
    _msg(fd.message_type, 'OpVersion', {1: ('version', _REQ, 'int32', None)})

    def pair(nt):
        _msg(nt, 'OpVersionPair', {1: ('op_name', _REQ, 'string', None),
                                   2: ('op_version', _REQ, P + 'OpVersion', None)})

    _msg(fd.message_type, 'OpVersionMap', {1: ('pair', _REP, P + 'OpVersionMap.OpVersionPair', None)}, nested=[pair])
    pd = _msg(fd.message_type, 'ProgramDesc', {1: ('blocks', _REP, P + 'BlockDesc', None),
                                              4: ('version', _OPT, P + 'Version', None),
                                              5: ('op_version_map', _OPT, P + 'OpVersionMap', None)})
    r = pd.reserved_range.add()
    r.start, r.end = 2, 4
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    get = lambda n: message_factory.GetMessageClass(pool.FindMessageTypeByName('paddle.framework.proto.' + n))
    return {n: get(n) for n in ('ProgramDesc', 'BlockDesc', 'VarDesc', 'VarType', 'OpDesc', 'Version',
                                'OpVersionMap', 'Scalar')}


_M = _build()
ProgramDesc = _M['ProgramDesc']
BlockDesc = _M['BlockDesc']
VarDesc = _M['VarDesc']
VarType = _M['VarType']
OpDesc = _M['OpDesc']

# ------------------------------------------------------------------- dtypes
_NP_OF = {0: np.bool_, 1: np.int16, 2: np.int32, 3: np.int64, 4: np.float16, 5: np.float32, 6: np.float64,
          20: np.uint8, 21: np.int8, 22: np.uint16, 23: np.complex64, 24: np.complex128}
_TORCH_OF = {0: torch.bool, 1: torch.int16, 2: torch.int32, 3: torch.int64, 4: torch.float16, 5: torch.float32,
             6: torch.float64, 20: torch.uint8, 21: torch.int8, 22: torch.bfloat16, 23: torch.complex64,
             24: torch.complex128}
_CODE_OF = {v: k for k, v in _TORCH_OF.items()}


def dtype_code(dt):
    """framework.proto VarType.Type code of a torch dtype."""
    return _CODE_OF[dt]


def torch_dtype(code):
    return _TORCH_OF[code]


# ------------------------------------------------------------------- LoDTensor streams
def tensor_to_stream(t, lod=()):
    """Bytes of one LoDTensor (reference SerializeToStream): t is a torch tensor (any device)."""
    t = t.detach().contiguous().cpu()
    code = dtype_code(t.dtype)
    out = io.BytesIO()
    out.write(struct.pack('<I', 0))
    out.write(struct.pack('<Q', len(lod)))
    for level in lod:
        arr = np.asarray(level, dtype=np.uint64)
        out.write(struct.pack('<Q', arr.nbytes))
        out.write(arr.tobytes())
    out.write(struct.pack('<I', 0))
    desc = VarType.TensorDesc()
    desc.data_type = code
    desc.dims.extend(list(t.shape))
    blob = desc.SerializeToString()
    out.write(struct.pack('<i', len(blob)))
    out.write(blob)
    if t.dtype == torch.bfloat16:
        out.write(t.view(torch.int16).numpy().tobytes())
    else:
        out.write(t.numpy().tobytes())
    return out.getvalue()


def tensor_from_stream(f):
    """Read one LoDTensor from a binary file object; returns (torch tensor on CPU, lod)."""
    hdr = f.read(4)
    if len(hdr) < 4:
        raise EOFError("no tensor in stream")
    (ver,) = struct.unpack('<I', hdr)
    if ver != 0:
        raise ValueError(f"Tensor version {ver} is not supported (not a paddle LoDTensor stream)")
    (levels,) = struct.unpack('<Q', f.read(8))
    lod = []
    for _ in range(levels):
        (nb,) = struct.unpack('<Q', f.read(8))
        lod.append(np.frombuffer(f.read(nb), dtype=np.uint64).tolist())
    (ver2,) = struct.unpack('<I', f.read(4))
    if ver2 != 0:
        raise ValueError(f"tensor version {ver2} is not supported")
    (dsz,) = struct.unpack('<i', f.read(4))
    desc = VarType.TensorDesc()
    desc.ParseFromString(f.read(dsz))
    shape = list(desc.dims)
    npdt = _NP_OF[desc.data_type]
    n = int(np.prod(shape)) if shape else 1
    raw = f.read(n * np.dtype(npdt).itemsize)
    arr = np.frombuffer(raw, dtype=npdt).reshape(shape).copy()
    if desc.data_type == 22:
        t = torch.from_numpy(arr.view(np.int16)).view(torch.bfloat16)
    else:
        t = torch.from_numpy(arr)
    return t, lod


def save_combine(named_tensors):
    """``.pdiparams`` bytes: LoDTensor streams of every (name, tensor) in sorted-name order."""
    return b''.join(tensor_to_stream(t) for _, t in sorted(named_tensors, key=lambda kv: kv[0]))


def load_combine(data, names):
    """Inverse of save_combine for the given (sorted) variable names -> {name: tensor}."""
    f = io.BytesIO(data)
    out = {}
    for n in sorted(names):
        out[n], _ = tensor_from_stream(f)
    return out
