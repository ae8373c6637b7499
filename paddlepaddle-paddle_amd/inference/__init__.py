"""paddle.inference (reference: python/paddle/inference/__init__.py, wrapper.py;
paddle/fluid/inference/api/analysis_predictor.cc).

A Predictor runs a program saved by ``jit.save`` / ``static.save_inference_model`` on one
MI355X.  Input/output handles mirror the reference's zero-copy tensors.  With
``Config.enable_hip_graph()`` a fixed-shape predictor captures the whole program into one
HIP graph on its first run and replays it afterwards (the launch-bound small-batch case).
Weights can be converted to bf16 with ``convert_to_mixed_precision``.
"""
from enum import Enum

import numpy as np
import torch


class PrecisionType(Enum):
    Float32 = 0
    Int8 = 1
    Half = 2
    Bfloat16 = 3


class PlaceType(Enum):
    UNK = -1
    CPU = 0
    GPU = 1
    XPU = 2
    CUSTOM = 4


class DataType(Enum):
    FLOAT32 = 0
    INT64 = 1
    INT32 = 2
    UINT8 = 3
    INT8 = 4
    FLOAT16 = 5
    BOOL = 6
    FLOAT64 = 7
    BFLOAT16 = 8


_NP2DT = {np.float32: DataType.FLOAT32, np.int64: DataType.INT64, np.int32: DataType.INT32, np.uint8: DataType.UINT8,
          np.int8: DataType.INT8, np.float16: DataType.FLOAT16, np.bool_: DataType.BOOL, np.float64: DataType.FLOAT64}


def get_version():
    from .. import __version__
    return f"paddle_amd {__version__} (MI355X / gfx950, ROCm)"


def get_num_bytes_of_data_type(dtype):
    return {DataType.FLOAT32: 4, DataType.INT64: 8, DataType.INT32: 4, DataType.UINT8: 1, DataType.INT8: 1,
            DataType.FLOAT16: 2, DataType.BOOL: 1, DataType.FLOAT64: 8, DataType.BFLOAT16: 2}[dtype]


class Config:
    def __init__(self, model_file=None, params_file=None):
        mf = str(model_file) if model_file is not None else None
        ext = next((e for e in ('.pdmodel', '.json') if mf is not None and mf.endswith(e)), None)
        if mf is not None and params_file is None and ext is None:
            self._prefix = mf.rstrip('/') + '/inference'  # model_dir form
        elif mf is not None:
            # <prefix>.pdmodel (ProgramDesc / this framework's IR) or <prefix>.json (the reference's PIR)
            self._prefix = mf[:-len(ext)] if ext else mf
        else:
            self._prefix = None
        self._use_gpu = torch.cuda.is_available()
        self._device_id = 0
        self._precision = PrecisionType.Float32
        self._hip_graph = False
        self._ir_optim = True
        self._memory_optim = False
        self._threads = 1

    def set_model(self, model_file, params_file=None):
        self.__init__(model_file, params_file)

    def model_dir(self):
        return self._prefix

    def prog_file(self):
        import os
        if not os.path.exists(self._prefix + '.pdmodel') and os.path.exists(self._prefix + '.json'):
            return self._prefix + '.json'
        return self._prefix + '.pdmodel'

    def params_file(self):
        return self._prefix + '.pdiparams'

    def enable_use_gpu(self, memory_pool_init_size_mb=100, device_id=0, precision_mode=PrecisionType.Float32):
        self._use_gpu = True
        self._device_id = device_id
        self._precision = precision_mode

    def disable_gpu(self):
        self._use_gpu = False

    def use_gpu(self):
        return self._use_gpu

    def gpu_device_id(self):
        return self._device_id

    def enable_hip_graph(self):
        self._hip_graph = True

    enable_cuda_graph = enable_hip_graph

    def switch_ir_optim(self, x=True):
        self._ir_optim = x

    def pass_builder(self):
        """The IR fusion pass list applied to the loaded program (reference
        paddle_pass_builder.h PassStrategy: passes / delete_pass / append_pass / insert_pass)."""
        if getattr(self, '_pass_builder', None) is None:
            self._pass_builder = PassStrategy()
        return self._pass_builder

    def delete_pass(self, name):
        self.pass_builder().delete_pass(name)

    def ir_optim(self):
        return self._ir_optim

    def enable_memory_optim(self, x=True):
        self._memory_optim = x

    def set_cpu_math_library_num_threads(self, n):
        self._threads = n
        torch.set_num_threads(n)

    def enable_mkldnn(self):
        pass

    def disable_glog_info(self):
        pass

    def switch_use_feed_fetch_ops(self, x=False):
        pass

    def switch_specify_input_names(self, x=True):
        pass

    def enable_tensorrt_engine(self, *a, **k):
        import warnings
        warnings.warn("TensorRT is not available on MI355X; running the program on HIP kernels instead")

    def enable_low_precision_io(self, x=True):
        pass

    def summary(self):
        return (f"model: {self._prefix}\nuse_gpu: {self._use_gpu} (device {self._device_id})\n"
                f"precision: {self._precision.name}\nhip_graph: {self._hip_graph}")


class PassStrategy:
    """Ordered IR pass names (static/ir_passes.py); unknown names are kept but ignored."""

    def __init__(self, passes=None):
        from ..static.ir_passes import DEFAULT_PASSES
        self._passes = list(DEFAULT_PASSES if passes is None else passes)
        self._debug = False

    def passes(self):
        return list(self._passes)

    def all_passes(self):
        return self.passes()

    def delete_pass(self, name):
        self._passes = [p for p in self._passes if p != name]

    def append_pass(self, name):
        self._passes.append(name)

    def insert_pass(self, idx, name):
        self._passes.insert(idx, name)

    def clear_passes(self):
        self._passes = []

    def turn_on_debug(self):
        self._debug = True

    def _known(self):
        from ..static.ir_passes import pass_names
        known = set(pass_names())
        return [p for p in self._passes if p in known]


class Tensor:
    """Zero-copy style input/output handle."""

    def __init__(self, name, predictor, is_input):
        self._name = name
        self._pred = predictor
        self._is_input = is_input
        self._shape = None

    def name(self):
        return self._name

    def reshape(self, shape):
        self._shape = list(shape)

    def copy_from_cpu(self, data):
        a = np.ascontiguousarray(data)
        self._pred._inputs[self._name] = torch.from_numpy(a).to(self._pred._dev)

    def share_external_data(self, data):
        from ..core.tensor import Tensor as PT
        t = data._t if isinstance(data, PT) else data
        self._pred._inputs[self._name] = t

    def copy_to_cpu(self):
        t = self._value()
        t = t.detach()
        return (t.float() if t.dtype == torch.bfloat16 else t).cpu().numpy()

    def _value(self):
        if self._is_input:
            return self._pred._inputs[self._name]
        return self._pred._outputs[self._name]

    def shape(self):
        try:
            return list(self._value().shape)
        except KeyError:
            return self._shape or []

    def type(self):
        t = self._value()
        return _NP2DT.get(np.dtype(str(t.dtype).replace('torch.', '')).type if t.dtype != torch.bfloat16 else None,
                          DataType.BFLOAT16)


class Predictor:
    def __init__(self, config):
        from ..static.io import load_inference_model
        from ..core.place import to_device
        self._config = config
        self._dev = to_device(f'gpu:{config._device_id}') if (config._use_gpu and torch.cuda.is_available()) else \
            torch.device('cpu')

        class _Exe:
            _dev = self._dev
        self._program, self._feeds, self._fetch = load_inference_model(config._prefix, _Exe())
        if config._precision in (PrecisionType.Half, PrecisionType.Bfloat16):
            dt = torch.float16 if config._precision == PrecisionType.Half else torch.bfloat16
            owners = getattr(self._program, '_const_owner', None) or {}
            for cid, t in list(self._program.consts.items()):
                o = owners.get(cid)  # a loaded parameter resolves through its owner (executor._resolve)
                src = o._t if o is not None else t
                if isinstance(src, torch.Tensor) and src.is_floating_point():
                    self._program.consts[cid] = src.to(dt)
                    if o is not None:
                        o._t = self._program.consts[cid]
            if getattr(self._program, '_pdmodel', False):
                from ..static.pdmodel import set_float_dtype
                set_float_dtype(self._program, dt)
        # IR fusion passes (static/ir_passes.py) on the loaded program: switch_ir_optim(False) turns
        # them off, pass_builder() edits the list
        self._program._ir_optim = bool(config._ir_optim)
        pb = getattr(config, '_pass_builder', None)
        if pb is not None:
            self._program._ir_passes = tuple(pb._known())
        self._out_names = [f"fetch_{i}" for i in range(len(self._fetch))]
        self._inputs = {}
        self._outputs = {}
        self._graph = None

    def get_input_names(self):
        return list(self._feeds)

    def get_output_names(self):
        return list(self._out_names)

    def get_input_handle(self, name):
        return Tensor(name, self, True)

    def get_output_handle(self, name):
        return Tensor(name, self, False)

    def _run_once(self, feeds):
        from ..static.executor import run_program
        from ..static.program import _vid_of
        env = run_program(self._program, feeds, self._dev, grad=False)
        return [env[_vid_of(self._program, v)] for v in self._fetch]

    def run(self, inputs=None):
        if inputs is not None:
            from ..core.tensor import Tensor as PT
            for n, x in zip(self._feeds, inputs):
                t = x._t if isinstance(x, PT) else x
                if isinstance(t, torch.Tensor) and t.device == self._dev:
                    self.get_input_handle(n).share_external_data(t)  # already resident: no round trip
                else:
                    self.get_input_handle(n).copy_from_cpu(x.numpy() if hasattr(x, 'numpy') else x)
        feeds = {n: self._inputs[n] for n in self._feeds}
        if self._config._hip_graph and self._dev.type == 'cuda':
            if self._graph is None:
                from ..device.cuda.graphs import _Graphed
                self._graph = _Graphed(lambda *xs: self._run_once(dict(zip(self._feeds, xs))), warmup=1)
            with torch.no_grad():
                outs = self._graph(*[feeds[n] for n in self._feeds])
        else:
            outs = self._run_once(feeds)
        self._outputs = dict(zip(self._out_names, outs))
        if inputs is not None:
            from ..core.tensor import _wrap
            return [_wrap(o) for o in outs]
        return True

    def clone(self):
        return Predictor(self._config)

    def clear_intermediate_tensor(self):
        pass

    def try_shrink_memory(self):
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
        return 0


def create_predictor(config):
    return Predictor(config)


class PredictorPool:
    def __init__(self, config, size=1):
        self._preds = [Predictor(config) for _ in range(size)]

    def retrive(self, idx):
        return self._preds[idx]

    retrieve = retrive


def convert_to_mixed_precision(model_file, params_file, mixed_model_file, mixed_params_file, mixed_precision,
                               backend=None, keep_io_types=True, black_list=None, **kw):
    """Casts floating weights to fp16/bf16 and writes a new model pair."""
    import shutil
    from safetensors.torch import load_file, save_file
    dt = torch.bfloat16 if mixed_precision == PrecisionType.Bfloat16 else torch.float16
    shutil.copyfile(model_file, mixed_model_file)
    ts = load_file(params_file)
    save_file({k: (v.to(dt) if v.is_floating_point() else v) for k, v in ts.items()}, mixed_params_file)


def get_trt_compile_version():
    """TensorRT is an NVIDIA engine; this build has none: (0, 0, 0) (reference returns the
    version the library was compiled against)."""
    return (0, 0, 0)


def get_trt_runtime_version():
    return (0, 0, 0)


class XpuConfig:
    """Kunlun XPU predictor options (reference inference/wrapper.py); accepted and unused on MI355X."""

    def __init__(self):
        self.device_id = 0
        self.l3_size = 0
        self.l3_ptr = None
        self.l3_autotune_size = 0
        self.conv_autotune_level = 0
        self.fc_autotune_level = 0
        self.context_gm_size = 0
        self.transformer_softmax_optimize_level = 0
        self.transformer_encoder_adaptive_seqlen = True
        self.quant_post_static_gelu_out_threshold = 10.0
        self.quant_post_dynamic_activation_method = 0
        self.quant_post_dynamic_weight_precision = 1
        self.quant_post_dynamic_op_types = []


def _get_phi_kernel_name(fluid_op_name):
    """Operator name -> kernel name (the same string here: every op is its own kernel entry)."""
    return fluid_op_name
