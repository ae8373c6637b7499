"""quant_aware / convert (reference python/paddle/static/quantization/quanter.py): QAT and freeze
of a static Program with a config dict."""
from .passes import (QuantizationTransformPass, QuantizationFreezePass, ConvertToInt8Pass, OutScaleForTrainingPass,
                     OutScaleForInferencePass, DEFAULT_TYPES)

_DEFAULT_CONFIG = {
    'weight_quantize_type': 'channel_wise_abs_max',
    'activation_quantize_type': 'moving_average_abs_max',
    'weight_bits': 8,
    'activation_bits': 8,
    'not_quant_pattern': ['skip_quant'],
    'quantize_op_types': list(DEFAULT_TYPES),
    'dtype': 'int8',
    'window_size': 10000,
    'moving_rate': 0.9,
    'for_tensorrt': False,
    'is_full_quantize': False,
    'onnx_format': True,
}


def _config(config):
    c = dict(_DEFAULT_CONFIG)
    c.update(config or {})
    return c


def quant_aware(program, place=None, config=None, scope=None, for_test=False, weight_quantize_func=None,
                act_quantize_func=None, weight_preprocess_func=None, act_preprocess_func=None, optimizer_func=None,
                executor=None, return_program=False, calib_config=None, model_type=None, pattern_ops=None, **kw):
    """Insert the QAT fake quant-dequant nodes (in place); returns the program."""
    c = _config(config)
    QuantizationTransformPass(weight_bits=c['weight_bits'], activation_bits=c['activation_bits'],
                              activation_quantize_type=c['activation_quantize_type'],
                              weight_quantize_type=c['weight_quantize_type'], moving_rate=c['moving_rate'],
                              quantizable_op_type=c['quantize_op_types']).apply(program)
    if not for_test:
        OutScaleForTrainingPass(moving_rate=c['moving_rate']).apply(program)
    return program


def convert(program, place=None, config=None, scope=None, save_int8=False, **kw):
    """Freeze a QAT program into the int8 inference program (in place); returns it (and the same
    program again when ``save_int8``, whose GEMM weights are already int8)."""
    c = _config(config)
    OutScaleForInferencePass().apply(program)
    QuantizationFreezePass(weight_bits=c['weight_bits'], activation_bits=c['activation_bits'],
                           weight_quantize_type=c['weight_quantize_type']).apply(program)
    if save_int8:
        ConvertToInt8Pass().apply(program)
        return program, program
    return program
