"""Static int8 inference on the GPU: a PTQ-quantised model saved in the onnx-format ProgramDesc
(quantize_linear / dequantize_linear + int8 weights) and reloaded by the Predictor runs its GEMMs on
the int8 MFMA kernel (quant_linear_fuse_pass -> pa_gemm8_i8) within quantisation error of fp32."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import paddle  # noqa: E402
from paddle import static  # noqa: E402
from paddle.static import quantization as Q, ir_passes as IP  # noqa: E402
from paddle.ops import int8 as I8  # noqa: E402


def test_ptq_int8_predictor_gpu(tmp_path):
    paddle.set_device('cpu')
    paddle.seed(3)
    paddle.enable_static()
    try:
        main, startup = static.Program(), static.Program()
        with static.program_guard(main, startup):
            x = static.data('x', [None, 256], 'float32')
            h = static.nn.fc(x, 512, activation='relu')
            y = static.nn.fc(h, 256)
        exe = static.Executor(paddle.CPUPlace())
        prefix = os.path.join(str(tmp_path), 'fp32', 'mlp')
        static.save_inference_model(prefix, [x], [y], exe, program=main)
        rng = np.random.RandomState(0)

        def gen():
            for _ in range(64):
                yield (rng.randn(256).astype('float32'),)
        ptq = Q.PostTrainingQuantization(exe, os.path.dirname(prefix), sample_generator=gen, batch_size=16,
                                         batch_nums=4, algo='abs_max')
        ptq.quantize()
        saved = ptq.save_quantized_model(os.path.join(str(tmp_path), 'int8') + os.sep)
        xs = np.random.RandomState(9).randn(40, 256).astype('float32')
        ref = exe.run(main, feed={'x': xs}, fetch_list=[y])[0]
    finally:
        paddle.disable_static()
    from paddle import inference as I
    cfg = I.Config(saved + '.pdmodel', saved + '.pdiparams')
    cfg.enable_use_gpu(256, 0)
    pred = I.create_predictor(cfg)
    calls = []
    orig = I8.i8_mm
    I8.i8_mm = lambda *a, **k: (calls.append(1), orig(*a, **k))[1]
    try:
        out = pred.run([paddle.to_tensor(xs)])[0].numpy()
    finally:
        I8.i8_mm = orig
    assert IP.fusion_stats(pred._program).get('quant_linear_fuse_pass') == 2
    assert len(calls) == 2, 'int8 MFMA GEMM did not run'
    assert np.abs(out - ref).max() / np.abs(ref).max() < 0.03
