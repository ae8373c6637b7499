"""CPU-side contract of the HIP op wrappers: every entry point the models and tests use exists,
and the non-GPU fallbacks compute the same math (the kernels themselves: test_hip_kernels.py)."""
import torch

import paddle
from paddle import ops


def test_op_entry_points_exist():
    for mod, names in [(ops.gemm, ['hip_mm', 'hip_mm_ok', 'wgrad_accumulate', 'hip_fp8_ok', 'hip_fp8_mm',
                                   'fp8_quantize', 'fp8_gemm']),
                       (ops.conv, ['supported', 'conv2d_fwd', 'conv2d_nhwc', 'conv2d_dgrad', 'conv2d_dgrad_classes',
                                   'conv2d_wgrad', 'conv2d_wgrad_1x1']),
                       (ops.flash_attn, ['flash_attention', 'flash_attention_packed', 'supported'])]:
        for n in names:
            assert hasattr(mod, n), f"{mod.__name__}.{n} missing"


def test_fp8_gemm_cpu_matches_dequantised_matmul():
    torch.manual_seed(0)
    x = torch.randn(16, 64)
    y = torch.randn(64, 32)
    out = ops.gemm.fp8_gemm(paddle.to_tensor(x), paddle.to_tensor(y), output_dtype='float32')._t
    ref = x @ y
    rel = (out - ref).norm() / ref.norm()
    assert rel < 0.08, rel


def test_conv_hip_path_not_taken_on_cpu():
    x = torch.randn(1, 8, 8, 32, dtype=torch.bfloat16)
    w = torch.randn(64, 32, 3, 3, dtype=torch.bfloat16)
    assert not ops.conv.supported(x, w, 1)
    out = paddle.nn.functional.conv2d(paddle.to_tensor(x), paddle.to_tensor(w), padding=1, data_format='NHWC')
    assert out.shape == [1, 8, 8, 64]
