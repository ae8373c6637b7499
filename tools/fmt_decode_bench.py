"""FusedMultiTransformer decode step on one MI355X: Llama-2-13B-shaped layers (hidden 5120, 40
heads, ffn 13824 SwiGLU, RMSNorm), bf16, batch B new tokens over a cache of L positions, 2 layers
timed per token; skinny decode GEMM on vs off (ops.gemm._skinny).  Reports ms per layer-token."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import paddle  # noqa: E402
from paddle.incubate.nn import FusedMultiTransformer  # noqa: E402
from paddle.ops import gemm  # noqa: E402


def main():
    paddle.set_device('gpu:0')
    E, H, F_, nl = 5120, 40, 13824, 2
    D = E // H
    paddle.seed(0)
    m = FusedMultiTransformer(E, H, F_, num_layers=nl, norm_type='rmsnorm', activation='swiglu')
    m.eval()
    m.to(dtype='bfloat16')
    for B, L in ((1, 2048), (16, 2048), (64, 2048)):
        caches = [paddle.zeros([2, B, H, L + 8, D], dtype='bfloat16') for _ in range(nl)]
        x = paddle.randn([B, 1, E]).astype('bfloat16')
        ts = paddle.to_tensor([L])
        res = []
        for sk in (False, True):
            gemm._skinny = sk
            with paddle.no_grad():
                for _ in range(3):
                    m(x, caches=caches, time_step=ts)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    o, _c = m(x, caches=caches, time_step=ts)
                e1.record()
                torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1) / 20 / nl)
        # the same decode step replayed from one captured hipGraph (device time_step)
        from paddle.device.cuda.graphs import DecodeStepGraph
        with paddle.no_grad():
            gs = DecodeStepGraph(lambda xx, t: m(xx, caches=caches, time_step=t)[0], x._t, L - 40, warmup=1)
            for _ in range(3):
                gs(x)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(20):
                gs(x)
            e1.record()
            torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / 20 / nl)
        print(f"B {B:3d} L {L}: {res[0]:.3f} ms/layer (library GEMMs) -> {res[1]:.3f} ms/layer (skinny GEMMs)"
              f"  [{res[0] / res[1]:.2f}x]; decode step as one hipGraph: {res[2]:.3f} ms/layer")
    gemm._skinny = True


if __name__ == '__main__':
    main()
