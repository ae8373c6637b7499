"""paddle.matmul family on the hand-written GEMM (ops/matmul.py) vs the library (torch), random
operands, same process (A/B interleaved): fp16 / bf16 2-D GPT-3 1.3B shapes, batched attention-
shaped bmm (broadcast and strided), einsum, no_grad Linear."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def bench(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3 / n


def main():
    import paddle  # noqa: F401
    from paddle.ops import matmul as hm, _native
    assert _native._load() is not None
    dev = 'cuda'

    def r(*s, dt):
        return (torch.rand(*s, device=dev) * 2 - 1).to(dt)
    cases = []
    for dt in (torch.float16, torch.bfloat16):
        for nm, M, K, N in [('qkv', 16384, 2048, 6144), ('fc1', 16384, 2048, 8192), ('fc2', 16384, 8192, 2048)]:
            a, b = r(M, K, dt=dt), r(K, N, dt=dt)
            cases.append((f'{nm} {str(dt)[6:]} [{M}x{K}]@[{K}x{N}]', 2.0 * M * K * N, lambda a=a, b=b: hm.matmul(a, b),
                          lambda a=a, b=b: torch.matmul(a, b)))
        q, k = r(16, 16, 1024, 128, dt=dt), r(16, 16, 1024, 128, dt=dt)
        cases.append((f'QK^T {str(dt)[6:]} [16,16,1024,128]', 2.0 * 256 * 1024 * 1024 * 128,
                      lambda q=q, k=k: hm.matmul(q, k.transpose(-1, -2)),
                      lambda q=q, k=k: torch.matmul(q, k.transpose(-1, -2))))
        p, v = r(16, 16, 1024, 1024, dt=dt), r(16, 16, 1024, 128, dt=dt)
        cases.append((f'PV {str(dt)[6:]} [16,16,1024,1024]@[..,128]', 2.0 * 256 * 1024 * 1024 * 128,
                      lambda p=p, v=v: hm.matmul(p, v), lambda p=p, v=v: torch.matmul(p, v)))
        x, w = r(8, 2048, 1024, dt=dt), r(1024, 4096, dt=dt)
        cases.append((f'einsum bsh,hd {str(dt)[6:]}', 2.0 * 8 * 2048 * 1024 * 4096,
                      lambda x=x, w=w: hm.einsum('bsh,hd->bsd', x, w), lambda x=x, w=w: torch.einsum('bsh,hd->bsd', x, w)))
    if os.environ.get('PADDLE_AMD_GEMM_AUTOTUNE', '1') != '0':
        hm._TUNE['on'] = True  # routed paddle.matmul: per-shape choice of kernel vs library
    with torch.no_grad():
        for name, fl, fh, ft in cases:
            before = set(hm.tuned_choices())
            fh()
            picks = [v for k, v in hm.tuned_choices().items() if k not in before]
            th, tt = bench(fh), bench(ft)
            th2 = bench(fh)
            th = min(th, th2)
            print(f"{name:44s} paddle {th*1e6:9.1f} us {fl/th/1e12:6.0f} TF | library {tt*1e6:9.1f} us "
                  f"{fl/tt/1e12:6.0f} TF | {tt/th:4.2f}x  autotune: {','.join(picks) or 'hip'}", flush=True)


if __name__ == '__main__':
    main()
