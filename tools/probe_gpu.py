"""One-off hardware probe: library GEMM / SDPA / conv throughput on the box (baseline for our kernels)."""
import time, json, torch, torch.nn.functional as F
d = torch.device('cuda:0')
p = torch.cuda.get_device_properties(0)
out = {"name": p.name, "cus": p.multi_processor_count, "mem_gb": p.total_memory / 2**30, "arch": getattr(p, 'gcnArchName', '')}
def bench(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(it): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / it
for n in (2048, 4096, 8192):
    a = torch.randn(n, n, device=d, dtype=torch.bfloat16); b = torch.randn(n, n, device=d, dtype=torch.bfloat16)
    t = bench(lambda: a @ b); out[f"mm_bf16_{n}_TF"] = 2 * n**3 / t / 1e12
# GPT-1.3B shapes: tokens=8192, h=2048
x = torch.randn(8192, 2048, device=d, dtype=torch.bfloat16)
for (k, nn_) in ((2048, 6144), (2048, 8192), (8192, 2048), (2048, 2048)):
    w = torch.randn(nn_, k, device=d, dtype=torch.bfloat16); xx = torch.randn(8192, k, device=d, dtype=torch.bfloat16)
    t = bench(lambda: F.linear(xx, w)); out[f"linear_8192x{k}x{nn_}_TF"] = 2 * 8192 * k * nn_ / t / 1e12
q = torch.randn(8, 16, 1024, 128, device=d, dtype=torch.bfloat16, requires_grad=True)
k_ = torch.randn_like(q, requires_grad=True); v = torch.randn_like(q, requires_grad=True)
t = bench(lambda: F.scaled_dot_product_attention(q, k_, v, is_causal=True))
out["sdpa_fwd_causal_TF"] = 4 * 8 * 16 * 1024 * 1024 * 128 / 2 / t / 1e12
def fb():
    o = F.scaled_dot_product_attention(q, k_, v, is_causal=True); o.sum().backward()
t = bench(fb); out["sdpa_fwdbwd_causal_ms"] = t * 1e3
xc = torch.randn(256, 64, 56, 56, device=d, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
wc = torch.randn(64, 64, 3, 3, device=d, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
t = bench(lambda: F.conv2d(xc, wc, padding=1)); out["conv3x3_64_56_nhwc_TF"] = 2 * 256 * 64 * 56 * 56 * 64 * 9 / t / 1e12
xc2 = xc.contiguous(); wc2 = wc.contiguous()
t = bench(lambda: F.conv2d(xc2, wc2, padding=1)); out["conv3x3_64_56_nchw_TF"] = 2 * 256 * 64 * 56 * 56 * 64 * 9 / t / 1e12
y = torch.randn(64 * 1024 * 1024, device=d)
t = bench(lambda: y * 2.0); out["copy_scale_TBps"] = 2 * y.numel() * 4 / t / 1e12
print(json.dumps(out, indent=1))
