"""RCCL ordering evidence on one GPU: GPT stage-3 sharding (grouped / deferred weight gradients on)
over a real 1-rank ``nccl`` process group with PADDLE_AMD_FORCE_COLLECTIVES=1, run under
``rocprofv3 --kernel-trace``; ``--report <kernel_trace.csv>`` then lists, for the last step, every
RCCL kernel with the hand-written weight-gradient kernels that precede it and the queue each ran on.

  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rccl -- python3 tools/rccl_order_trace.py
  python3 tools/rccl_order_trace.py --report gpurun_out/rccl/.../kernel_trace.csv
"""
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(steps=3):
    import socket
    import torch
    import torch.distributed as dist
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(s.getsockname()[1])
    s.close()
    os.environ['PADDLE_AMD_FORCE_COLLECTIVES'] = '1'
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda', 0))
    import paddle
    from paddle.models.gpt import gpt_config, GPTForPretraining
    paddle.seed(0)
    cfg = gpt_config('gpt-tiny', hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    model = GPTForPretraining(cfg)
    opt = paddle.optimizer.AdamW(learning_rate=1e-3, parameters=model.parameters(), multi_precision=True,
                                 grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
    model, opt = paddle.amp.decorate(model, opt, level='O2', dtype='bfloat16')
    model, opt, _ = paddle.distributed.sharding.group_sharded_parallel(model, opt, level='p_g_os')
    assert opt.engine.collectives
    inner = model._layers if hasattr(model, '_layers') else model
    ids = paddle.to_tensor(torch.randint(0, cfg.vocab_size, (4, 129), device='cuda'))
    x, y = ids[:, :-1], ids[:, 1:]
    for i in range(steps):
        torch.cuda.synchronize()
        # step marker kernel: a named fill the report splits steps on
        torch.full((1,), float(i), device='cuda')
        loss = inner.loss(model(x), y)
        loss.backward()
        opt.step()
        opt.clear_grad()
        print(f'step {i} loss {float(loss):.4f}', flush=True)
    torch.cuda.synchronize()
    dist.destroy_process_group()


def report(path):
    rows = list(csv.DictReader(open(path)))
    key = 'Kernel_Name' if 'Kernel_Name' in rows[0] else 'Kernel-Name'
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    is_rccl = lambda n: 'nccl' in n.lower() or 'rccl' in n.lower()  # noqa: E731
    is_wgrad = lambda n: ('pa::' in n or 'pa_' in n) and ('wgrad' in n or 'grouped' in n or 'gemm' in n)  # noqa: E731
    rccl_idx = [i for i, r in enumerate(rows) if is_rccl(r[key])]
    print(f'{len(rows)} kernels, {len(rccl_idx)} RCCL kernels')
    if not rccl_idx:
        return
    # the last third of the trace ~ the last step
    lo = rows[rccl_idx[len(rccl_idx) * 2 // 3]]
    t_lo = int(lo['Start_Timestamp'])
    q = lambda r: r.get('Queue_Id', r.get('Stream_Id', '?'))  # noqa: E731
    last_w = None
    for r in rows:
        if int(r['Start_Timestamp']) < t_lo - 2_000_000:
            continue
        n = r[key]
        if is_wgrad(n):
            last_w = r
        if is_rccl(n):
            prev = last_w[key][:70] if last_w else '-'
            gap = (int(r['Start_Timestamp']) - int(last_w['End_Timestamp'])) / 1e3 if last_w else float('nan')
            print(f'RCCL q{q(r):>3} {n[:60]:60s} | after {prev:70s} q{q(last_w) if last_w else "-":>3} '
                  f'(+{gap:.1f} us after its end)')


if __name__ == '__main__':
    if len(sys.argv) > 2 and sys.argv[1] == '--report':
        report(sys.argv[2])
    else:
        run()
