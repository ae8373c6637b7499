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


def run(steps=3, model_name='gpt-tiny', batch=4, seq=128):
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
    cfg = gpt_config(model_name, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0,
                     max_position_embeddings=max(seq, 1024))
    model = GPTForPretraining(cfg)
    opt = paddle.optimizer.AdamW(learning_rate=1e-3, parameters=model.parameters(), multi_precision=True,
                                 grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
    model, opt = paddle.amp.decorate(model, opt, level='O2', dtype='bfloat16')
    model, opt, _ = paddle.distributed.sharding.group_sharded_parallel(model, opt, level='p_g_os')
    assert opt.engine.collectives
    inner = model._layers if hasattr(model, '_layers') else model
    ids = paddle.to_tensor(torch.randint(0, cfg.vocab_size, (batch, seq + 1), device='cuda'))
    x, y = ids[:, :-1], ids[:, 1:]
    for i in range(steps):
        torch.cuda.synchronize()
        # step marker: a spin kernel the reports split steps on
        torch.cuda._sleep(1000)
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


def overlap(path):
    """The last step (after the last spin marker) of a rocprofv3 kernel trace: the compute queue is
    the one running the most kernels; every kernel on another queue is collective work (RCCL
    kernels, or — for a 1-rank group, where RCCL turns a reduce-scatter / all-gather into a device
    copy — its copies on the RCCL stream).  Prints those kernels by name and the share of their time
    that runs concurrently with compute-queue kernels."""
    from collections import Counter
    rows = list(csv.DictReader(open(path)))
    key = 'Kernel_Name' if 'Kernel_Name' in rows[0] else 'Kernel-Name'
    qk = 'Queue_Id' if 'Queue_Id' in rows[0] else ('Stream_Id' if 'Stream_Id' in rows[0] else None)
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    marks = [i for i, r in enumerate(rows) if 'spin' in r[key].lower() or 'sleep' in r[key].lower()]
    t0 = int(rows[marks[-1]]['End_Timestamp']) if marks else 0
    sel = [r for r in rows if int(r['Start_Timestamp']) >= t0]
    qs = Counter(r[qk] for r in sel) if qk else Counter()
    cq = qs.most_common(1)[0][0] if qs else None
    is_comm = lambda r: ('nccl' in r[key].lower() or 'rccl' in r[key].lower() or  # noqa: E731
                         (qk is not None and r[qk] != cq))
    comm = [(int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in sel if is_comm(r)]
    comp = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in sel if not is_comm(r))
    merged = []
    for a, b in comp:
        if merged and a <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], b)
        else:
            merged.append([a, b])
    tot = sum(b - a for a, b in comm)
    ov = 0
    for a, b in comm:
        for c, d in merged:
            if d <= a:
                continue
            if c >= b:
                break
            ov += min(b, d) - max(a, c)
    span = (max(b for _, b in comm + comp) - min(a for a, _ in comm + comp)) / 1e6 if comm else 0
    print(f"queues in the last step (kernels): {dict(qs)}; compute queue {cq}")
    names = Counter(r[key][:90] for r in sel if is_comm(r))
    for n, c in names.most_common(12):
        print(f"  collective-queue kernel x{c}: {n}")
    print(f"last step: {len(comm)} collective-queue kernels, {tot / 1e6:.3f} ms, {ov / 1e6:.3f} ms of it "
          f"({100.0 * ov / max(tot, 1):.1f} %) concurrent with compute-queue kernels; step span {span:.2f} ms")


if __name__ == '__main__':
    if len(sys.argv) > 2 and sys.argv[1] == '--report':
        report(sys.argv[2])
    elif len(sys.argv) > 2 and sys.argv[1] == '--overlap':
        overlap(sys.argv[2])
    elif len(sys.argv) > 1 and sys.argv[1] == '--gpt13':
        run(steps=3, model_name='gpt3-1.3b', batch=4, seq=1024)
    else:
        run()
