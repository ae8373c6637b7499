"""Where do device-to-device copies / fills come from in the GPT-3 1.3B step?  One profiled step
under torch.profiler; prints aten copy/fill ops grouped by the first frames inside our package."""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    import paddle
    import paddle.distributed as pdist
    from paddle.models.gpt import gpt_config, GPTForPretraining
    torch.cuda.set_device(0)
    paddle.seed(1234)
    cfg = gpt_config('gpt3-1.3b', hidden_dropout_prob=0.1, attention_probs_dropout_prob=0.0)
    model = GPTForPretraining(cfg)
    opt = paddle.optimizer.AdamW(learning_rate=1e-4, parameters=model.parameters(), weight_decay=0.01,
                                 multi_precision=True, grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
    model, opt = paddle.amp.decorate(model, opt, level='O2', dtype='bfloat16')
    model, opt, _ = pdist.sharding.group_sharded_parallel(model, opt, level='p_g_os')
    inner = model._layers if hasattr(model, '_layers') else model
    ids = torch.randint(0, cfg.vocab_size, (16, 1025), device='cuda')
    x, y = paddle.to_tensor(ids[:, :-1]), paddle.to_tensor(ids[:, 1:])

    def step():
        loss = inner.loss(model(x), y)
        loss.backward()
        opt.step()
        opt.clear_grad()

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU], record_shapes=True, with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    groups = collections.Counter()
    for ev in prof.events():
        if ev.name not in ('aten::copy_', 'aten::fill_', 'aten::zero_', 'aten::clone', 'aten::cat'):
            continue
        frames = [f for f in (ev.stack or []) if 'paddlepaddle-paddle_amd' in f or 'paddle_amd' in f][:3]
        shapes = str(ev.input_shapes)[:80] if ev.input_shapes else ''
        groups[(ev.name, ' <- '.join(f.split('/')[-1] for f in frames), shapes)] += 1
    for (name, where, shapes), c in groups.most_common(40):
        print(f"{c:4d}  {name:14s} {where}  {shapes}", flush=True)


if __name__ == '__main__':
    main()
