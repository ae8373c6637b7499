"""Headline benchmark: GPT-3 1.3B bf16 pretraining with group-sharded stage-3 (p_g_os), tokens/s.

BASELINE.json metric: "samples/sec ResNet50 bf16 + tokens/sec GPT-3 1.3B sharding-3, at 1/2/4/8 MI355X".
Default (`--model gpt3-1.3b`) reports the GPT-3 1.3B tokens/s as ``value`` and then times ResNet50
(bf16 O2, NHWC, batch 256 per GPU, Momentum, data parallel) in the same run with the same K/W,
reported under the extra key ``resnet50`` (``--no-resnet`` skips it); `--model resnet50` reports
ResNet50 alone as ``value``.

Extra keys for the other BASELINE configs (``--no-extra`` skips them; a failure is reported in the
key, never replaces the headline line):
* ``llama2_13b`` — config 4 (Llama-2 13B, TP2 x PP2 x sharding-2 on 8 GPUs) on ONE GPU: bf16
  training tok/s of a Llama-2-13B-shaped decoder stack at full width (hidden 5120, 40 heads of 128,
  SwiGLU 13824, vocab 32000, seq 4096) holding this GPU's share of the 8-way model — 10 of the 40
  layers (PP2 halves the depth, TP2 halves the width: 40 / 2 / 2) — sharding-2 engine (os_g),
  AdamW with fp32 masters; every GEMM / RMSNorm / RoPE / flash-attention / SwiGLU on the HIP
  kernels.  Per-GPU work equals the 8-GPU config's; it is not the full 13B model.
* ``ernie_fp8`` — config 5: ERNIE-3.0-base (12 x 768) sequence classification as a static Program
  run by the Executor with static.amp AMP-O2, fp8 Linears (e4m3 fwd / e5m2 grads, delayed scaling,
  8-phase fp8 MFMA GEMM) vs the same program in bf16; tokens/s of each.

Single node, one process per GPU (torch.distributed.run sets RANK/LOCAL_RANK/WORLD_SIZE);
collectives are RCCL over xGMI.  Synthetic data of the real shapes, random-init weights.
W untimed warmup steps, then K timed steps bracketed by barrier + device sync; the
reported step time is the MAX over ranks; rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--model', default='gpt3-1.3b')
    ap.add_argument('--micro-batch', type=int, default=16)
    ap.add_argument('--seq', type=int, default=1024)
    ap.add_argument('--sharding', default='p_g_os', choices=['os', 'os_g', 'p_g_os', 'dp'])
    ap.add_argument('--dropout', type=float, default=0.1)
    ap.add_argument('--attn-dropout', type=float, default=0.1,
                    help='attention-probability dropout (in-kernel in csrc/flash_attn.hip)')
    ap.add_argument('--resnet-batch', type=int, default=256)
    ap.add_argument('--no-resnet', action='store_true')
    ap.add_argument('--no-extra', action='store_true', help='skip the llama2_13b / ernie_fp8 extra keys')
    ap.add_argument('--llama-layers', type=int, default=10)
    ap.add_argument('--llama-seq', type=int, default=4096)
    ap.add_argument('--llama-batch', type=int, default=2)
    ap.add_argument('--ernie-batch', type=int, default=64)
    ap.add_argument('--ernie-seq', type=int, default=512)
    ap.add_argument('--cpu', action='store_true',
                    help='rehearsal only (tests): run the same bench path on the CPU with gloo, e.g. with '
                         '--model gpt-tiny --resnet-model resnet18; the numbers mean nothing')
    ap.add_argument('--resnet-model', default='resnet50', help=argparse.SUPPRESS)
    ap.add_argument('--graph', action='store_true',
                    help='replay the whole training step as one captured hipGraph (dropout re-randomised per '
                         'replay by a device generation counter; device/cuda/graphs.py TrainStepGraph)')
    return ap.parse_args()


def _pool_len(args):
    """Distinct pre-generated batches: one per warmup + timed step (cycled past 32)."""
    return max(1, min(args.steps + args.warmup, 32))


def _feeder(dsts, pool):
    """feed(): copy the next pre-generated batch of ``pool`` into the step's input tensors ``dsts``
    (a device-to-device copy inside the timed step, so a captured hipGraph replays with new data
    too): every step trains on different samples, and the logged losses mean something."""
    it = [0]

    def feed():
        src = pool[it[0] % len(pool)]
        it[0] += 1
        for d, s_ in zip(dsts[0], src):
            d.copy_(s_)
    return feed


class _Step:
    """A bench step: ``feed()`` copies the next pre-generated batch into the input tensors, ``core()``
    runs forward / backward / optimizer on them; calling the step runs both.  ``--graph`` captures
    only ``core`` (the feed stays outside the graph, so every replay trains on new data)."""

    def __init__(self, feed, core):
        self.feed, self.core = feed, core

    def __call__(self):
        self.feed()
        return self.core()


def build_gpt(args, world, rank, dev):
    import torch
    import paddle
    import paddle.distributed as pdist
    from paddle.models.gpt import gpt_config, GPTForPretraining
    cfg = gpt_config(args.model, max_position_embeddings=max(args.seq, 1024), hidden_dropout_prob=args.dropout,
                     attention_probs_dropout_prob=args.attn_dropout)
    paddle.seed(1234)  # identical init on every rank
    model = GPTForPretraining(cfg)
    opt = paddle.optimizer.AdamW(learning_rate=1e-4, parameters=model.parameters(), weight_decay=0.01,
                                 beta1=0.9, beta2=0.95, epsilon=1e-8, multi_precision=True,
                                 grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
    model, opt = paddle.amp.decorate(model, opt, level='O2', dtype='bfloat16')
    if args.sharding == 'dp':
        if world > 1:
            model = pdist.DataParallel(model)
    else:  # same sharded engine at every N (degenerate single shard at N=1)
        model, opt, _ = pdist.sharding.group_sharded_parallel(model, opt, level=args.sharding)
    B, S = args.micro_batch, args.seq
    g = torch.Generator(device=dev).manual_seed(rank)
    pool = [torch.randint(0, cfg.vocab_size, (B, S + 1), device=dev, generator=g) for _ in range(_pool_len(args))]
    x, y = paddle.to_tensor(pool[0][:, :-1].contiguous()), paddle.to_tensor(pool[0][:, 1:].contiguous())
    feed = _feeder([(x._t, y._t)], [(p[:, :-1], p[:, 1:]) for p in pool])
    inner = model._layers if hasattr(model, '_layers') else model

    def core():
        logits = model(x)
        loss = inner.loss(logits, y)
        loss.backward()
        opt.step()
        opt.clear_grad()
        return loss
    step = _Step(feed, core)

    mcfg = {'model': args.model, 'global_batch': B * world, 'micro_batch_per_gpu': B, 'seq_len': S,
            'parallelism': (f"sharding-{ {'os': 1, 'os_g': 2, 'p_g_os': 3}.get(args.sharding, 0)}x{world}"
                            if args.sharding != 'dp' else f"dp{world}"),
            'hidden_dropout': args.dropout, 'attention_dropout': args.attn_dropout, 'optimizer': 'AdamW (fused, fp32 master)',
            'vocab': cfg.vocab_size}
    return step, B * S * world, 'tokens/sec GPT-3 1.3B sharding-3', 'tokens/s', mcfg


def build_resnet(args, world, rank, dev):
    import torch
    import paddle
    import paddle.distributed as pdist
    from paddle.vision.models import resnet50
    paddle.seed(1234)
    B = args.resnet_batch
    from paddle.vision import models as _vm
    model = resnet50(data_format='NHWC') if args.resnet_model == 'resnet50' else \
        getattr(_vm, args.resnet_model)(data_format='NHWC')
    opt = paddle.optimizer.Momentum(learning_rate=0.1, momentum=0.9, parameters=model.parameters(),
                                    weight_decay=1e-4, multi_precision=True)
    model, opt = paddle.amp.decorate(model, opt, level='O2', dtype='bfloat16')
    if world > 1:
        model = pdist.DataParallel(model)
    g = torch.Generator(device=dev).manual_seed(rank)
    res = 224 if args.resnet_model == 'resnet50' else 32
    pool = [(torch.randn(B, res, res, 3, device=dev, dtype=torch.bfloat16, generator=g),
             torch.randint(0, 1000, (B,), device=dev, generator=g)) for _ in range(_pool_len(args))]
    img, lab = paddle.to_tensor(pool[0][0].clone()), paddle.to_tensor(pool[0][1].clone())
    feed = _feeder([(img._t, lab._t)], pool)

    def core():
        out = model(img)
        loss = paddle.nn.functional.cross_entropy(out, lab)
        loss.backward()
        opt.step()
        opt.clear_grad()
        return loss
    step = _Step(feed, core)

    mcfg = {'model': args.resnet_model, 'global_batch': B * world, 'image': f'{res}x{res} NHWC', 'parallelism': f"dp{world}",
            'optimizer': 'Momentum'}
    return step, B * world, 'samples/sec ResNet50 bf16', 'samples/s', mcfg


def build_llama(args, world, rank, dev):
    """BASELINE config 4 on one GPU: this GPU's share (args.llama_layers full-width layers) of
    Llama-2 13B under TP2 x PP2 x sharding-2."""
    import torch
    import paddle
    import paddle.distributed as pdist
    from paddle.models.llama import llama_config, LlamaForCausalLM
    cfg = llama_config('llama2-13b', num_hidden_layers=args.llama_layers,
                       max_position_embeddings=max(args.llama_seq, 4096))
    paddle.seed(1234)
    model = LlamaForCausalLM(cfg)
    opt = paddle.optimizer.AdamW(learning_rate=1e-4, parameters=model.parameters(), weight_decay=0.01,
                                 beta1=0.9, beta2=0.95, epsilon=1e-8, multi_precision=True,
                                 grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
    model, opt = paddle.amp.decorate(model, opt, level='O2', dtype='bfloat16')
    model, opt, _ = pdist.sharding.group_sharded_parallel(model, opt, level='os_g')
    B, S = args.llama_batch, args.llama_seq
    g = torch.Generator(device=dev).manual_seed(rank)
    pool = [torch.randint(0, cfg.vocab_size, (B, S + 1), device=dev, generator=g) for _ in range(_pool_len(args))]
    x, y = paddle.to_tensor(pool[0][:, :-1].contiguous()), paddle.to_tensor(pool[0][:, 1:].contiguous())
    feed = _feeder([(x._t, y._t)], [(p[:, :-1], p[:, 1:]) for p in pool])
    inner = model._layers if hasattr(model, '_layers') else model

    def core():
        loss = inner.loss(model(x), y)
        loss.backward()
        opt.step()
        opt.clear_grad()
        return loss
    step = _Step(feed, core)
    nparam = sum(p._t.numel() for p in inner.parameters())
    mcfg = {'model': 'llama2-13b (per-GPU share of TP2xPP2xsharding2)', 'layers': args.llama_layers,
            'of_layers': 40, 'hidden': 5120, 'heads': 40, 'ffn': 13824, 'vocab': cfg.vocab_size,
            'seq_len': S, 'micro_batch_per_gpu': B, 'params_on_gpu': nparam, 'parallelism': f'sharding-2x{world}',
            'optimizer': 'AdamW (fused, fp32 master)'}
    return step, B * S * world, 'tokens/sec Llama-2 13B layer stack', 'tokens/s', mcfg


def build_ernie_static(args, world, rank, dev, fp8):
    """BASELINE config 5: ERNIE-3.0 static Program + Executor + AMP-O2 (fp8 Linears or bf16)."""
    import numpy as np
    import paddle
    from paddle import static
    from paddle.models import ernie_config, ErnieForSequenceClassification
    paddle.enable_static()
    try:
        paddle.seed(1234)
        cfg = ernie_config('ernie-3.0-base', hidden_dropout_prob=0.1, attention_probs_dropout_prob=0.1)
        B, S = args.ernie_batch, args.ernie_seq
        main, startup = static.Program(), static.Program()
        with static.program_guard(main, startup):
            ids = static.data('ids', [None, S], 'int64')
            lab = static.data('lab', [None], 'int64')
            model = ErnieForSequenceClassification(cfg, num_classes=2)
            loss = paddle.nn.functional.cross_entropy(model(ids), lab)
            opt = paddle.optimizer.AdamW(learning_rate=1e-4, parameters=model.parameters())
            if fp8:
                opt = static.amp.decorate(opt, level='O2', use_fp8=True,
                                          fp8_recipe=paddle.amp.DelayedScaling(amax_history_len=16))
            else:
                opt = static.amp.decorate(opt, level='O2', dtype='bfloat16')
            opt.minimize(loss)
        place = paddle.CUDAPlace(dev.index or 0) if dev.type == 'cuda' else paddle.CPUPlace()
        exe = static.Executor(place)
        exe.run(startup)
        opt.amp_init(place)
    finally:
        paddle.disable_static()
    rng = np.random.RandomState(rank)
    # a different pre-generated batch every step, already on the device; the loss is fetched every
    # step as a device tensor (return_numpy=False): the host does not wait for the device inside the
    # loop (as the dygraph benches); measure() reads it after the timing
    pool = [(paddle.to_tensor(rng.randint(1, cfg.vocab_size, size=(B, S)).astype('int64'), place=place)._t,
             paddle.to_tensor(rng.randint(0, 2, size=(B,)).astype('int64'), place=place)._t)
            for _ in range(_pool_len(args))]
    fed = {'ids': paddle.to_tensor(pool[0][0].clone()), 'lab': paddle.to_tensor(pool[0][1].clone())}
    feed = _feeder([(fed['ids']._t, fed['lab']._t)], pool)

    def core():
        paddle.enable_static()
        try:
            return exe.run(main, feed=fed, fetch_list=[loss], return_numpy=False)[0]
        finally:
            paddle.disable_static()
    step = _Step(feed, core)
    mcfg = {'model': 'ernie-3.0-base seq-cls', 'batch': B, 'seq_len': S,
            'mode': 'static Program + Executor, static.amp O2 ' + ('fp8 (e4m3/e5m2, delayed scaling)' if fp8 else 'bf16')}
    return step, B * S * world, 'tokens/sec ERNIE-3.0 static AMP-O2', 'tokens/s', mcfg


def _extra(args, world, rank, dev, out):
    """The llama2_13b / ernie_fp8 keys; each in isolation (state released after it)."""
    import gc
    import torch

    def run(key, builder):
        try:
            st, work, metric, unit, cfg = builder()
            ms, lossv = measure(st, args.steps, args.warmup, world, rank, dev, key)
            return {"metric": metric, "value": round(work / (ms / 1e3), 2), "unit": unit, "ms_per_step": round(ms, 3),
                    "config": cfg, "final_loss": round(lossv, 4)}
        except Exception as e:  # noqa: BLE001 — reported in the key, never replaces the headline
            return {"error": f"{type(e).__name__}: {str(e)[:300]}"}
        finally:
            gc.collect()
            if dev.type == 'cuda':
                torch.cuda.empty_cache()
    out["llama2_13b"] = run('llama2_13b', lambda: build_llama(args, world, rank, dev))
    e8 = run('ernie_fp8', lambda: build_ernie_static(args, world, rank, dev, True))
    eb = run('ernie_bf16', lambda: build_ernie_static(args, world, rank, dev, False))
    if 'value' in e8 and 'value' in eb:
        e8['bf16_value'] = eb['value']
        e8['bf16_ms_per_step'] = eb['ms_per_step']
        e8['fp8_speedup_vs_bf16'] = round(e8['value'] / eb['value'], 3)
    elif 'value' in eb:
        e8['bf16_value'] = eb['value']
    out["ernie_fp8"] = e8


def _maybe_graph(args, step, cfg):
    """--graph: the step as one captured hipGraph, captured inside the untimed warmup."""
    if not args.graph or args.warmup < 2:
        return step
    from paddle.device.cuda.graphs import capture_train_step
    cfg['hip_graph'] = True
    return _Step(step.feed, capture_train_step(step.core, warmup=args.warmup - 1))


def measure(step, steps, warmup, world, rank, dev, tag):
    """W untimed warmup steps, then K timed steps bracketed by barrier + device sync; MAX over ranks."""
    import torch
    import torch.distributed as dist
    if dev.type != 'cuda':  # --cpu rehearsal
        torch.cuda.synchronize = lambda *a, **k: None
    loss = None
    for i in range(warmup):
        loss = step()
        if rank == 0:  # progress on stderr; stdout carries only the JSON line
            torch.cuda.synchronize()
            print(f"[{tag}] warmup step {i} loss {float(loss.item()):.4f}", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    if world > 1:
        tt = torch.tensor([ms], device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        ms = float(tt.item())
    return ms, float(loss.item())


def _self_launch(args):
    """``--gpus N`` (N > 1) without a launcher: start the N rank processes here, one per GPU, over
    ``torch.distributed.run`` on 127.0.0.1, and exit with its status.  The parent never touches the
    GPU (no HIP call before the children exist); the ranks print the one JSON line."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')  # dmabuf IPC for RCCL (the host driver's only mode)
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={args.gpus}',
           '--master-addr=127.0.0.1', f'--master-port={port}', os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(_self_launch(args))
    import torch
    import torch.distributed as dist
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)")
    if args.cpu:
        return _main_cpu(args, world, rank)
    # one rank per GPU; the modulo only matters when rehearsing several ranks on fewer GPUs
    local_rank = int(os.environ.get('LOCAL_RANK', '0')) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank)
    if world > 1:
        # RCCL over xGMI; PADDLE_AMD_BENCH_BACKEND=gloo only to rehearse several ranks on one GPU
        # (RCCL refuses two ranks on one device)
        be = os.environ.get('PADDLE_AMD_BENCH_BACKEND', 'nccl')
        dist.init_process_group(be, **({'device_id': torch.device('cuda', local_rank)} if be == 'nccl' else {}))
    import paddle
    paddle.seed(1234 + rank)
    dev = torch.device('cuda', local_rank)
    _run(args, world, rank, dev)


def _main_cpu(args, world, rank):
    """--cpu: the identical bench flow on the CPU over gloo (multi-rank rehearsal in tests)."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group('gloo')
    import paddle
    paddle.set_device('cpu')
    paddle.seed(1234 + rank)
    _run(args, world, rank, torch.device('cpu'))


def _run(args, world, rank, dev):
    import gc
    import torch
    import torch.distributed as dist

    build = build_gpt if args.model.startswith('gpt') else build_resnet
    step, work, metric, unit, mcfg = build(args, world, rank, dev)
    step = _maybe_graph(args, step, mcfg)
    ms, final_loss = measure(step, args.steps, args.warmup, world, rank, dev, args.model)
    value = work / (ms / 1e3)
    out = {"metric": metric, "value": round(value, 2), "unit": unit, "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "bf16",
           "data": "synthetic (random token ids / random images), random-init weights",
           "config": mcfg, "final_loss": round(final_loss, 4),
           "world_size": dist.get_world_size() if dist.is_initialized() else 1,
           "backend": (("nccl (RCCL over xGMI)" if dist.get_backend() == 'nccl' else dist.get_backend())
                       if dist.is_initialized() else "none (1 rank)")}
    assert out["world_size"] == world == args.gpus, (out["world_size"], world, args.gpus)
    if args.model.startswith('gpt') and not args.no_resnet:
        # the second half of the BASELINE metric, same process, same K/W, GPT state released first
        del step
        gc.collect()
        torch.cuda.empty_cache()
        rstep, rwork, _, runit, rcfg = build_resnet(args, world, rank, dev)
        rstep = _maybe_graph(args, rstep, rcfg)
        rms, rloss = measure(rstep, args.steps, args.warmup, world, rank, dev, 'resnet50')
        out["resnet50"] = {"metric": "samples/sec ResNet50 bf16", "value": round(rwork / (rms / 1e3), 2),
                           "unit": runit, "ms_per_step": round(rms, 3), "config": rcfg, "final_loss": round(rloss, 4)}
    if args.model.startswith('gpt') and not args.no_extra and world == 1:
        # single-GPU evidence for BASELINE configs 4 and 5 (the multi-GPU scaling run times GPT /
        # ResNet only: the llama stack is one GPU's share of an 8-GPU hybrid layout)
        step = rstep = None  # noqa: F841 — release the earlier models' state
        gc.collect()
        if dev.type == 'cuda':
            torch.cuda.empty_cache()
        _extra(args, world, rank, dev, out)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
