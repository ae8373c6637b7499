"""CPU checks of the captured-step host hooks (device/cuda/graphs.py on_replay): registration only
inside a TrainStepGraph capture, and the optimizers' host-LR fallback when nothing captures.
The replay behaviour itself is covered on the GPU (tests/test_hip_kernels.py
test_train_step_graph_lr_scheduler)."""
import paddle
from paddle.device.cuda import graphs


def test_on_replay_outside_capture_registers_nothing():
    calls = []
    assert graphs.on_replay(pre=lambda: calls.append('pre'), post=lambda: calls.append('post')) is False
    assert graphs._CAPTURE_HOOKS is None
    assert calls == []


def test_on_replay_collects_into_active_capture_list():
    saved = graphs._CAPTURE_HOOKS
    try:
        graphs._CAPTURE_HOOKS = []
        pre, post = (lambda: None), (lambda: None)
        assert graphs.on_replay(pre=pre, post=post) is True
        assert graphs._CAPTURE_HOOKS == [(pre, post)]
    finally:
        graphs._CAPTURE_HOOKS = saved


def test_train_step_graph_cpu_runs_eagerly_with_scheduler():
    paddle.seed(3)
    net = paddle.nn.Linear(8, 4)
    sched = paddle.optimizer.lr.StepDecay(learning_rate=0.1, step_size=1, gamma=0.5)
    opt = paddle.optimizer.AdamW(learning_rate=sched, parameters=net.parameters())
    x = paddle.randn([16, 8])

    def step():
        loss = net(x).square().mean()
        loss.backward()
        opt.step()
        opt.clear_grad()
        return loss
    run = graphs.capture_train_step(step, warmup=1)
    losses = []
    for _ in range(4):
        losses.append(float(run()))
        sched.step()
    assert run.graph is None and run.hooks == []  # no GPU: every call ran eagerly
    assert losses[-1] < losses[0]
    assert abs(opt.get_lr() - 0.1 * 0.5 ** 4) < 1e-12
