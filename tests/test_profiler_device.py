"""paddle.profiler (native host tracer) and paddle.device APIs on CPU; GPU kernel capture."""
import glob
import json

import pytest

import paddle
import paddle.profiler as profiler


def test_scheduler_states():
    s = profiler.make_scheduler(closed=1, ready=1, record=2, repeat=1)
    st = [s(i) for i in range(6)]
    P = profiler.ProfilerState
    assert st == [P.CLOSED, P.READY, P.RECORD, P.RECORD_AND_RETURN, P.CLOSED, P.CLOSED]


def test_profiler_host_ranges_and_chrome_export(tmp_path):
    net = paddle.nn.Linear(8, 8)
    opt = paddle.optimizer.SGD(0.1, parameters=net.parameters())
    prof = profiler.Profiler(targets=[profiler.ProfilerTarget.CPU], scheduler=(1, 3),
                             on_trace_ready=profiler.export_chrome_tracing(str(tmp_path)))
    prof.start()
    for _ in range(4):
        with profiler.RecordEvent("fwd_bwd"):
            net(paddle.randn([4, 8])).sum().backward()
        opt.step()
        opt.clear_grad()
        prof.step()
    prof.stop()
    files = glob.glob(str(tmp_path / '*.json'))
    assert files
    trace = profiler.load_profiler_result(files[0])
    names = {e['name'] for e in trace['traceEvents']}
    assert 'fwd_bwd' in names and 'SGD.step' in names
    assert any(n.startswith('ProfileStep#') for n in names)
    res = prof.get_profiler_result()
    assert sum(1 for e in res.host if e['name'] == 'fwd_bwd') == 2  # steps 1 and 2 recorded
    text = prof.summary()
    assert 'fwd_bwd' in text


def test_timer_only_step_info():
    prof = profiler.Profiler(timer_only=True)
    prof.start()
    for _ in range(3):
        prof.step(num_samples=8)
    info = prof.step_info()
    prof.stop()
    assert 'ips' in info and 'samples/s' in info


def test_device_api_cpu():
    assert paddle.device.get_device() in ('cpu',) or paddle.device.get_device().startswith('gpu')
    assert 'cpu' in paddle.device.get_all_device_type()
    assert paddle.device.cuda.device_count() >= 0


@pytest.mark.gpu
def test_profiler_captures_hip_kernels(tmp_path):
    x = paddle.randn([256, 1024]).astype('bfloat16')
    ln = paddle.nn.LayerNorm(1024)
    ln.to(dtype='bfloat16')
    with profiler.Profiler(on_trace_ready=profiler.export_chrome_tracing(str(tmp_path))) as prof:
        for _ in range(2):
            y = ln(x)
            prof.step()
    res = prof.get_profiler_result()
    assert any('norm' in e['name'] for e in res.device), [e['name'] for e in res.device][:20]


@pytest.mark.gpu
def test_streams_events_graph():
    s = paddle.device.Stream()
    e1, e2 = paddle.device.Event(enable_timing=True), paddle.device.Event(enable_timing=True)
    x = paddle.randn([1024, 1024])
    with paddle.device.stream_guard(s):
        e1.record(s)
        y = x @ x
        e2.record(s)
    s.synchronize()
    assert e1.elapsed_time(e2) >= 0
    f = paddle.device.cuda.wrap_cuda_graph(lambda a: a * 2 + 1)
    for i in range(4):
        out = f(x)
    assert float((out - (x * 2 + 1)).abs().max()) == 0
    assert paddle.device.cuda.memory_allocated() > 0
    _ = y
