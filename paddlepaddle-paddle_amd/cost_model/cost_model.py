"""Operator cost model of static programs.

Reference: python/paddle/cost_model/cost_model.py (CostModel: build_program, profile_measure via
the C++ profiler, static_cost_data / get_static_op_time over a bundled op-benchmark table).

Here ``profile_measure`` replays the program in the Executor with every recorded node timed
(device-synchronised per node: static/executor.py ``_PROFILE``), and the static table
``static_op_benchmark.json`` next to this file holds forward / backward times of common ops
measured on MI355X by ``tools/op_benchmark.py`` (same record keys as the reference's table:
op, config, paddle_gpu_time, paddle_gpu_time_backward — milliseconds).
"""
import json
import os

import numpy as np


class CostData:
    """Per-node and whole-program times of one profiled run (milliseconds)."""

    def __init__(self, records):
        self._records = list(records)

    def get_whole_time_ms(self):
        return float(sum(r[2] for r in self._records))

    def get_op_time_ms(self, op_id):
        return float(self._records[op_id][2])

    def get_op_name(self, op_id):
        return self._records[op_id][1]

    def op_times(self):
        """{op name: total ms} over the run."""
        out = {}
        for _, name, ms in self._records:
            out[name] = out.get(name, 0.0) + ms
        return out

    def __len__(self):
        return len(self._records)


class CostModel:
    def __init__(self):
        self._static_cost_data = None

    def build_program(self):
        import paddle
        from paddle import static
        paddle.enable_static()
        main_program, startup_program = static.Program(), static.Program()
        with static.program_guard(main_program=main_program, startup_program=startup_program):
            data = static.data(name='X', shape=[None, 1], dtype='float32')
            hidden = static.nn.fc(data, 10)
            loss = paddle.mean(hidden)
            paddle.optimizer.SGD(learning_rate=0.01).minimize(loss)
        return startup_program, main_program

    def profile_measure(self, startup_program, main_program, device='gpu', fetch_cost_list=('time',), feed=None):
        """Run ``main_program`` once with every node timed; returns a CostData.  ``feed``
        defaults to random data of each fed variable's shape (dynamic dims = 10)."""
        import paddle
        from ..static import executor as ex
        place = paddle.set_device('gpu' if device == 'gpu' and paddle.is_compiled_with_cuda() else 'cpu')
        exe = paddle.static.Executor(place)
        exe.run(startup_program)
        if feed is None:
            feed = {}
            for name, (_, shape, dt) in main_program.feeds.items():
                shp = [10 if s == -1 else s for s in shape]
                feed[name] = np.random.random(shp).astype(str(dt).replace('torch.', '').replace('paddle.', ''))
        exe.run(main_program, feed=feed, fetch_list=[])  # warm
        rec = []
        ex._PROFILE['rec'] = rec
        try:
            exe.run(main_program, feed=feed, fetch_list=[])
        finally:
            ex._PROFILE['rec'] = None
        return CostData(rec)

    def static_cost_data(self):
        path = os.path.join(os.path.dirname(__file__), 'static_op_benchmark.json')
        with open(path) as f:
            self._static_cost_data = json.load(f)
        return self._static_cost_data

    def get_static_op_time(self, op_name, forward=True, dtype='float32'):
        if op_name is None:
            raise ValueError('op_name should not be empty when you want to get static op time')
        if self._static_cost_data is None:
            self.static_cost_data()
        op_cost = {}
        for rec in self._static_cost_data:
            if rec['op'] == op_name and dtype in rec['config']:
                op_cost['op_time'] = rec['paddle_gpu_time'] if forward else rec['paddle_gpu_time_backward']
                op_cost['config'] = rec['config']
        return op_cost
