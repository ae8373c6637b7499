"""Step timer / throughput (reference: python/paddle/profiler/timer.py Benchmark:349 —
reader_cost, batch_cost, ips averaged over the logging window)."""
import time


class _Avg:
    def __init__(self):
        self.reset()

    def reset(self):
        self.total, self.cnt, self.samples = 0.0, 0, 0

    def record(self, t, n=None):
        self.total += t
        self.cnt += 1
        if n:
            self.samples += n

    def avg(self):
        return self.total / self.cnt if self.cnt else 0.0

    def ips(self):
        if self.total == 0:
            return 0.0
        return (self.samples if self.samples else self.cnt) / self.total


class Benchmark:
    def __init__(self):
        self.reader = _Avg()
        self.batch = _Avg()
        self._t_step = None
        self._t_reader = None
        self.speed_unit = 'steps/s'
        self.enabled = False

    def begin(self):
        self.enabled = True
        self._t_step = time.perf_counter()
        self._t_reader = self._t_step

    def before_reader(self):
        self._t_reader = time.perf_counter()

    def after_reader(self):
        if self.enabled and self._t_reader is not None:
            self.reader.record(time.perf_counter() - self._t_reader)

    def step(self, num_samples=None):
        if not self.enabled:
            return
        now = time.perf_counter()
        self.batch.record(now - self._t_step, num_samples)
        if num_samples:
            self.speed_unit = 'samples/s'
        self._t_step = now
        self._t_reader = now

    def step_info(self, unit=None):
        unit = unit or self.speed_unit
        msg = (f" reader_cost: {self.reader.avg():.5f} s batch_cost: {self.batch.avg():.5f} s "
               f"ips: {self.batch.ips():.3f} {unit}")
        self.reader.reset()
        self.batch.reset()
        return msg

    def end(self):
        self.enabled = False


_bench = Benchmark()


def benchmark():
    return _bench
