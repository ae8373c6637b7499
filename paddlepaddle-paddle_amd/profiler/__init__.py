"""paddle.profiler (reference: python/paddle/profiler/__init__.py)."""
from .profiler import (Profiler, ProfilerState, ProfilerTarget, SummaryView, SortedKeys,  # noqa: F401
                       export_chrome_tracing, export_protobuf, make_scheduler)
from .utils import RecordEvent, TracerEventType, load_profiler_result, in_profiler_mode  # noqa: F401
from .timer import benchmark  # noqa: F401

__all__ = ['ProfilerState', 'ProfilerTarget', 'make_scheduler', 'export_chrome_tracing', 'export_protobuf',
           'Profiler', 'RecordEvent', 'load_profiler_result', 'SortedKeys', 'SummaryView']
