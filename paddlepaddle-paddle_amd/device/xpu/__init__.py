"""paddle.device.xpu (reference: python/paddle/device/xpu/__init__.py).  This build targets AMD
MI355X only: there are no XPU devices, so the count is 0 and device operations raise."""

__all__ = ['synchronize', 'device_count', 'set_debug_level']


def device_count():
    return 0


def synchronize(device=None):
    raise ValueError("paddle.device.xpu.synchronize: this build has no XPU devices (MI355X / HIP only)")


def set_debug_level(level=1):
    raise ValueError("paddle.device.xpu.set_debug_level: this build has no XPU devices (MI355X / HIP only)")
