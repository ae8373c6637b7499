"""paddle.callbacks (reference: python/paddle/callbacks.py): the hapi training callbacks."""
from .hapi.callbacks import *  # noqa: F401,F403
from .hapi.callbacks import (Callback, ProgBarLogger, ModelCheckpoint, VisualDL, LRScheduler,  # noqa: F401
                             EarlyStopping, ReduceLROnPlateau, WandbCallback)

__all__ = ['Callback', 'ProgBarLogger', 'ModelCheckpoint', 'VisualDL', 'LRScheduler', 'EarlyStopping',
           'ReduceLROnPlateau', 'WandbCallback']
