"""rgbac -- MI355X-native hot path of the learned RGBA codec (masked window attention).

Drop-in mirrors of the reference modules live in ``rgbac.models`` and
``rgbac.layers``; the compute is librgbac_hip.so (C ABI: include/rgbac.h)."""
from . import _lib  # noqa: F401

__version__ = "0.1.0"
