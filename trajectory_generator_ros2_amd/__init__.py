"""trajectory_generator_ros2_amd — MI355X-native batched minimum-snap solver.

The product is ``lib/libtgms.so`` (HIP kernels for gfx950 behind the C ABI in
``include/tgms.h``) plus the C++ ``MinSnap`` primitive in ``host/`` that plugs it
behind the reference's ``Trajectory`` interface.  This Python package only
marshals buffers for tests, the benchmark and multi-GPU sharding.
"""
from ._lib import (ERR_DEVICE, ERR_INVALID_ARG, ERR_NO_DEVICE, ERR_NONFINITE, ERR_SINGULAR, ERR_SKIPPED,
                   ERR_UNSUPPORTED, METHOD_BAND_KKT, METHOD_DENSE_KKT, METHOD_REDUCED, OK, YAW_CONSTANT,
                   YAW_VELOCITY, TgmsError)

__all__ = [
    "OK", "ERR_INVALID_ARG", "ERR_SINGULAR", "ERR_NONFINITE", "ERR_NO_DEVICE", "ERR_DEVICE",
    "ERR_UNSUPPORTED", "ERR_SKIPPED", "METHOD_REDUCED", "METHOD_DENSE_KKT", "METHOD_BAND_KKT", "YAW_CONSTANT", "YAW_VELOCITY",
    "TgmsError",
]
