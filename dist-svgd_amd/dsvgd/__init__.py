"""dsvgd -- MI355X-native SVGD (drop-in for Sandy4321/dist-svgd's `dsvgd`).

Reference surface (dsvgd/__init__.py:1-3): `name`, `Sampler`, `DistSampler`.
The particle update runs in hand-written gfx950 kernels (libdsvgd_hip.so,
C ABI in include/dsvgd.h); there is no CPU compute path.
"""
name = 'dsvgd'
from .sampler import Sampler  # noqa: E402
from .distsampler import DistSampler  # noqa: E402
from . import kernels, metrics, targets  # noqa: E402
from .kernels import RBF  # noqa: E402
from .engine import PhiEngine  # noqa: E402

__all__ = ["name", "Sampler", "DistSampler", "RBF", "PhiEngine", "kernels", "metrics", "targets"]
