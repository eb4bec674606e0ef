"""octree_pathtracing_amd -- MI355X-native (gfx950) octree path-tracing hot path.

Drop-in replacement for the per-pixel hot path of kekley/octree_pathtracing
(renderer::render -> octree traversal -> Sphere/Cuboid hit -> ray scatter) behind the C ABI
in include/octpt.h.  Python modules:
  _lib       ctypes binding of liboctpt.so (fails loudly when it is missing)
  scene      Scene / Octree / Material / Camera mirror + seeded synthetic configs C1-C5
  renderer   HipRenderer: the RenderingBackend / FrameInFlight surface
  distributed  tile-sharded multi-GPU rendering with an RCCL gather
"""
from . import _lib  # noqa: F401

__all__ = ["_lib"]
