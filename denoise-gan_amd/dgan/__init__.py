"""dgan — MI355X-native (gfx950) hot path of the denoise-gan training step.

Layers:
  dgan._lib     ctypes binding of libdgan.so (include/dgan.h)
  dgan.ops      tensor-level wrappers (conv, BN, losses, Adam, data movement)
  dgan.nets     pix2pix generator / discriminator executors (explicit fwd/bwd)
  dgan.dist     data-parallel gradient exchange (RCCL via torch.distributed)
"""
from .build import LIB_PATH, build  # noqa: F401

__all__ = ["LIB_PATH", "build"]
