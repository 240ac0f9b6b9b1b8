"""radnerf_amd — MI355X-native (gfx950) Rad-NeRF rendering hot path.

The product is librn.so (HIP kernels behind the C ABI of include/radnerf.h);
this package is the Python host side mirroring the reference's interfaces:
  vren               drop-in for the `vren` CUDA extension (binding.cpp)
  custom_functions   RayAABBIntersector / RayMarcher / VolumeRenderer / TruncExp
  networks           MNGP / NGP / Ray_Gate on the fused HIP field + gate
  rendering          render / ml_render (reference structure)
  fused              single-chain fused ml_render for training
  dist               ray-batch data parallelism over RCCL
"""
from ._lib import lib, LIB_PATH  # noqa: F401

__version__ = "0.1.0"
