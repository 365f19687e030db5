"""eigen_value_amd — MI355X (gfx950) similarity-transform max-eigenvalue
iteration, drop-in for itzmeanjan/eigen_value's SYCL path.

Public surface:
  EigenValue                       drop-in mirror of wrapper/python/similarity_transform.py
  device.DeviceSolver / device.*   device-resident solve and step kernels (torch tensors)
  sharded.ShardedSimilarityTransform  row-block sharding over torch.distributed (RCCL)
"""
from ._lib import EigenValueError, ST_SEM_MAINPY, ST_SEM_SYCL, lib_path, load  # noqa: F401
from .similarity_transform import EigenValue  # noqa: F401

__version__ = "0.5.0"  # st_version() reports the same (tests/test_capi.py)
