"""datafusion-parallelism_amd — MI355X-native parallel hash join (build + inner probe).

A drop-in for the hot path of jamesfer/datafusion-parallelism: gfx950
HIP kernels behind the C ABI of ``include/hj.h`` (library ``lib/libdfp_hj.so``), a host
mirror of the reference's operator interface (:mod:`.operator`) and the multi-GPU radix
exchange (:mod:`.distributed`).

Importing the package does not need a GPU; calling into the kernels does, and fails
loudly (``HJ_ERR_NO_DEVICE``) without one — there is no CPU fallback.
"""
from ._lib import HjError, device_count, load  # noqa: F401
from .table import HashTable  # noqa: F401

__all__ = ["HashTable", "HjError", "device_count", "load"]
