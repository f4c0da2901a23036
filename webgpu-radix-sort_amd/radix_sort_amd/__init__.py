"""MI355X-native 4-way LSD radix sort — Python host mirror of the WebGPU-Radix-Sort API.

    from radix_sort_amd import RadixSortKernel
    k = RadixSortKernel(keys=keys_tensor, values=values_tensor, count=n, bit_count=32)
    k.dispatch()            # sorts keys/values in place on the current HIP stream

All compute runs in librsort.so (hand-written gfx950 HIP kernels); this package only marshals
arguments across the C ABI (include/rsort.h).
"""
from ._lib import RadixSortError, load as load_library  # noqa: F401
from .kernel import (DeviceBuffer, PrefixSumKernel, RadixSortBufferKernel,  # noqa: F401
                     RadixSortKernel, RadixSortTextureKernel)
from . import ops  # noqa: F401
from .group import RadixSortGroup  # noqa: F401

__all__ = ["RadixSortKernel", "RadixSortBufferKernel", "RadixSortTextureKernel", "PrefixSumKernel",
           "DeviceBuffer", "RadixSortGroup",
           "RadixSortError", "load_library", "ops"]
