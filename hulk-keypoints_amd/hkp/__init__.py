"""hkp — host runtime of the MI355X-native keypoint-heatmap path.

_lib      ctypes binding of libhulkkp.so (include/hulkkp.h)
ops       tensor-level kernel wrappers
net       network executor over the reference-shaped module tree
autograd  the autograd.Function that runs the backward kernels
"""
from ._lib import HkpError, LIB_PATH, lib, version  # noqa: F401
