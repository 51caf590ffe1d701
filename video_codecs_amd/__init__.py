"""video_codecs_amd -- MI355X-native HM-16.5rc1 CU mode-decision hot path.

The product is the HIP/C++ library `libhvx.so` (C-ABI in include/hvx.h);
`video_codecs_amd.hvx` is its Python binding (device buffers via torch).
Importing this package loads nothing native.
"""
__all__ = ["hvx"]
