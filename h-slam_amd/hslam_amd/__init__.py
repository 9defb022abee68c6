"""hslam_amd — MI355X-native photometric-BA hot path of H-SLAM (host-side Python bindings).

The product is the C-ABI library ``libhslam_amd.so`` (HIP kernels for gfx950 +
C++ host layer) built from ``h-slam_amd/csrc``; this package only wraps it with
ctypes and generates synthetic scenes.  See DESIGN.md.
"""
