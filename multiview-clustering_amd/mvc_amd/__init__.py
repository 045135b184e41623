"""mvc_amd — MI355X-native Gibbs sampler for JunR3/Multiview-Clustering.

Host-side Python mirror of the reference's R entry point
(``run_gibbs_cpp``, /root/reference/Multiview/multiview_gibbs.cpp:105-131)
over the C ABI of libmvc_hip.so (include/mvc.h).
"""
from ._lib import LIB_PATH, MvcError, lib  # noqa: F401
from .sampler import (Sampler, ari, device_gemm_check, device_math, device_seq_uniforms,  # noqa: F401
                      device_tree64, get_final_clusters, run_gibbs_cpp)

__all__ = ["run_gibbs_cpp", "get_final_clusters", "Sampler", "ari", "MvcError", "lib", "LIB_PATH"]
