"""ipfixprobe_amd -- MI355X-native drop-in for ipfixprobe's parse -> hash -> biflow-cache path.

The product is libipxg.so (HIP kernels for gfx950 behind the C-ABI in include/ipxg.h) and
the C++ host layer in ipfixprobe_amd/host.  `engine` holds ctypes bindings used by the tests
and bench.py.
"""
from .engine import (BATCH_DEVICE, DESC_DTYPE, DLT_EN10MB, DLT_LINUX_SLL, DLT_LINUX_SLL2,  # noqa: F401
                     DLT_RAW, FLOW_DTYPE, PARSED_DTYPE, STATS_FIELDS, Engine, IpxgError,
                     load_capture, make_config, run_capture)

__all__ = ["Engine", "IpxgError", "load_capture", "make_config", "run_capture"]
