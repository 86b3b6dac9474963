"""cndp_amd -- MI355X-native drop-in for CNDP's per-burst parse / flow-hash /
LPM classify hot path.

Native code: cndp_amd/lib/libcndp_gpu.so (HIP kernels for gfx950 + the C
control plane), C-ABI in include/cndp_fib.h and include/cndp_gpu.h.  The
Python modules here are thin ctypes mirrors of that ABI plus a synthetic
packet generator; importing them never falls back to a CPU path.
"""
from . import native
from .native import (CNDP_MODE_CNET, CNDP_MODE_HASH, CNDP_MODE_L3FWD, CNDP_NH_INVALID,  # noqa: F401
                     CNE_FIB_DIR24_8, CNE_FIB_DUMMY, CNE_FIB_TRIE, MS_RSS_KEY)

__version__ = "0.1.0"


def __getattr__(name):
    # lazy: these load libcndp_gpu.so on first use (and raise if it is absent)
    if name in ("Fib", "Fib6", "node_ip4_route_add", "node_ip4_add_input", "node_ip6_add_input"):
        from . import fib
        return getattr(fib, name)
    if name == "Classifier":
        from .classify import Classifier
        return Classifier
    raise AttributeError(name)
