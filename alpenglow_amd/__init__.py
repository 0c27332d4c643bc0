"""alpenglow_amd: MI355X-native Reed-Solomon shredder path for the Alpenglow reference.

The hot path (reed-solomon-simd 3.1.0 encode / reconstruct behind
/root/reference/src/shredder/reed_solomon.rs) runs as HIP kernels for gfx950 in
libalpenglow_rs.so (C ABI: include/alpenglow_rs.h).  ``alpenglow_amd.rs`` is the Python
host-side mirror used by tests and bench.py.
"""

from . import rs  # noqa: F401

__all__ = ["rs"]
