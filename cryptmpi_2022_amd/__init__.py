"""cryptmpi_2022_amd — MI355X-native AEAD seal/open engine for CryptMPI's per-message hot path.

The product is libcmpi_aead.so (hand-written gfx950 HIP kernels behind the C ABI in
include/cmpi_aead.h).  This package holds its sources (csrc/), the ctypes binding (_native),
the Python mirror of the reference interface (aead), and synthetic-input helpers (synth).
"""
__all__ = ["aead", "synth"]
