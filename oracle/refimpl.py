"""refimpl — ctypes binding of oracle/_ref/libref_hll.so — the reference's own HyperLogLog.hpp and
MurmurHash3.cpp compiled unmodified (oracle/ref_hll.cpp, `make -C oracle ref`).
TEST INFRASTRUCTURE ONLY: imported by tests/, never by the product path."""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PATH = os.path.join(HERE, "_ref", "libref_hll.so")
_lib = None


def available() -> bool:
    return os.path.exists(PATH)


def lib():
    global _lib
    if _lib is None:
        L = C.CDLL(PATH)
        L.ref_hll_registers.restype = C.c_int
        L.ref_hll_registers.argtypes = [C.POINTER(C.c_uint64), C.c_uint64, C.c_int, C.POINTER(C.c_uint8),
                                        C.POINTER(C.c_double)]
        L.ref_murmur3_x86_32.restype = C.c_uint32
        L.ref_murmur3_x86_32.argtypes = [C.c_char_p, C.c_int, C.c_uint32]
        _lib = L
    return _lib


def murmur3_x86_32(data: bytes, seed: int) -> int:
    return int(lib().ref_murmur3_x86_32(data, len(data), seed))


def hll(codes, b: int = 10):
    """(registers, estimate) of the reference hll::HyperLogLog(b) after add() of every code."""
    c = np.ascontiguousarray(codes, np.uint64)
    regs = np.zeros(1 << b, np.uint8)
    est = C.c_double()
    rc = lib().ref_hll_registers(c.ctypes.data_as(C.POINTER(C.c_uint64)), len(c), b,
                                 regs.ctypes.data_as(C.POINTER(C.c_uint8)), C.byref(est))
    if rc != 0:
        raise ValueError(f"reference HyperLogLog failed ({rc})")
    return regs, est.value
