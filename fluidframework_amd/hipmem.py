"""Device buffers from the HIP runtime libmtgpu.so itself links (ctypes; no torch).

PyTorch-ROCm ships its own copy of the HIP runtime; buffers handed to libmtgpu.so's device-side
entry points (mt_deli_ticket_device, mt_deli_raw_from_ops, ...) are allocated here, by the
runtime the library uses, so one process never mixes two runtimes' pointers."""
import ctypes

import numpy as np

from .engine import MtError, lib

_hip = None


def hip():
    global _hip
    if _hip is None:
        lib()  # loads libmtgpu.so and with it /opt/rocm's libamdhip64
        _hip = ctypes.CDLL('libamdhip64.so.7', mode=ctypes.RTLD_GLOBAL)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        _hip.hipMalloc.argtypes = [ctypes.POINTER(vp), sz]
        _hip.hipFree.argtypes = [vp]
        _hip.hipMemcpy.argtypes = [vp, vp, sz, ctypes.c_int]
        _hip.hipMemset.argtypes = [vp, ctypes.c_int, sz]
        _hip.hipDeviceSynchronize.argtypes = []
        _hip.hipHostMalloc.argtypes = [ctypes.POINTER(vp), sz, ctypes.c_uint]
        _hip.hipHostFree.argtypes = [vp]
        for f in ('hipMalloc', 'hipFree', 'hipMemcpy', 'hipMemset', 'hipDeviceSynchronize', 'hipHostMalloc',
                  'hipHostFree'):
            getattr(_hip, f).restype = ctypes.c_int
    return _hip


class DeviceBuffer:
    """`nbytes` of HBM; .ptr is the device address (int)."""

    def __init__(self, nbytes):
        p = ctypes.c_void_p()
        if hip().hipMalloc(ctypes.byref(p), max(1, nbytes)) != 0:
            raise MtError(f'hipMalloc({nbytes}) failed')
        self.ptr, self.nbytes = p.value, nbytes

    def upload(self, arr):
        arr = np.ascontiguousarray(arr)
        assert arr.nbytes <= self.nbytes
        if hip().hipMemcpy(self.ptr, arr.ctypes.data, arr.nbytes, 1) != 0:
            raise MtError('hipMemcpy H2D failed')
        return self

    def download(self, dtype, count=None):
        dtype = np.dtype(dtype)
        count = self.nbytes // dtype.itemsize if count is None else count
        out = np.empty(count, dtype=dtype)
        if hip().hipMemcpy(out.ctypes.data, self.ptr, out.nbytes, 2) != 0:
            raise MtError('hipMemcpy D2H failed')
        return out

    def free(self):
        if self.ptr:
            hip().hipFree(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def device_synchronize():
    """hipDeviceSynchronize on libmtgpu's runtime (bench.py's timed-region brackets)."""
    if hip().hipDeviceSynchronize() != 0:
        raise MtError('hipDeviceSynchronize failed')


class PinnedArray:
    """A numpy array in page-locked host memory (hipHostMalloc): H2D copies from it run at the
    PCIe rate without a staging bounce.  .a is the array; free() (or GC) releases it."""

    def __init__(self, count, dtype):
        dtype = np.dtype(dtype)
        nbytes = max(1, count * dtype.itemsize)
        p = ctypes.c_void_p()
        if hip().hipHostMalloc(ctypes.byref(p), nbytes, 0) != 0:
            raise MtError(f'hipHostMalloc({nbytes}) failed')
        self.ptr = p.value
        buf = (ctypes.c_uint8 * nbytes).from_address(self.ptr)
        self.a = np.frombuffer(buf, dtype=np.uint8)[:count * dtype.itemsize].view(dtype)

    def free(self):
        if self.ptr:
            self.a = None
            hip().hipHostFree(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
