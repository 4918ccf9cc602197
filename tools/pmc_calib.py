#!/usr/bin/env python3
"""Drives tools/libpmc_calib.so (tools/pmc_calib.hip): each calibration kernel once over a 1 GiB
buffer (4x the Infinity Cache), so rocprofv3's FETCH_SIZE / WRITE_SIZE can be compared with the
bytes each kernel moves.  Run under rocprofv3 on the GPU box (tools/pmc_calib.sh); prints the
known byte counts as JSON (pmc_calib.sh joins them with the counters).
The text pattern: 8 bytes written at the start of every 512-byte region (a short insert appended
to a document's arena)."""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
from fluidframework_amd.hipmem import DeviceBuffer, hip  # noqa: E402

N = 1 << 30
L = ctypes.CDLL(os.path.join(HERE, 'tools', 'libpmc_calib.so'))
for f in ('calib_read_u32', 'calib_read_u64', 'calib_read_u128'):
    getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
for f in ('calib_write_u32', 'calib_write_u64', 'calib_write_u128'):
    getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_size_t]
L.calib_write_text.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32]
buf = DeviceBuffer(N)
sink = DeviceBuffer(4096 * 256 * 4)
known = {}
for w in ('u32', 'u64', 'u128'):
    assert getattr(L, 'calib_write_' + w)(ctypes.c_void_p(buf.ptr), N) == 0
    known['calib_write<%s>' % w] = {'write_bytes': N}
for w in ('u32', 'u64', 'u128'):
    assert getattr(L, 'calib_read_' + w)(ctypes.c_void_p(buf.ptr), N, ctypes.c_void_p(sink.ptr)) == 0
    known['calib_read<%s>' % w] = {'read_bytes': N}
STRIDE, LEN = 512, 8
assert L.calib_write_text(ctypes.c_void_p(buf.ptr), N, STRIDE, LEN) == 0
known['calib_write_bytes'] = {'write_bytes': (N // STRIDE) * LEN, 'lines_touched_128B': N // STRIDE}
assert hip().hipDeviceSynchronize() == 0
print(json.dumps(known))
buf.free()
sink.free()
