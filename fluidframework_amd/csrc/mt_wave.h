// mt_wave.h -- wave64 primitives for gfx950 (CDNA4): DPP inclusive scan, ballot helpers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MT_DEV __device__ __forceinline__

MT_DEV int lane_id() { return (int)__lane_id(); }

// Order this wave's LDS traffic across a pass boundary (lanes exchange data through LDS).
MT_DEV void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Inclusive prefix sum over the 64 lanes: 4 row_shr steps inside each 16-lane row, then
// row_bcast:15 / row_bcast:31 to carry across rows (GFX9-family DPP; no LDS round trip).
MT_DEV int wave_incl_scan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

MT_DEV int wave_bcast(int v, int src_lane) { return __shfl(v, src_lane, 64); }
MT_DEV int wave_last(int v) { return __builtin_amdgcn_readlane(v, 63); }

MT_DEV int wave_sum(int v) {
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 8, 64);
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    return v;
}

MT_DEV int wave_max(int v) {
    v = max(v, __shfl_xor(v, 1, 64));
    v = max(v, __shfl_xor(v, 2, 64));
    v = max(v, __shfl_xor(v, 4, 64));
    v = max(v, __shfl_xor(v, 8, 64));
    v = max(v, __shfl_xor(v, 16, 64));
    v = max(v, __shfl_xor(v, 32, 64));
    return v;
}

MT_DEV int wave_min(int v) {
    v = min(v, __shfl_xor(v, 1, 64));
    v = min(v, __shfl_xor(v, 2, 64));
    v = min(v, __shfl_xor(v, 4, 64));
    v = min(v, __shfl_xor(v, 8, 64));
    v = min(v, __shfl_xor(v, 16, 64));
    v = min(v, __shfl_xor(v, 32, 64));
    return v;
}

MT_DEV uint64_t wave_ballot(bool p) { return __ballot(p); }
MT_DEV int first_lane(uint64_t m) { return m ? __ffsll((unsigned long long)m) - 1 : -1; }
