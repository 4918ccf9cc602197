// Calibration of the HBM counters (rocprofv3 FETCH_SIZE / WRITE_SIZE) for the access widths the
// merge engine uses (MI355X_MICROARCH.md: only 16 B/lane streaming reads and writes are calibrated).
// Each kernel moves a known number of bytes over a buffer far larger than the Infinity Cache;
// tools/pmc_calib.py launches them and compares the counters with the bytes.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/pmc_calib.hip -o tools/libpmc_calib.so
#include <hip/hip_runtime.h>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// streaming read of n elements of T, one per lane per iteration, grid-stride; the xor lands in
// out[] only for an impossible value, so the loads stay
template <class T>
__global__ void calib_read(const T* __restrict__ src, size_t n, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const T v = src[i];
        uint32_t w[sizeof(T) / 4];
        __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
        for (unsigned k = 0; k < sizeof(T) / 4; k++) acc ^= w[k];
    }
    if (acc == 0x9E3779B9u) out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
template <class T>
__global__ void calib_write(T* __restrict__ dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        T v;
        uint32_t w[sizeof(T) / 4];
#pragma unroll
        for (unsigned k = 0; k < sizeof(T) / 4; k++) w[k] = (uint32_t)i + k;
        __builtin_memcpy(&v, w, sizeof(T));
        dst[i] = v;
    }
}
// the text arena's pattern: one wave writes `len` consecutive bytes (one byte per lane) at the start
// of every `stride`-byte region (an insert appending a short text to a document's arena)
__global__ void calib_write_bytes(uint8_t* __restrict__ dst, size_t regions, uint32_t stride, uint32_t len) {
    const uint32_t lane = threadIdx.x & 63u;
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
    for (size_t r = wave; r < regions; r += nw)
        if (lane < len) dst[r * stride + lane] = (uint8_t)(r + lane);
}

extern "C" {
#define LAUNCH(kern, ...) hipLaunchKernelGGL(kern, dim3(4096), dim3(256), 0, 0, __VA_ARGS__)
hipError_t calib_read_u32(const void* src, size_t bytes, void* out) {
    LAUNCH(calib_read<uint32_t>, (const uint32_t*)src, bytes / 4, (uint32_t*)out);
    return hipGetLastError();
}
hipError_t calib_read_u64(const void* src, size_t bytes, void* out) {
    LAUNCH(calib_read<uint64_t>, (const uint64_t*)src, bytes / 8, (uint32_t*)out);
    return hipGetLastError();
}
hipError_t calib_read_u128(const void* src, size_t bytes, void* out) {
    LAUNCH(calib_read<u32x4>, (const u32x4*)src, bytes / 16, (uint32_t*)out);
    return hipGetLastError();
}
hipError_t calib_write_u32(void* dst, size_t bytes) {
    LAUNCH(calib_write<uint32_t>, (uint32_t*)dst, bytes / 4);
    return hipGetLastError();
}
hipError_t calib_write_u64(void* dst, size_t bytes) {
    LAUNCH(calib_write<uint64_t>, (uint64_t*)dst, bytes / 8);
    return hipGetLastError();
}
hipError_t calib_write_u128(void* dst, size_t bytes) {
    LAUNCH(calib_write<u32x4>, (u32x4*)dst, bytes / 16);
    return hipGetLastError();
}
hipError_t calib_write_text(void* dst, size_t bytes, uint32_t stride, uint32_t len) {
    LAUNCH(calib_write_bytes, (uint8_t*)dst, bytes / stride, stride, len);
    return hipGetLastError();
}
}
