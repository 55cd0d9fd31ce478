// mb_fetch.hip — FETCH_SIZE calibration: stream a known number of bytes (1 GiB, far past the
// 256 MiB MALL) with 4 B/lane, 8 B/lane and 16 B/lane coalesced loads, one launch each, so
// `rocprofv3 --pmc FETCH_SIZE` per kernel can be compared with the bytes actually read
// (profiles/README.md: the correction applied to roofline.traffic).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

template <class T>
__global__ void __launch_bounds__(256) k_read(const T* __restrict__ src, size_t n, unsigned* __restrict__ out) {
    unsigned acc = 0;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const T v = src[i];
        const unsigned* w = reinterpret_cast<const unsigned*>(&v);
#pragma unroll
        for (int k = 0; k < (int)(sizeof(T) / 4); k++) acc ^= w[k];
    }
    if (acc == 0x9e3779b9u) out[0] = acc;  // keeps the loads; practically never stores
}

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));          \
            return 1;                                                             \
        }                                                                         \
    } while (0)

int main() {
    const size_t bytes = (size_t)1 << 30;
    void* buf = nullptr;
    unsigned* out = nullptr;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, 4));
    CK(hipMemset(buf, 1, bytes));
    const int grid = 256 * 8 * 4;
    for (int rep = 0; rep < 3; rep++) {
        k_read<unsigned><<<grid, 256>>>((const unsigned*)buf, bytes / 4, out);
        k_read<uint2><<<grid, 256>>>((const uint2*)buf, bytes / 8, out);
        k_read<uint4><<<grid, 256>>>((const uint4*)buf, bytes / 16, out);
    }
    CK(hipDeviceSynchronize());
    std::printf("bytes_per_launch %zu\n", bytes);
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
