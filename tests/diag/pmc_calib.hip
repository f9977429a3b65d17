// PMC calibration (TEST INFRASTRUCTURE): kernels that move a known number
// of bytes with the access widths the physics kernels use, so FETCH_SIZE /
// WRITE_SIZE can be converted to bytes for those widths (MI355X_MICROARCH.md
// calibrates only 16-B-per-lane streaming loads and stores).  Each buffer is
// 1 GiB, past the 256 MiB Infinity Cache, and each kernel runs 3 times.
//   read4   : 4 B per lane, coalesced loads      (1 GiB read)
//   read16  : 16 B per lane, coalesced loads     (1 GiB read)
//   write4  : 4 B per lane, coalesced stores     (1 GiB written)
//   write16 : 16 B per lane, coalesced stores    (1 GiB written)
//   copy116 : 116-B records copied as dwords, 29 per record (refit's node
//             write-back pattern): 1 GiB read + 1 GiB written
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__global__ void read4(const uint32_t *__restrict__ p, size_t n, uint32_t *out)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc ^= p[i];
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void read16(const uint4 *__restrict__ p, size_t n, uint32_t *out)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void write4(uint32_t *__restrict__ p, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (uint32_t)i;
}

__global__ void write16(uint4 *__restrict__ p, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

__global__ void copy116(const uint32_t *__restrict__ src, uint32_t *__restrict__ dst, size_t words)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < words; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e__ = (x);                                                                  \
        if (e__ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e__));                      \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

int main()
{
    const size_t bytes = (size_t)1 << 30;
    uint32_t *a = nullptr, *b = nullptr, *out = nullptr;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(b, 2, bytes));
    const dim3 grid(256 * 8), block(256);
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(read4, grid, block, 0, 0, a, bytes / 4, out);
        hipLaunchKernelGGL(read16, grid, block, 0, 0, (const uint4 *)a, bytes / 16, out);
        hipLaunchKernelGGL(write4, grid, block, 0, 0, b, bytes / 4);
        hipLaunchKernelGGL(write16, grid, block, 0, 0, (uint4 *)b, bytes / 16);
        // 116-B records: (1 GiB / 116) whole records
        const size_t recs = bytes / 116;
        hipLaunchKernelGGL(copy116, grid, block, 0, 0, a, b, recs * 29);
        CK(hipGetLastError());
    }
    CK(hipDeviceSynchronize());
    std::printf("pmc_calib: 1 GiB per kernel (copy116: %zu B each way)\n", (bytes / 116) * 116);
    return 0;
}
