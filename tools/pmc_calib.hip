// PMC calibration (profiling only): known-byte streaming kernels with the access
// widths invsim's kernels use (8-B and 16-B per lane loads/stores, 1-B stores),
// over a 1 GiB buffer (beyond L2 and the 256 MiB Infinity Cache).  Run under
// `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (separate passes) and
// divide the counter (KiB) by the bytes printed here to get the correction
// factor per access width (MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 of a wide
// 16-B/lane stream on gfx950; other widths must be calibrated).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void read8(const int64_t *__restrict__ a, int64_t n, int64_t *out) {
    int64_t s = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) s ^= a[i];
    if (s == 0x1234567) out[0] = s;
}
__global__ void read16(const v4i *__restrict__ a, int64_t n, int64_t *out) {
    int s = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        v4i v = a[i];
        s ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (s == 0x1234567) out[0] = s;
}
__global__ void write8(int64_t *__restrict__ a, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) a[i] = i;
}
__global__ void write16(v4i *__restrict__ a, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        v4i v = {(int)i, 1, 2, 3};
        a[i] = v;
    }
}
__global__ void write1(uint8_t *__restrict__ a, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) a[i] = (uint8_t)i;
}

int main() {
    const int64_t bytes = 1ll << 30;
    void *buf;
    int64_t *out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    hipMemset(buf, 1, bytes);
    const dim3 g(2048), b(256);
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(read8, g, b, 0, 0, (const int64_t *)buf, bytes / 8, out);
        hipLaunchKernelGGL(read16, g, b, 0, 0, (const v4i *)buf, bytes / 16, out);
        hipLaunchKernelGGL(write8, g, b, 0, 0, (int64_t *)buf, bytes / 8);
        hipLaunchKernelGGL(write16, g, b, 0, 0, (v4i *)buf, bytes / 16);
        hipLaunchKernelGGL(write1, g, b, 0, 0, (uint8_t *)buf, bytes / 4);
    }
    hipDeviceSynchronize();
    std::printf("bytes per read8/read16/write8/write16 launch: %lld (%.1f KiB); write1: %lld\n", (long long)bytes,
                bytes / 1024.0, (long long)(bytes / 4));
    return 0;
}
