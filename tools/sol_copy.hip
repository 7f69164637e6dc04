// Speed-of-light reference for a single env.step() launch (profiling only).
// A kernel with no arithmetic that moves the same bytes in the same shape as
// the InvMgmt step at 65 536 envs: one env per lane, SoA rows of Npad 8-byte
// words read and written coalesced, the state buffer reused every launch (as
// the env state is), one launch per "step", timed with hipEvents over 2000
// back-to-back launches.  The gap between this time and the step kernel's is
// the part of the step that the dynamics / Poisson chain costs; the gap
// between this time and bytes / 8 TB/s is launch + ramp + drain overhead that
// no step kernel of this size can avoid.
//   hipcc -O3 --offload-arch=gfx950 tools/sol_copy.hip -o tools/sol_copy && tools/sol_copy
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

template <int RROWS, int WROWS>
__global__ void __launch_bounds__(256) soa_move(const int64_t *__restrict__ src, int64_t *__restrict__ dst, int64_t S) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t acc[RROWS > 0 ? RROWS : 1];
#pragma unroll
    for (int r = 0; r < RROWS; r++) acc[r] = src[r * S + e];
    int64_t x = 0;
#pragma unroll
    for (int r = 0; r < RROWS; r++) x += acc[r];
#pragma unroll
    for (int r = 0; r < WROWS; r++) dst[r * S + e] = x + r;
}

__global__ void empty_kernel(int64_t *p) {
    if (p == nullptr && threadIdx.x == 999) p[0] = 0;
}

template <int R, int W>
static void run(const char *name, int64_t n, int bs, int64_t *src, int64_t *dst, hipEvent_t a, hipEvent_t b) {
    const dim3 g((unsigned)(n / bs)), blk(bs);
    for (int i = 0; i < 100; i++) hipLaunchKernelGGL((soa_move<R, W>), g, blk, 0, 0, src, dst, n);
    const int K = 2000;
    hipEventRecord(a, 0);
    for (int i = 0; i < K; i++) hipLaunchKernelGGL((soa_move<R, W>), g, blk, 0, 0, src, dst, n);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double us = ms * 1e3 / K;
    const double bytes = (double)n * 8 * (R + W);
    std::printf("%-34s envs=%lld wg=%d read=%dB write=%dB per env: %.2f us/launch, %.0f GB/s (%.3f of 8 TB/s)\n", name,
                (long long)n, bs, R * 8, W * 8, us, bytes / us * 1e-3, bytes / us * 1e-3 / 8000.0);
}

int main() {
    const int64_t n = 65536;
    int64_t *src, *dst;
    if (hipMalloc(&src, n * 8 * 64) != hipSuccess || hipMalloc(&dst, n * 8 * 64) != hipSuccess) return 1;
    hipMemset(src, 1, n * 8 * 64);
    hipMemset(dst, 0, n * 8 * 64);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    {
        const int K = 2000;
        for (int i = 0; i < 100; i++) hipLaunchKernelGGL(empty_kernel, dim3(1024), dim3(64), 0, 0, src);
        hipEventRecord(a, 0);
        for (int i = 0; i < K; i++) hipLaunchKernelGGL(empty_kernel, dim3(1024), dim3(64), 0, 0, src);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        std::printf("%-34s 1024 x 64 threads: %.2f us/launch\n", "empty kernel", ms * 1e3 / K);
    }
    // InvMgmt Backlog step, measured traffic shape: ~244 B read, ~382 B written per env
    run<31, 48>("invmgmt step bytes (actual)", n, 64, src, dst, a, b);
    run<31, 48>("invmgmt step bytes (actual)", n, 128, src, dst, a, b);
    run<31, 48>("invmgmt step bytes (actual)", n, 256, src, dst, a, b);
    // algorithmic B1 = 746 B: 448 read + 298 write (rounded to 8-B rows)
    run<56, 37>("invmgmt step bytes (algorithmic B1)", n, 64, src, dst, a, b);
    run<56, 37>("invmgmt step bytes (algorithmic B1)", n, 256, src, dst, a, b);
    run<62, 0>("read only 496 B", n, 256, src, dst, a, b);
    run<1, 62>("write only 496 B", n, 256, src, dst, a, b);
    run<8, 8>("small 128 B", n, 256, src, dst, a, b);
    // Newsvendor step: ~96 B read, ~94 B written
    run<12, 12>("newsvendor step bytes", n, 64, src, dst, a, b);
    // Net default step at 32 768 envs: 1046 B
    run<72, 59>("net step bytes (32768 envs)", n / 2, 64, src, dst, a, b);
    return 0;
}
