// Would a persistent, software-pipelined step beat the one-shot step launch?
// (profiling only.)  The same no-arithmetic SoA copy as
// tools/sol_copy.hip, with the InvMgmt step's bytes per env (248 B read,
// 384 B written) at 65 536 envs, launched two ways:
//   one-shot   one env per lane, every workgroup loads, then stores (the
//              step kernels' shape: all waves in the same phase)
//   pipelined  a grid of ngroups / G workgroups; each walks G tiles
//              (tile j at blockIdx + j * gridDim, so the grid sweeps memory
//              together) and issues tile j+1's loads before tile j's stores,
//              so reads and writes overlap inside every wave
// One launch per "step", 2000 back-to-back launches timed with hipEvents.  If
// the pipelined copy is not faster than the one-shot copy, the step kernel
// (whose body is ~1 us above the one-shot copy) will not be either.
//   hipcc -O3 --offload-arch=gfx950 tools/pipe_copy.hip -o tools/pipe_copy && tools/pipe_copy
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

template <int R, int W, int G>
__global__ void __launch_bounds__(256) soa_pipe(const int64_t *__restrict__ src, int64_t *__restrict__ dst, int64_t S) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t cur[R], nxt[R];
#pragma unroll
    for (int r = 0; r < R; r++) cur[r] = src[r * S + e];
#pragma unroll
    for (int j = 0; j < G; j++) {
        if (j + 1 < G) {
#pragma unroll
            for (int r = 0; r < R; r++) nxt[r] = src[r * S + e + stride];
        }
        int64_t x = 0;
#pragma unroll
        for (int r = 0; r < R; r++) x += cur[r];
#pragma unroll
        for (int r = 0; r < W; r++) dst[r * S + e] = x + r;
#pragma unroll
        for (int r = 0; r < R; r++) cur[r] = nxt[r];
        e += stride;
    }
}

template <int R, int W, int G>
static void run(int64_t n, int bs, int64_t *src, int64_t *dst, hipEvent_t a, hipEvent_t b) {
    const dim3 g((unsigned)(n / bs / G)), blk(bs);
    for (int i = 0; i < 100; i++) hipLaunchKernelGGL((soa_pipe<R, W, G>), g, blk, 0, 0, src, dst, n);
    const int K = 2000;
    hipEventRecord(a, 0);
    for (int i = 0; i < K; i++) hipLaunchKernelGGL((soa_pipe<R, W, G>), g, blk, 0, 0, src, dst, n);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double us = ms * 1e3 / K;
    const double bytes = (double)n * 8 * (R + W);
    std::printf("%-10s envs=%lld wg=%3d G=%d grid=%5u read=%dB write=%dB per env: %.2f us/launch, %.0f GB/s (%.3f of 8 TB/s)\n",
                G == 1 ? "one-shot" : "pipelined", (long long)n, bs, G, g.x, R * 8, W * 8, us, bytes / us * 1e-3,
                bytes / us * 1e-3 / 8000.0);
}

template <int R, int W>
static void sweep(int64_t n, int64_t *src, int64_t *dst, hipEvent_t a, hipEvent_t b) {
    for (int bs : {64, 128, 256}) {
        run<R, W, 1>(n, bs, src, dst, a, b);
        run<R, W, 2>(n, bs, src, dst, a, b);
        run<R, W, 4>(n, bs, src, dst, a, b);
        if (n / bs / 8 >= 64) run<R, W, 8>(n, bs, src, dst, a, b);
    }
}

int main() {
    const int64_t nmax = 262144;
    int64_t *src, *dst;
    if (hipMalloc(&src, nmax * 8 * 64) != hipSuccess || hipMalloc(&dst, nmax * 8 * 64) != hipSuccess) return 1;
    hipMemset(src, 1, nmax * 8 * 64);
    hipMemset(dst, 0, nmax * 8 * 64);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    std::printf("# InvMgmt step bytes (31 rows read, 48 written), 65 536 envs\n");
    sweep<31, 48>(65536, src, dst, a, b);
    std::printf("# the same bytes at 32 768 envs (the LostSales shard's size)\n");
    sweep<31, 48>(32768, src, dst, a, b);
    std::printf("# 262 144 envs\n");
    sweep<31, 48>(262144, src, dst, a, b);
    return 0;
}
