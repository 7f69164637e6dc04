// Micro-benchmark (profiling only): cost of numpy-exact Poisson(lam) draws on
// gfx950 for the sequential per-lane sampler vs the 4-lane group sampler, at
// several lane counts (1 wave/SIMD = 65536 lanes ... 8 waves/SIMD).
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17 \
//          -I or-gym-inventory_amd/csrc tools/poisson_bench.hip -o tools/poisson_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "group_rng.hpp"

using namespace invsim;

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
            return 1;                                                            \
        }                                                                        \
    } while (0)

template <int MODE>
__global__ void __launch_bounds__(64) draw_kernel(PtrsConst c, const double *rhs, int K, int64_t *out,
                                                  int n_env) {
    const int lane = threadIdx.x;
    const bool seq = MODE == 0 || MODE == 3;
    const int env = seq ? (int)(blockIdx.x * 64 + lane) : (int)(blockIdx.x * 16 + lane / 4);
    if (env >= n_env) return;
    Pcg g;
    uint32_t w[4] = {(uint32_t)env, 0, 0, 0};
    seed_pcg64(w, 1, g);
    int64_t acc = 0;
    for (int k = 0; k < K; k++) {
        int64_t d;
        if (MODE == 0) d = np_poisson(g, c);
        else if (MODE == 1) d = np_poisson_grp(g, c, nullptr);
        else if (MODE == 2) d = np_poisson_grp(g, c, rhs);
        else d = np_poisson(g, c, rhs);
        acc += d;
    }
    if (seq || (lane & 3) == 0) out[env] = acc;
}

__global__ void __launch_bounds__(64) rng_only_kernel(int K, int64_t *out, int n_env) {
    const int env = (int)(blockIdx.x * 64 + threadIdx.x);
    if (env >= n_env) return;
    Pcg g;
    uint32_t w[4] = {(uint32_t)env, 0, 0, 0};
    seed_pcg64(w, 1, g);
    uint64_t acc = 0;
    for (int k = 0; k < 3 * K; k++) acc ^= g.next64();
    out[env] = (int64_t)acc;
}

int main() {
    const double lam = 20.0;
    PtrsConst c = ptrs_const(lam);
    std::vector<double> tab;
    {
        const int k0 = 0, n = 200;
        for (int k = k0; k < k0 + n; k++) tab.push_back(-c.lam + (double)k * c.loglam - np_loggam((double)(k + 1)));
        c.k0 = k0;
        c.nk = n;
        c.toff = 0;
    }
    double *d_tab;
    int64_t *d_out;
    CK(hipMalloc(&d_tab, tab.size() * 8));
    CK(hipMemcpy(d_tab, tab.data(), tab.size() * 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&d_out, (size_t)8 * 1048576 * 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int K = 64;
    for (int n_env : {65536, 131072, 262144, 524288}) {
        for (int mode = -1; mode < 4; mode++) {
            int lanes_per_env = (mode == 1 || mode == 2) ? 4 : 1;
            int blocks = (n_env * lanes_per_env + 63) / 64;
            float best = 1e30f;
            for (int rep = 0; rep < 5; rep++) {
                CK(hipEventRecord(a, 0));
                if (mode == -1) hipLaunchKernelGGL(rng_only_kernel, dim3(blocks), dim3(64), 0, 0, K, d_out, n_env);
                if (mode == 0) hipLaunchKernelGGL(draw_kernel<0>, dim3(blocks), dim3(64), 0, 0, c, d_tab, K, d_out, n_env);
                if (mode == 1) hipLaunchKernelGGL(draw_kernel<1>, dim3(blocks), dim3(64), 0, 0, c, d_tab, K, d_out, n_env);
                if (mode == 2) hipLaunchKernelGGL(draw_kernel<2>, dim3(blocks), dim3(64), 0, 0, c, d_tab, K, d_out, n_env);
                if (mode == 3) hipLaunchKernelGGL(draw_kernel<3>, dim3(blocks), dim3(64), 0, 0, c, d_tab, K, d_out, n_env);
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                if (ms < best) best = ms;
            }
            const char *name[] = {"rng3x (6 next64/draw-equiv)", "seq+fast", "grp+fast", "grp+tab+fast", "seq+tab+fast"};
            std::printf("n_env=%7d %-28s  %8.3f us/launch  %7.3f us per draw-round  %6.2f Gdraws/s\n", n_env,
                        name[mode + 1], best * 1e3, best * 1e3 / K, (double)n_env * K / (best * 1e-3) / 1e9);
        }
    }
    // parity spot check: seq vs grp+tab produce identical sums
    std::vector<int64_t> h1(65536), h2(65536);
    hipLaunchKernelGGL(draw_kernel<0>, dim3(1024), dim3(64), 0, 0, c, d_tab, K, d_out, 65536);
    CK(hipMemcpy(h1.data(), d_out, 65536 * 8, hipMemcpyDeviceToHost));
    hipLaunchKernelGGL(draw_kernel<2>, dim3(4096), dim3(64), 0, 0, c, d_tab, K, d_out, 65536);
    CK(hipMemcpy(h2.data(), d_out, 65536 * 8, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < 65536; i++) bad += h1[i] != h2[i];
    std::printf("seq vs grp+tab mismatches: %d\n", bad);
    hipLaunchKernelGGL(draw_kernel<3>, dim3(1024), dim3(64), 0, 0, c, d_tab, K, d_out, 65536);
    CK(hipMemcpy(h2.data(), d_out, 65536 * 8, hipMemcpyDeviceToHost));
    bad = 0;
    for (int i = 0; i < 65536; i++) bad += h1[i] != h2[i];
    std::printf("seq vs seq+tab mismatches: %d\n", bad);
    return 0;
}
