// Seeding kernels shared by all env families.
//
// gymnasium Env.reset(seed=s) -> seeding.np_random(s) -> numpy SeedSequence(s)
// -> PCG64 (newsvendor.py:102, inventory_management.py:197,
// network_management.py:303).  One thread per env, pure 32-bit integer work.
#include "kernels.hpp"

namespace invsim {

__global__ void __launch_bounds__(256)
seed_range_kernel(Common cm, uint64_t base_lo, uint64_t base_hi, int64_t first, const uint8_t *mask) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= cm.N) return;
    if (mask && !mask[e]) return;
    // seed = base + first + e as a 128-bit integer (first + e >= 0)
    uint64_t add = (uint64_t)(first + e);
    uint64_t lo = base_lo + add;
    uint64_t hi = base_hi + (lo < base_lo ? 1ULL : 0ULL);
    uint32_t w[4] = {(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
    int nw = 4;
    while (nw > 1 && w[nw - 1] == 0) nw--;  // numpy _coerce_to_uint32_array: minimal words
    Pcg g;
    seed_pcg64(w, nw, g);
    cm.rng.store_all(e, g);
    if (cm.u32buf) cm.u32buf[e] = 0;   // a new Generator: pcg64 has_uint32 = 0
}

__global__ void __launch_bounds__(256)
seed_words_kernel(Common cm, const uint32_t *words, const int32_t *nwords, const uint8_t *mask) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= cm.N) return;
    if (mask && !mask[e]) return;
    uint32_t w[4] = {words[4 * e], words[4 * e + 1], words[4 * e + 2], words[4 * e + 3]};
    int nw = nwords[e];
    nw = nw < 1 ? 1 : (nw > 4 ? 4 : nw);
    Pcg g;
    seed_pcg64(w, nw, g);
    cm.rng.store_all(e, g);
    if (cm.u32buf) cm.u32buf[e] = 0;   // a new Generator: pcg64 has_uint32 = 0
}

__global__ void __launch_bounds__(256) period_fill_kernel(Common cm, int32_t t) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < cm.N) cm.period[e] = t;
}

// Episodic-return reduction of K steps of outputs (the statistics the
// reference's harness keeps per episode, benchmark_InvManagementBacklogEnv.py:
// 389-440): per env, ret += reward[k]; at a terminated|truncated step the return
// is folded into acc = [sum, sum of squares, episodes] and restarts at 0.  acc[3]
// sums every folded reward.  One lane per env walks its K rows (each row a
// coalesced 8-B / 1-B stream); the workgroup reduces in registers + LDS and
// adds its four partials to acc with vector f64 atomics.
__global__ void __launch_bounds__(256)
episode_fold_kernel(const double *rew, const uint8_t *term, const uint8_t *trunc, int32_t K, int64_t N,
                    double *ret, double *acc) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double s = 0.0, s2 = 0.0, c = 0.0, all = 0.0;
    if (e < N) {
        double r = ret[e];
        // rows in blocks of FB with every load of a block issued before the first
        // add: one memory latency per block instead of one per row
        constexpr int FB = 16;
        for (int k0 = 0; k0 < K; k0 += FB) {
            double x[FB];
            uint8_t d[FB];
#pragma unroll
            for (int u = 0; u < FB; ++u) {
                const int64_t i = (int64_t)min(k0 + u, K - 1) * N + e;
                // streamed once: non-temporal, so the env state stays cached for the next step launch
                x[u] = __builtin_nontemporal_load(rew + i);
                d[u] = (uint8_t)((term ? __builtin_nontemporal_load(term + i) : 0) |
                                 (trunc ? __builtin_nontemporal_load(trunc + i) : 0));
            }
#pragma unroll
            for (int u = 0; u < FB; ++u) {
                if (k0 + u < K) {
                    r += x[u];
                    all += x[u];
                    if (d[u]) {
                        s += r;
                        s2 += r * r;
                        c += 1.0;
                        r = 0.0;
                    }
                }
            }
        }
        ret[e] = r;
    }
    for (int off = 32; off > 0; off >>= 1) {
        s += __shfl_xor(s, off);
        s2 += __shfl_xor(s2, off);
        c += __shfl_xor(c, off);
        all += __shfl_xor(all, off);
    }
    __shared__ double part[4][4];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (l == 0) {
        part[w][0] = s;
        part[w][1] = s2;
        part[w][2] = c;
        part[w][3] = all;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        const int j = threadIdx.x;
        const double v = part[0][j] + part[1][j] + part[2][j] + part[3][j];
        atomicAdd(&acc[j], v);
    }
}

// The episode sink's fold (kernels.hpp EpLane / EpPart) of K output rows: one
// wave per 64-env group g, lane e walks its rows in step order (loads issued in
// blocks of FB, as above), then the wave's butterfly and lane 0's update of
// part[g].  The fused step / rollout kernels run the same per-lane code on the
// rows they produce, so both give the same ret and part bits.
__global__ void __launch_bounds__(256)
episode_fold_groups_kernel(const double *rew, const uint8_t *term, const uint8_t *trunc, int32_t K, int64_t N,
                           double *ret, double *part) {
    const int lane = threadIdx.x & 63;
    const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t e = g * 64 + lane;
    if (g * 64 >= N) return;                      // wave-uniform: a whole group past the batch
    EpPart pp;
    pp.load(part + 4 * g);
    EpLane a;
    bool any_done = false;
    if (e < N) {
        a.r = ret[e];
        constexpr int FB = 16;
        for (int k0 = 0; k0 < K; k0 += FB) {
            double x[FB];
            uint8_t d[FB];
#pragma unroll
            for (int u = 0; u < FB; ++u) {
                const int64_t i = (int64_t)min(k0 + u, K - 1) * N + e;
                x[u] = __builtin_nontemporal_load(rew + i);
                d[u] = (uint8_t)((term ? __builtin_nontemporal_load(term + i) : 0) |
                                 (trunc ? __builtin_nontemporal_load(trunc + i) : 0));
            }
#pragma unroll
            for (int u = 0; u < FB; ++u) {
                if (k0 + u < K) {
                    a.add(x[u], d[u] != 0);
                    any_done |= d[u] != 0;
                }
            }
        }
        ret[e] = a.r;
    }
    pp.flush(part + 4 * g, a, __ballot(any_done) != 0, lane);
}

static inline unsigned grid_for(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

hipError_t episode_fold_groups_launch(const double *rew, const uint8_t *term, const uint8_t *trunc, int32_t K,
                                      int64_t N, double *ret, double *part, hipStream_t s) {
    if (N == 0 || K == 0) return hipSuccess;
    hipLaunchKernelGGL(episode_fold_groups_kernel, dim3(grid_for(N, 256)), dim3(256), 0, s, rew, term, trunc, K, N,
                       ret, part);
    return hipGetLastError();
}

hipError_t episode_fold_launch(const double *rew, const uint8_t *term, const uint8_t *trunc, int32_t K,
                               int64_t N, double *ret, double *acc, hipStream_t s) {
    if (N == 0) return hipSuccess;
    hipLaunchKernelGGL(episode_fold_kernel, dim3(grid_for(N, 256)), dim3(256), 0, s, rew, term, trunc, K, N,
                       ret, acc);
    return hipGetLastError();
}

hipError_t seed_range_launch(const Common &cm, uint64_t base_lo, uint64_t base_hi, int64_t first,
                             const uint8_t *mask, hipStream_t s) {
    if (cm.N == 0) return hipSuccess;
    hipLaunchKernelGGL(seed_range_kernel, dim3(grid_for(cm.N, 256)), dim3(256), 0, s, cm, base_lo,
                       base_hi, first, mask);
    return hipGetLastError();
}

hipError_t seed_words_launch(const Common &cm, const uint32_t *words, const int32_t *nwords,
                             const uint8_t *mask, hipStream_t s) {
    if (cm.N == 0) return hipSuccess;
    hipLaunchKernelGGL(seed_words_kernel, dim3(grid_for(cm.N, 256)), dim3(256), 0, s, cm, words,
                       nwords, mask);
    return hipGetLastError();
}

hipError_t period_fill_launch(const Common &cm, int32_t t, hipStream_t s) {
    if (cm.N == 0) return hipSuccess;
    hipLaunchKernelGGL(period_fill_kernel, dim3(grid_for(cm.N, 256)), dim3(256), 0, s, cm, t);
    return hipGetLastError();
}

}  // namespace invsim
