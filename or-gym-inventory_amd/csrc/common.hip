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

static inline unsigned grid_for(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

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
