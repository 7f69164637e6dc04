// VALU issue cost per wave-instruction on gfx950 for the ops the PTRS / PCG64
// draw chain is made of (profiling aid for the issue-cycle floor of the stream
// waves).  One kernel per op: every SIMD runs W waves (W = 1: the
// op's issue interval for one wave with 8 independent chains; W = 4: the SIMD's
// throughput), each wave a loop of 8 independent instances per iteration;
// s_memtime (shader clock) around the loop, lane 0 of each wave.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rates.hip -o tools/valu_rates && tools/valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int ITERS = 2048;

#define OP8(ASM)                                                                                       \
    asm volatile(ASM : "+v"(x0) : "v"(y) : "vcc"); asm volatile(ASM : "+v"(x1) : "v"(y) : "vcc");      \
    asm volatile(ASM : "+v"(x2) : "v"(y) : "vcc"); asm volatile(ASM : "+v"(x3) : "v"(y) : "vcc");      \
    asm volatile(ASM : "+v"(x4) : "v"(y) : "vcc"); asm volatile(ASM : "+v"(x5) : "v"(y) : "vcc");      \
    asm volatile(ASM : "+v"(x6) : "v"(y) : "vcc"); asm volatile(ASM : "+v"(x7) : "v"(y) : "vcc");

#define KERNEL(NAME, T, TY, ASM)                                                                       \
    __global__ void NAME(unsigned long long *cyc, T *sink, T seed) {                                   \
        T x0 = seed, x1 = seed + 1, x2 = seed + 2, x3 = seed + 3, x4 = seed + 4, x5 = seed + 5,        \
          x6 = seed + 6, x7 = seed + 7;                                                                \
        TY y = (TY)seed + (TY)threadIdx.x;                                                             \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                                    \
        for (int i = 0; i < ITERS; i++) {                                                              \
            OP8(ASM)                                                                                   \
        }                                                                                              \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                                    \
        if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0; \
        sink[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;           \
    }

KERNEL(k_mad_u64_u32, unsigned long long, unsigned int, "v_mad_u64_u32 %0, vcc, %1, %1, %0")
KERNEL(k_mul_lo_u32, unsigned int, unsigned int, "v_mul_lo_u32 %0, %0, %1")
KERNEL(k_mul_hi_u32, unsigned int, unsigned int, "v_mul_hi_u32 %0, %0, %1")
KERNEL(k_add_u32, unsigned int, unsigned int, "v_add_u32 %0, %0, %1")
KERNEL(k_lshl_add_u64, unsigned long long, unsigned long long, "v_lshl_add_u64 %0, %0, 0, %1")
KERNEL(k_fma_f64, double, double, "v_fma_f64 %0, %0, %1, %1")
KERNEL(k_add_f64, double, double, "v_add_f64 %0, %0, %1")
KERNEL(k_mul_f64, double, double, "v_mul_f64 %0, %0, %1")
KERNEL(k_rcp_f64, double, double, "v_rcp_f64 %0, %0")
KERNEL(k_fma_f32, float, float, "v_fma_f32 %0, %0, %1, %1")
KERNEL(k_log_f32, float, float, "v_log_f32 %0, %0")

struct Op {
    const char *name;
    void (*k64)(unsigned long long *, unsigned long long *, unsigned long long);
    void (*k32)(unsigned long long *, unsigned int *, unsigned int);
    void (*kd)(unsigned long long *, double *, double);
    void (*kf)(unsigned long long *, float *, float);
};

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const Op ops[] = {{"v_mad_u64_u32", k_mad_u64_u32, nullptr, nullptr, nullptr},
                      {"v_mul_lo_u32", nullptr, k_mul_lo_u32, nullptr, nullptr},
                      {"v_mul_hi_u32", nullptr, k_mul_hi_u32, nullptr, nullptr},
                      {"v_add_u32", nullptr, k_add_u32, nullptr, nullptr},
                      {"v_lshl_add_u64", k_lshl_add_u64, nullptr, nullptr, nullptr},
                      {"v_fma_f64", nullptr, nullptr, k_fma_f64, nullptr},
                      {"v_add_f64", nullptr, nullptr, k_add_f64, nullptr},
                      {"v_mul_f64", nullptr, nullptr, k_mul_f64, nullptr},
                      {"v_rcp_f64", nullptr, nullptr, k_rcp_f64, nullptr},
                      {"v_fma_f32", nullptr, nullptr, nullptr, k_fma_f32},
                      {"v_log_f32", nullptr, nullptr, nullptr, k_log_f32}};
    unsigned long long *cyc;
    void *sink;
    const int maxw = cus * 4 * 4;
    hipMalloc(&cyc, maxw * sizeof(unsigned long long));
    hipMalloc(&sink, (size_t)maxw * 64 * 8);
    std::vector<unsigned long long> h(maxw);
    printf("cycles per wave-instruction (s_memtime), %d CUs; W = waves per SIMD\n", cus);
    for (const Op &op : ops) {
        for (int W : {1, 2, 4}) {
            const dim3 grid(cus), block(64 * 4 * W);   // one workgroup per CU: W waves on each of 4 SIMDs
            for (int rep = 0; rep < 2; rep++) {
                if (op.k64) hipLaunchKernelGGL(op.k64, grid, block, 0, 0, cyc, (unsigned long long *)sink, 3ull);
                if (op.k32) hipLaunchKernelGGL(op.k32, grid, block, 0, 0, cyc, (unsigned int *)sink, 3u);
                if (op.kd) hipLaunchKernelGGL(op.kd, grid, block, 0, 0, cyc, (double *)sink, 1.0000001);
                if (op.kf) hipLaunchKernelGGL(op.kf, grid, block, 0, 0, cyc, (float *)sink, 1.0001f);
            }
            hipDeviceSynchronize();
            const int nw = cus * 4 * W;
            hipMemcpy(h.data(), cyc, nw * sizeof(unsigned long long), hipMemcpyDeviceToHost);
            double s = 0;
            for (int i = 0; i < nw; i++) s += (double)h[i];
            const double per_wave = s / nw / (ITERS * 8.0);          // cycles per instruction, one wave's view
            printf("%-16s W=%d  %6.2f cycles/instr per wave  -> SIMD issue interval %6.2f cycles\n", op.name, W,
                   per_wave, per_wave / W);
        }
    }
    return 0;
}
