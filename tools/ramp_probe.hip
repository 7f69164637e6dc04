// Dispatch ramp of a launch (profiling aid): every wave records
// s_memrealtime (100 MHz) at entry; the spread of the entries over the grid is
// how long the dispatcher takes to start it.  Workgroups, waves per workgroup,
// LDS and VGPRs are varied to see which one the ramp follows.
//   hipcc --offload-arch=gfx950 -O2 tools/ramp_probe.hip -o tools/ramp_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

template <int NW, int BIGV>
__global__ void __launch_bounds__(64 * NW) probe(unsigned long long *out, int spin) {
    extern __shared__ int lds[];
    if (BIGV) asm volatile("v_mov_b32 v127, 0" ::: "v127");   // 128 VGPRs per wave
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * NW + threadIdx.x / 64] = t;
    lds[threadIdx.x] = (int)t;
    long long t0 = clock64();
    while (clock64() - t0 < spin) {
    }
    if (lds[(threadIdx.x + 1) % (64 * NW)] == 12345) out[0] = 0;
}

template <int NW, int BIGV>
static void run(int wgs, int lds_kb, int spin, const char *what) {
    unsigned long long *d;
    const int nw = wgs * NW;
    (void)hipMalloc(&d, sizeof(unsigned long long) * nw);
    std::vector<unsigned long long> h(nw);
    double best = 1e30, p50s = 0;
    for (int rep = 0; rep < 11; rep++) {
        hipLaunchKernelGGL((probe<NW, BIGV>), dim3(wgs), dim3(64 * NW), lds_kb * 1024, 0, d, spin);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(h.data(), d, sizeof(unsigned long long) * nw, hipMemcpyDeviceToHost);
        std::sort(h.begin(), h.end());
        const double span = (h[nw - 1] - h[0]) * 10.0, p50 = (h[nw / 2] - h[0]) * 10.0;
        if (span < best) {
            best = span;
            p50s = p50;
        }
    }
    printf("%-34s wgs=%5d waves/wg=%d lds=%2dKB vgpr=%s spin=%d: entry spread %6.0f ns (p50 %5.0f)\n", what, wgs, NW,
           lds_kb, BIGV ? "128" : "low", spin, best, p50s);
    (void)hipFree(d);
}

int main() {
    const int S = 20000;   // ~8 us of residency: every workgroup is resident at once
    for (int round = 0; round < 2; round++) {
        printf("-- round %d\n", round);
        run<2, 1>(1536, 19, S, "InvMgmt step shape (65536 envs)");
        run<4, 1>(768, 38, S, "4-wave workgroups, same waves");
        run<1, 1>(3072, 10, S, "1-wave workgroups, same waves");
        run<2, 1>(1024, 19, S, "step workgroups only");
        run<4, 1>(512, 38, S, "4-wave workgroups, 2048 waves");
        run<2, 1>(768, 19, S, "32768-env step shape");
        run<4, 1>(384, 38, S, "32768-env shape, 4-wave workgroups");
        run<2, 0>(1536, 19, S, "low VGPR");
        run<2, 1>(1536, 0, S, "no LDS");
        run<2, 1>(1536, 19, 0, "no spin");
        run<4, 1>(768, 38, 0, "4-wave, no spin");
        run<6, 1>(512, 57, S, "6-wave workgroups, same waves");
    }
    return 0;
}
