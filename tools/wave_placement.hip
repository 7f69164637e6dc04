// Where the waves of multi-wave workgroups land (profiling aid): each wave
// records its hardware ids (s_getreg HW_ID: wave, SIMD, CU, SE; XCC_ID).
//   hipcc --offload-arch=gfx950 -O2 tools/wave_placement.hip -o tools/wave_placement
//   tools/wave_placement [waves_per_wg] [workgroups]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <set>
#include <vector>

__global__ void probe(unsigned *out, int spin) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    // keep every wave resident for a while so that the workgroups co-exist
    long long t0 = clock64();
    while (clock64() - t0 < spin) {
    }
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        out[2 * w] = hw;
        out[2 * w + 1] = xcc;
    }
}

int main(int argc, char **argv) {
    const int wpg = argc > 1 ? atoi(argv[1]) : 2;
    const int nwg = argc > 2 ? atoi(argv[2]) : 512;
    const int nw = wpg * nwg;
    unsigned *d;
    (void)hipMalloc(&d, sizeof(unsigned) * 2 * nw);
    hipLaunchKernelGGL(probe, dim3(nwg), dim3(64 * wpg), 0, 0, d, 2000000);
    (void)hipDeviceSynchronize();
    std::vector<unsigned> h(2 * nw);
    (void)hipMemcpy(h.data(), d, sizeof(unsigned) * 2 * nw, hipMemcpyDeviceToHost);
    // gfx9 HW_ID: wave[3:0] simd[5:4] cu[11:8] sh[12] se[15:13]
    int same_simd = 0, wgs_multi_simd = 0;
    std::map<long, int> simd_load;
    for (int g = 0; g < nwg; g++) {
        std::set<int> simds;
        for (int k = 0; k < wpg; k++) {
            const unsigned hw = h[2 * (g * wpg + k)], xcc = h[2 * (g * wpg + k) + 1] & 0xf;
            const int simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
            simds.insert(simd);
            simd_load[(((long)xcc * 8 + se) * 2 + sh) * 64 + cu * 4 + simd]++;
        }
        if ((int)simds.size() == 1 && wpg > 1) same_simd++;
        if ((int)simds.size() == wpg) wgs_multi_simd++;
    }
    int maxl = 0;
    for (auto &kv : simd_load) maxl = kv.second > maxl ? kv.second : maxl;
    std::map<long, int> cu_wgs;   // workgroups per CU (all waves of a workgroup share its CU)
    for (int g = 0; g < nwg; g++) {
        const unsigned hw = h[2 * (g * wpg)], xcc = h[2 * (g * wpg) + 1] & 0xf;
        const int cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
        cu_wgs[(((long)xcc * 8 + se) * 2 + sh) * 16 + cu]++;
    }
    std::map<int, int> hcu, hsimd;
    for (auto &kv : cu_wgs) hcu[kv.second]++;
    for (auto &kv : simd_load) hsimd[kv.second]++;
    printf("  CUs used=%zu; workgroups per CU histogram:", cu_wgs.size());
    for (auto &kv : hcu) printf(" %dx%d", kv.first, kv.second);
    printf("; waves per SIMD histogram:");
    for (auto &kv : hsimd) printf(" %dx%d", kv.first, kv.second);
    printf("\n");
    printf("waves/wg=%d wgs=%d: wgs with all waves on one SIMD=%d, on distinct SIMDs=%d; "
           "SIMDs used=%zu, max waves on a SIMD=%d\n",
           wpg, nwg, same_simd, wgs_multi_simd, simd_load.size(), maxl);
    // the SIMD pattern of a workgroup's waves, relative to its wave 0 ((simd_k - simd_0) mod 4)
    std::map<std::vector<int>, int> pat;
    for (int g = 0; g < nwg; g++) {
        std::vector<int> v;
        const int s0 = (h[2 * (g * wpg)] >> 4) & 3;
        for (int k = 0; k < wpg; k++) v.push_back((((h[2 * (g * wpg + k)] >> 4) & 3) - s0 + 4) & 3);
        pat[v]++;
    }
    printf("  wave -> SIMD patterns (relative to wave 0):");
    for (auto &kv : pat) {
        printf(" [");
        for (int x : kv.first) printf("%d", x);
        printf("]x%d", kv.second);
    }
    printf("\n");
    // per CU: how many waves of role k (wave index k mod roles) share a SIMD with another of the same role
    const int roles = argc > 3 ? atoi(argv[3]) : wpg;
    std::map<long, int> role_simd;   // (cu-simd, role) -> count
    for (int g = 0; g < nwg; g++)
        for (int k = 0; k < wpg; k++) {
            const unsigned hw = h[2 * (g * wpg + k)], xcc = h[2 * (g * wpg + k) + 1] & 0xf;
            const int simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
            role_simd[((((long)xcc * 8 + se) * 2 + sh) * 64 + cu * 4 + simd) * 16 + (k % roles)]++;
        }
    std::map<int, std::map<int, int>> rh;   // role -> (waves of that role on one SIMD -> SIMDs)
    for (auto &kv : role_simd) rh[(int)(kv.first % 16)][kv.second]++;
    for (auto &r : rh) {
        printf("  role %d: SIMDs holding n waves of it:", r.first);
        for (auto &kv : r.second) printf(" %dx%d", kv.first, kv.second);
        printf("\n");
    }
    return 0;
}
