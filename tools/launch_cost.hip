// Host cost of a kernel launch on this ROCm stack (tools/launch_cost.py splits
// the invsim_step call; this isolates hipLaunchKernelGGL itself).
//   hipcc --offload-arch=gfx950 -O2 tools/launch_cost.hip -o tools/launch_cost
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <algorithm>
#include <vector>

struct Big { char b[704]; };

__global__ void k_small(int *p) { if (p && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) p[0] = 1; }
__global__ void k_big(Big a, int *p) { if (p && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) p[0] = a.b[0]; }

template <class F>
static double host_us(F f, int reps) {
    std::vector<double> v;
    for (int t = 0; t < 21; t++) {
        (void)hipDeviceSynchronize();
        auto a = std::chrono::steady_clock::now();
        for (int i = 0; i < reps; i++) f();
        auto b = std::chrono::steady_clock::now();
        v.push_back(std::chrono::duration<double, std::micro>(b - a).count() / reps);
    }
    (void)hipDeviceSynchronize();
    std::sort(v.begin(), v.end());
    return v[10];
}

int main() {
    hipStream_t s;
    (void)hipStreamCreate(&s);
    Big big{};
    for (int i = 0; i < 100; i++) hipLaunchKernelGGL(k_small, dim3(1024), dim3(64), 0, s, nullptr);
    (void)hipDeviceSynchronize();
    for (int grid : {1, 1024, 2048}) {
        printf("small args grid %5d: %.2f us/launch (host)\n", grid,
               host_us([&] { hipLaunchKernelGGL(k_small, dim3(grid), dim3(64), 0, s, nullptr); }, 10));
        printf("704-B args grid %5d: %.2f us/launch (host)\n", grid,
               host_us([&] { hipLaunchKernelGGL(k_big, dim3(grid), dim3(128), 4096, s, big, nullptr); }, 10));
    }
    int dev = 0;
    printf("hipGetDevice: %.3f us\n", host_us([&] { (void)hipGetDevice(&dev); }, 1000));
    printf("hipGetLastError: %.3f us\n", host_us([&] { (void)hipGetLastError(); }, 1000));
    // launch + wait: first launch after idle to completion seen by the host
    std::vector<double> v;
    for (int t = 0; t < 41; t++) {
        (void)hipDeviceSynchronize();
        auto a = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(k_small, dim3(1024), dim3(64), 0, s, nullptr);
        (void)hipStreamSynchronize(s);
        auto b = std::chrono::steady_clock::now();
        v.push_back(std::chrono::duration<double, std::micro>(b - a).count());
    }
    std::sort(v.begin(), v.end());
    printf("idle launch -> stream sync return: p10 %.2f med %.2f us\n", v[4], v[20]);
    return 0;
}
