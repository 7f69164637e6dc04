// Device time of back-to-back empty launches against grid and block size
// (profiling aid): how much of a short step kernel is workgroup dispatch.
// Eager launches (one host call each) and, with "graph", the same 2 000
// launches captured into one HIP graph and replayed (one host call), which
// takes host submission out of the timing.
//   hipcc --offload-arch=gfx950 -O2 tools/dispatch_cost.hip -o tools/dispatch_cost
//   tools/dispatch_cost [quick|graph]
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty(int *p) {
    if (p && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) p[0] = 1;
}

int main(int argc, char **argv) {
    const bool quick = argc > 1 && argv[1][0] == 'q';   // one line: block 128, grid 768
    const bool graph = argc > 1 && argv[1][0] == 'g';
    hipStream_t s;
    (void)hipStreamCreate(&s);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int reps = 2000;
    for (int i = 0; i < 200; i++) hipLaunchKernelGGL(k_empty, dim3(1024), dim3(64), 0, s, nullptr);
    (void)hipStreamSynchronize(s);
    const int grids[] = {1, 64, 256, 384, 512, 768, 1024, 1536, 2048, 4096};
    const int blocks[] = {64, 128, 192, 256};
    for (int bs : blocks) {
        if (quick && bs != 128) continue;
        for (int g : grids) {
            if (quick && g != 768) continue;
            float best = 1e30f, bestg = 1e30f;
            for (int t = 0; t < 3; t++) {
                (void)hipEventRecord(a, s);
                for (int i = 0; i < reps; i++) hipLaunchKernelGGL(k_empty, dim3(g), dim3(bs), 0, s, nullptr);
                (void)hipEventRecord(b, s);
                (void)hipEventSynchronize(b);
                float ms = 0;
                (void)hipEventElapsedTime(&ms, a, b);
                best = ms < best ? ms : best;
            }
            if (graph) {
                hipGraph_t gr;
                hipGraphExec_t ge;
                (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
                for (int i = 0; i < reps; i++) hipLaunchKernelGGL(k_empty, dim3(g), dim3(bs), 0, s, nullptr);
                (void)hipStreamEndCapture(s, &gr);
                (void)hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0);
                (void)hipGraphLaunch(ge, s);
                (void)hipStreamSynchronize(s);
                for (int t = 0; t < 3; t++) {
                    (void)hipEventRecord(a, s);
                    (void)hipGraphLaunch(ge, s);
                    (void)hipEventRecord(b, s);
                    (void)hipEventSynchronize(b);
                    float ms = 0;
                    (void)hipEventElapsedTime(&ms, a, b);
                    bestg = ms < bestg ? ms : bestg;
                }
                (void)hipGraphExecDestroy(ge);
                (void)hipGraphDestroy(gr);
                printf("block %3d grid %5d: eager %.3f us/launch  graph replay %.3f us/launch\n", bs, g,
                       best * 1e3f / reps, bestg * 1e3f / reps);
            } else {
                printf("block %3d grid %5d: %.3f us/launch\n", bs, g, best * 1e3f / reps);
            }
        }
    }
    return 0;
}
