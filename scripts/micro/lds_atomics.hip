// Microbenchmark: LDS float atomic add vs int atomic add vs plain read-modify-write,
// distinct addresses per lane (no conflicts).  One block per CU, 16 waves.
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITERS 4096
template <int MODE>
__global__ __launch_bounds__(1024) void k(float *out, int salt) {
    __shared__ float tab[16 * 1024];
    for (int i = threadIdx.x; i < 16 * 1024; i += 1024) tab[i] = 0.f;
    __syncthreads();
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float *mine = tab + wv * 1024;  // wave-private region (for the plain RMW mode)
    float g = 1.0f + lane * 1e-3f;
    for (int it = 0; it < ITERS; it++) {
        const int row = ((it * 7 + salt) & 15);  // uniform row, 64 distinct lanes
        if (MODE == 0) atomicAdd(&tab[(wv * 16 + row) * 64 + lane], g);
        else if (MODE == 1) atomicAdd(reinterpret_cast<unsigned *>(&tab[(wv * 16 + row) * 64 + lane]), 1u);
        else if (MODE == 2) { float *p = &mine[row * 64 + lane]; *p = *p + g; }
        else if (MODE == 3) { // 8 lanes same address (8 groups), float atomics
            atomicAdd(&tab[(wv * 16 + row) * 64 + (lane & 7)], g);
        }
    }
    __syncthreads();
    float s = 0;
    for (int i = threadIdx.x; i < 16 * 1024; i += 1024) s += tab[i];
    out[blockIdx.x * 1024 + threadIdx.x] = s;
}
int main() {
    float *out; hipMalloc(&out, 256 * 1024 * 4 * 4);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const char *names[] = {"ds_add_f32 distinct", "ds_add_u32 distinct", "plain RMW wave-private", "ds_add_f32 8-way same addr"};
    for (int m = 0; m < 4; m++) {
        for (int rep = 0; rep < 2; rep++) {
            hipEventRecord(a);
            if (m == 0) hipLaunchKernelGGL(k<0>, dim3(256), dim3(1024), 0, 0, out, rep);
            if (m == 1) hipLaunchKernelGGL(k<1>, dim3(256), dim3(1024), 0, 0, out, rep);
            if (m == 2) hipLaunchKernelGGL(k<2>, dim3(256), dim3(1024), 0, 0, out, rep);
            if (m == 3) hipLaunchKernelGGL(k<3>, dim3(256), dim3(1024), 0, 0, out, rep);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            double instr_per_cu = 16.0 * ITERS;
            if (rep) printf("%-28s %.3f ms  %.1f cycles per wave-instr per CU (2.4GHz)\n", names[m], ms, ms * 1e-3 * 2.4e9 / instr_per_cu);
        }
    }
    return 0;
}
