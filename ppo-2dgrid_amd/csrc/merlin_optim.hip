// merlin_optim.hip -- the optimizer step of PPO.update (src/ppo.py:153-156):
//   clip_grad_norm_(params, max_norm)  then  Adam.step()
// in two launches over all parameter tensors at once (torch's chain is ~10 launches: foreach
// norm + its cleanup, stack, vector_norm, coefficient, clamp, foreach mul, step-count add,
// fused Adam).  The tensors are passed by value in the kernel arguments (pointer lists, at most
// OPT_MAX_TENSORS), each cut into OPT_CHUNK-element blocks.
//   k_opt_sumsq   per block: sum of squared gradients (f64 partial); the first block of a tensor
//                 advances its Adam step counter (f32, torch's on-device `step` state).
//   k_opt_adam    per block: the global norm from the partials (every block sums the same
//                 partials in the same order, so all agree bit for bit), the clip coefficient
//                 min(max_norm / (norm + 1e-6), 1) applied to the gradient (written back, as
//                 clip_grad_norm_ does), then torch's fused-Adam arithmetic on (p, m, v).
// Bytes per parameter: 4 (grad, pass 1) + 16 read + 16 written (pass 2).
#include "merlin_internal.h"

namespace merlin {
namespace {

constexpr int OPT_BLK = 256;
constexpr int OPT_PER_THREAD = 4;  // ~730 blocks for the 745k parameters: fills the chip
constexpr int OPT_CHUNK = OPT_BLK * OPT_PER_THREAD;

struct OptList {
    int n;
    int blk0[OPT_MAX_TENSORS + 1];  // first block of tensor i; blk0[n] = total blocks
    int64_t numel[OPT_MAX_TENSORS];
    float *p[OPT_MAX_TENSORS];
    float *g[OPT_MAX_TENSORS];
    float *m[OPT_MAX_TENSORS];
    float *v[OPT_MAX_TENSORS];
    float *step[OPT_MAX_TENSORS];
};

__device__ __forceinline__ int tensor_of(const OptList &L, int b) {
    int i = 0;
    while (i + 1 < L.n && L.blk0[i + 1] <= b) i++;
    return i;
}

__device__ double block_sum(double x, double *red) {
    const int t = threadIdx.x;
    for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o, 64);
    if ((t & 63) == 0) red[t >> 6] = x;
    __syncthreads();
    double s = 0.0;
    if (t == 0)
        for (int w = 0; w < OPT_BLK / 64; w++) s += red[w];
    return s;  // valid in thread 0
}

__global__ __launch_bounds__(OPT_BLK) void k_opt_sumsq(OptList L, double *partial) {
    __shared__ double red[OPT_BLK / 64];
    const int b = blockIdx.x, i = tensor_of(L, b);
    const int64_t base = (int64_t)(b - L.blk0[i]) * OPT_CHUNK, n = L.numel[i];
    const float *g = L.g[i];
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < OPT_PER_THREAD; k++) {
        const int64_t e = base + k * OPT_BLK + threadIdx.x;
        if (e < n) {
            const float x = g[e];
            acc += x * x;
        }
    }
    const double s = block_sum((double)acc, red);
    if (threadIdx.x == 0) {
        partial[b] = s;
        if (b == L.blk0[i] && L.step[i]) L.step[i][0] += 1.0f;
    }
}

__global__ __launch_bounds__(OPT_BLK) void k_opt_adam(OptList L, const double *partial, int nblk, double lr, double beta1,
                                                     double beta2, double eps, float max_norm, float *norm_out) {
    __shared__ double red[OPT_BLK / 64];
    __shared__ float coef_s;
    double x = 0.0;
    for (int j = threadIdx.x; j < nblk; j += OPT_BLK) x += partial[j];
    const double tot = block_sum(x, red);
    if (threadIdx.x == 0) {
        const float norm = (float)sqrt(tot);
        float c = max_norm / (norm + 1e-6f);
        // torch.clamp(max=1) keeps a NaN coefficient (non-finite norm): every gradient and
        // parameter then turns NaN, as with clip_grad_norm_, instead of a partly hidden step
        coef_s = (c != c) ? c : (c < 1.0f ? c : 1.0f);
        if (blockIdx.x == 0 && norm_out) norm_out[0] = norm;
    }
    __syncthreads();
    const float coef = coef_s;
    const int b = blockIdx.x, i = tensor_of(L, b);
    const int64_t base = (int64_t)(b - L.blk0[i]) * OPT_CHUNK, n = L.numel[i];
    // torch fused Adam (ATen fused_adam_utils.cuh adam_math, no weight decay / amsgrad / maximize):
    // lr, beta1, beta2, eps are doubles there, so the moment updates and the bias corrections are
    // evaluated in double and rounded to fp32 once, step_size / denom / the parameter in fp32
    const double stepc = (double)L.step[i][0];
    const float bc1 = (float)(1.0 - pow(beta1, stepc));
    const float bc2_sqrt = (float)sqrt(1.0 - pow(beta2, stepc));
    const float step_size = (float)(lr / (double)bc1);
    float *__restrict__ p = L.p[i];
    float *__restrict__ g = L.g[i];
    float *__restrict__ m = L.m[i];
    float *__restrict__ v = L.v[i];
    float rg[OPT_PER_THREAD], rm[OPT_PER_THREAD], rv[OPT_PER_THREAD], rp[OPT_PER_THREAD];
#pragma unroll
    for (int k = 0; k < OPT_PER_THREAD; k++) {  // all loads in flight before the arithmetic
        const int64_t e = base + k * OPT_BLK + threadIdx.x;
        if (e < n) {
            rg[k] = g[e];
            rm[k] = m[e];
            rv[k] = v[e];
            rp[k] = p[e];
        }
    }
#pragma unroll
    for (int k = 0; k < OPT_PER_THREAD; k++) {
        const int64_t e = base + k * OPT_BLK + threadIdx.x;
        if (e < n) {
            const float gr = rg[k] * coef;
            const float ma = (float)(beta1 * (double)rm[k] + (1.0 - beta1) * (double)gr);
            const float va = (float)(beta2 * (double)rv[k] + (1.0 - beta2) * (double)gr * (double)gr);
            const float denom = (float)((double)(sqrtf(va) / bc2_sqrt) + eps);
            g[e] = gr;
            m[e] = ma;
            v[e] = va;
            p[e] = rp[k] - step_size * ma / denom;
        }
    }
}

}  // namespace

int64_t opt_blocks(int n, const int64_t *numel) {
    int64_t b = 0;
    for (int i = 0; i < n; i++) b += (numel[i] + OPT_CHUNK - 1) / OPT_CHUNK;
    return b;
}

hipError_t launch_clip_adam(int n, float *const *params, float *const *grads, float *const *exp_avg,
                            float *const *exp_avg_sq, float *const *steps, const int64_t *numel, double lr, double beta1,
                            double beta2, double eps, float max_norm, float *norm_out, double *partial, hipStream_t s) {
    OptList L{};
    L.n = n;
    int blocks = 0;
    for (int i = 0; i < n; i++) {
        L.blk0[i] = blocks;
        L.numel[i] = numel[i];
        L.p[i] = params[i];
        L.g[i] = grads[i];
        L.m[i] = exp_avg[i];
        L.v[i] = exp_avg_sq[i];
        L.step[i] = steps[i];
        blocks += (int)((numel[i] + OPT_CHUNK - 1) / OPT_CHUNK);
    }
    L.blk0[n] = blocks;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_opt_sumsq, dim3((unsigned)blocks), dim3(OPT_BLK), 0, s, L, partial);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_opt_adam, dim3((unsigned)blocks), dim3(OPT_BLK), 0, s, L, (const double *)partial, blocks, lr,
                       beta1, beta2, eps, max_norm, norm_out);
    return hipGetLastError();
}

}  // namespace merlin
