// merlin_stage.hip -- the parameter-only part of PPO.update's minibatch step (merlin/fast_step.py WeightStage):
// the conv1 / conv2 tables T2 of both towers from the stacked weights, and their adjoint down to the conv1 /
// conv2 weight and bias gradients, in two launches each way instead of the ~10 + ~14 small torch kernels of
// CNNActorCritic.conv2_tables_from + its autograd backward (src/actor_critic.py:9-14 conv1, conv2).
//
//   P[t][o][slot][bin]  = sum_{c, k, l} W1[t][o][c][4 dy + k][4 dx + l] * A[z][c][4 qy + k][4 qx + l]
//                         (slot = 2 dy + dx, bin = 4 z + 2 qy + qx: conv1 of atlas tile z at sub-offset (qy, qx)
//                         seen through kernel quadrant (dy, dx); A = the /255-scaled tile atlas)
//   HT[t][v][o]         = relu(b1[t][o] + sum_{e < 4} P[t][o][idx[v][e]])   conv1 of tile combination v
//   T2[t][4 v + j][co]  = sum_o HT[t][v][o] * W2[t][co][o][2 a + yp][2 b + xp]   (j = 2 a + b, (yp, xp) = v's
//                         parity type; csrc/merlin_conv2lut.hip's table layout)
// Backward from dT2: dH = [HT > 0] * (dT2 . W2), dW2 = sum over the type's combinations of HT x dT2, db1 = sum_v dH,
// dP[o][k] = sum over the (v, e) with idx[v][e] = k of dH[v][o], dW1 = dP contracted with the atlas.  Every sum
// runs in a fixed order: the same bits every call.
#include "merlin_internal.h"

namespace merlin {
namespace {

constexpr int C1 = 32, C2 = 64, NV = 680, NROW = 4 * NV;  // conv1 / conv2 channels, combinations, T2 rows
constexpr int VB = 8;                                    // combinations per block of the forward / dH kernels
// combinations of parity types ee, eo, oe, oo: v in [off[p], off[p + 1])
__device__ __forceinline__ int part_of(int v) { return v < 5 ? 0 : v < 30 ? 1 : v < 55 ? 2 : 3; }
__device__ __forceinline__ int part_off(int p) { return p == 0 ? 0 : p == 1 ? 5 : p == 2 ? 30 : 55; }

// P[o][k] (k = slot * 20 + bin) of one tower into LDS: 2,560 values, 48 products each
__device__ void conv1_tables(const float *__restrict__ W1, const float *__restrict__ atlas, float *__restrict__ P) {
    for (int q = threadIdx.x; q < C1 * 80; q += blockDim.x) {
        const int o = q / 80, k = q - o * 80;
        const int slot = k / 20, bin = k - slot * 20;
        const int dy = slot >> 1, dx = slot & 1, z = bin >> 2, qy = (bin >> 1) & 1, qx = bin & 1;
        float acc = 0.0f;
        for (int c = 0; c < 3; c++)
            for (int kk = 0; kk < 4; kk++)
                for (int l = 0; l < 4; l++)
                    acc += W1[((o * 3 + c) * 8 + 4 * dy + kk) * 8 + 4 * dx + l] *
                           atlas[((z * 3 + c) * 8 + 4 * qy + kk) * 8 + 4 * qx + l];
        P[q] = acc;
    }
}

// grid (NV / VB, T): HT rows v0 .. v0 + VB and their T2 rows; HT saved for the backward
__global__ __launch_bounds__(256) void k_stage_fwd(const float *__restrict__ W1, const float *__restrict__ b1,
                                                   const float *__restrict__ W2, const float *__restrict__ atlas,
                                                   const int16_t *__restrict__ idx, float *__restrict__ HT,
                                                   float *__restrict__ T2) {
    __shared__ float P[C1 * 80];
    __shared__ float H[VB][C1];
    const int t = blockIdx.y, v0 = blockIdx.x * VB;
    W1 += (size_t)t * C1 * 3 * 64;
    b1 += t * C1;
    W2 += (size_t)t * C2 * C1 * 16;
    conv1_tables(W1, atlas, P);
    __syncthreads();
    {
        const int vl = threadIdx.x / C1, o = threadIdx.x - vl * C1;  // VB * C1 == 256
        const int v = v0 + vl;
        float s = b1[o];
        for (int e = 0; e < 4; e++) s += P[o * 80 + idx[v * 4 + e]];
        s = s != s ? s : fmaxf(s, 0.0f);
        H[vl][o] = s;
        HT[((size_t)t * NV + v) * C1 + o] = s;
    }
    __syncthreads();
    // T2 rows 4 v + j, v in the block: VB * 4 * 64 = 2048 outputs, 8 per thread
    for (int q = threadIdx.x; q < VB * 4 * C2; q += 256) {
        const int vl = q / (4 * C2), r = q - vl * 4 * C2, j = r / C2, co = r - j * C2;
        const int v = v0 + vl, p = part_of(v), yp = p >> 1, xp = p & 1, a = j >> 1, b = j & 1;
        const float *w = W2 + (size_t)co * C1 * 16 + (2 * a + yp) * 4 + 2 * b + xp;
        float acc = 0.0f;
        for (int o = 0; o < C1; o++) acc += H[vl][o] * w[o * 16];
        T2[((size_t)t * NROW + 4 * v + j) * C2 + co] = acc;
    }
}

// grid (NV / VB, T): dH[t][v][o] = [HT > 0] * sum_{j, co} dT2[4 v + j][co] * W2[co][o][tap(v, j)]
__global__ __launch_bounds__(256) void k_stage_bwd_h(const float *__restrict__ W2, const float *__restrict__ HT,
                                                     const float *__restrict__ dT2, float *__restrict__ dH) {
    __shared__ float G[VB][4 * C2];
    const int t = blockIdx.y, v0 = blockIdx.x * VB;
    W2 += (size_t)t * C2 * C1 * 16;
    for (int q = threadIdx.x; q < VB * 4 * C2; q += 256)
        G[q / (4 * C2)][q % (4 * C2)] = dT2[((size_t)t * NROW + 4 * v0) * C2 + q];
    __syncthreads();
    const int vl = threadIdx.x / C1, o = threadIdx.x - vl * C1;
    const int v = v0 + vl, p = part_of(v), yp = p >> 1, xp = p & 1;
    float acc = 0.0f;
    for (int j = 0; j < 4; j++) {
        const int tap = (2 * (j >> 1) + yp) * 4 + 2 * (j & 1) + xp;
        for (int co = 0; co < C2; co++) acc += G[vl][j * C2 + co] * W2[((size_t)co * C1 + o) * 16 + tap];
    }
    const size_t hi = ((size_t)t * NV + v) * C1 + o;
    dH[hi] = HT[hi] > 0.0f ? acc : 0.0f;
}

// blocks [0, T * 128): dW2, 256 outputs each (t, co, o, tap): sum over the combinations of the tap's parity type
// of HT[v][o] * dT2[4 v + j][co];  blocks [T * 128, T * 128 + T * C1): tower t, conv1 channel o: db1[o] =
// sum_v dH[v][o], dP[o][k] for the 80 k (combinations in v order, through the CSR kinv), then dW1[o][c][ky][kx]
__global__ __launch_bounds__(256) void k_stage_bwd_w(const float *__restrict__ HT, const float *__restrict__ dT2,
                                                     const float *__restrict__ dH, const float *__restrict__ atlas,
                                                     const int16_t *__restrict__ koff, const int16_t *__restrict__ kv,
                                                     int T, float *__restrict__ dW1, float *__restrict__ db1,
                                                     float *__restrict__ dW2) {
    const int nb2 = T * (C2 * C1 * 16 / 256);
    if ((int)blockIdx.x < nb2) {
        const int q = blockIdx.x * 256 + threadIdx.x;  // (t, co, o, tap) in dW2's layout
        const int t = q / (C2 * C1 * 16), r = q - t * (C2 * C1 * 16);
        const int co = r / (C1 * 16), o = (r / 16) % C1, tap = r % 16, ky = tap >> 2, kx = tap & 3;
        const int p = 2 * (ky & 1) + (kx & 1), j = 2 * (ky >> 1) + (kx >> 1);
        const int va = part_off(p), vb = p == 3 ? NV : part_off(p + 1);
        const float *h = HT + (size_t)t * NV * C1 + o;
        const float *g = dT2 + (size_t)t * NROW * C2 + j * C2 + co;
        float acc = 0.0f;
        for (int v = va; v < vb; v++) acc += h[(size_t)v * C1] * g[(size_t)v * 4 * C2];
        dW2[q] = acc;
        return;
    }
    __shared__ float dP[80];
    const int b = blockIdx.x - nb2, t = b / C1, o = b - t * C1;
    const float *d = dH + (size_t)t * NV * C1 + o;
    if (threadIdx.x < 80) {  // dP[o][k]: the (v, e) entries with idx[v][e] = k, in (v, e) order
        const int k = threadIdx.x;
        float acc = 0.0f;
        for (int i = koff[k]; i < koff[k + 1]; i++) acc += d[(size_t)kv[i] * C1];
        dP[k] = acc;
    } else if (threadIdx.x == 128) {
        float acc = 0.0f;
        for (int v = 0; v < NV; v++) acc += d[(size_t)v * C1];
        db1[t * C1 + o] = acc;
    }
    __syncthreads();
    for (int q = threadIdx.x; q < 3 * 64; q += 256) {  // dW1[t][o][c][ky][kx]
        const int c = q >> 6, ky = (q >> 3) & 7, kx = q & 7;
        const int dy = ky >> 2, kk = ky & 3, dx = kx >> 2, l = kx & 3, slot = 2 * dy + dx;
        float acc = 0.0f;
        for (int bin = 0; bin < 20; bin++) {
            const int z = bin >> 2, qy = (bin >> 1) & 1, qx = bin & 1;
            acc += dP[slot * 20 + bin] * atlas[((z * 3 + c) * 8 + 4 * qy + kk) * 8 + 4 * qx + l];
        }
        dW1[(((size_t)t * C1 + o) * 3 + c) * 64 + ky * 8 + kx] = acc;
    }
}

}  // namespace

hipError_t launch_stage_fwd(const float *W1, const float *b1, const float *W2, const float *atlas, const int16_t *idx,
                            int T, float *HT, float *T2, hipStream_t s) {
    hipLaunchKernelGGL(k_stage_fwd, dim3(NV / VB, T), dim3(256), 0, s, W1, b1, W2, atlas, idx, HT, T2);
    return hipGetLastError();
}

hipError_t launch_stage_bwd(const float *W2, const float *HT, const float *dT2, const float *atlas,
                            const int16_t *koff, const int16_t *kv, int T, float *dH, float *dW1, float *db1,
                            float *dW2, hipStream_t s) {
    hipLaunchKernelGGL(k_stage_bwd_h, dim3(NV / VB, T), dim3(256), 0, s, W2, HT, dT2, dH);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_stage_bwd_w, dim3(T * (C2 * C1 * 16 / 256) + T * C1), dim3(256), 0, s, HT, dT2, dH, atlas,
                       koff, kv, T, dW1, db1, dW2);
    return hipGetLastError();
}

}  // namespace merlin
