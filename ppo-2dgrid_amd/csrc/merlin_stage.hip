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
// dP[o][k] = sum over the (v, e) with idx[v][e] = k of dH[v][o], dW1 = dP contracted with the atlas.
//
// The combinations of one parity type (ee 5, eo 25, oe 25, oo 625) all read the same 4 of W2's 16 taps, so the
// forward and dH kernels work on chunks of up to 8 combinations of one type with that type's W2 slice ([64][4][32],
// 32 KB) in LDS; dW2 is one block per (tower, type, tap) summing over the type's combinations in chunks staged
// through LDS.  Every sum runs in a fixed order (the same bits every call) and accumulates in f64, rounded once to
// f32 (dH, HT, T2 and the gradients): more accurate than the fp32 blocked sums of the torch formulation
// (tests/test_gpu_stage_precision.py), for ~11 M multiply-adds per table, where the f64 rate costs nothing visible.
#include "merlin_internal.h"

namespace merlin {
namespace {

constexpr int C1 = 32, C2 = 64, NV = 680, NROW = 4 * NV;  // conv1 / conv2 channels, combinations, T2 rows
constexpr int VB = 8;                                    // combinations per chunk
constexpr int NCH = 1 + 4 + 4 + 79;                      // chunks of 8 per type: ceil(5/8) + 2 ceil(25/8) + ceil(625/8)

__device__ __forceinline__ int part_off(int p) { return p == 0 ? 0 : p == 1 ? 5 : p == 2 ? 30 : p == 3 ? 55 : NV; }

// chunk -> (type, first combination, count)
__device__ __forceinline__ void chunk_of(int c, int &p, int &v0, int &nv) {
    const int first[5] = {0, 1, 5, 9, NCH};
    p = c < first[1] ? 0 : c < first[2] ? 1 : c < first[3] ? 2 : 3;
    v0 = part_off(p) + (c - first[p]) * VB;
    nv = min(VB, part_off(p + 1) - v0);
}

// W2[t] slice of type p into LDS as [co][j][o] (o fastest: conflict-free reads across o)
__device__ void load_w2_slice(const float *__restrict__ W2, int p, float *__restrict__ Ws) {
    const int yp = p >> 1, xp = p & 1;
    for (int q = threadIdx.x; q < C2 * 4 * C1; q += blockDim.x) {
        const int co = q / (4 * C1), r = q - co * 4 * C1, j = r / C1, o = r - j * C1;
        Ws[q] = W2[((size_t)co * C1 + o) * 16 + (2 * (j >> 1) + yp) * 4 + 2 * (j & 1) + xp];
    }
}

// W2[t] slice of type p into LDS as [j][o][co] (co fastest, rows padded to WSP words): the forward's T2 loop has
// consecutive threads on consecutive co (in load_w2_slice's [co][j][o] layout they read 128 words apart: one bank,
// 64-way conflicts); the padding keeps the stores (consecutive o) on distinct banks too
constexpr int WSP = C2 + 1;
__device__ void load_w2_slice_co(const float *__restrict__ W2, int p, float *__restrict__ Ws) {
    const int yp = p >> 1, xp = p & 1;
    for (int q = threadIdx.x; q < C2 * 4 * C1; q += blockDim.x) {  // o fastest: W2 read 64 B apart
        const int co = q / (4 * C1), r = q - co * 4 * C1, j = r / C1, o = r - j * C1;
        Ws[(j * C1 + o) * WSP + co] = W2[((size_t)co * C1 + o) * 16 + (2 * (j >> 1) + yp) * 4 + 2 * (j & 1) + xp];
    }
}

// grid (NCH, T): HT rows of one chunk and their T2 rows; HT saved for the backward
__global__ __launch_bounds__(256) void k_stage_fwd(const float *__restrict__ W1, const float *__restrict__ b1,
                                                   const float *__restrict__ W2, const float *__restrict__ atlas,
                                                   const int16_t *__restrict__ idx, float *__restrict__ HT,
                                                   float *__restrict__ T2) {
    __shared__ float Wl[C1 * 3 * 64], Al[5 * 3 * 64], H[VB][C1], Ws[4 * C1 * WSP];
    __shared__ double P[C1 * 80];
    const int t = blockIdx.y;
    int p, v0, nv;
    chunk_of(blockIdx.x, p, v0, nv);
    W1 += (size_t)t * C1 * 3 * 64;
    for (int q = threadIdx.x; q < C1 * 3 * 64; q += 256) Wl[q] = W1[q];
    for (int q = threadIdx.x; q < 5 * 3 * 64; q += 256) Al[q] = atlas[q];
    load_w2_slice_co(W2 + (size_t)t * C2 * C1 * 16, p, Ws);
    __syncthreads();
    for (int q = threadIdx.x; q < C1 * 80; q += 256) {  // P[o][k], 48 products each
        const int o = q / 80, k = q - o * 80;
        const int slot = k / 20, bin = k - slot * 20;
        const int dy = slot >> 1, dx = slot & 1, z = bin >> 2, qy = (bin >> 1) & 1, qx = bin & 1;
        double acc = 0.0;
        for (int c = 0; c < 3; c++)
#pragma unroll
            for (int kk = 0; kk < 4; kk++)
#pragma unroll
                for (int l = 0; l < 4; l++)
                    acc += (double)Wl[(o * 3 + c) * 64 + (4 * dy + kk) * 8 + 4 * dx + l] *
                           (double)Al[(z * 3 + c) * 64 + (4 * qy + kk) * 8 + 4 * qx + l];
        P[q] = acc;
    }
    __syncthreads();
    {
        const int vl = threadIdx.x / C1, o = threadIdx.x - vl * C1;  // VB * C1 == 256
        if (vl < nv) {
            const int v = v0 + vl;
            double d = b1[t * C1 + o];
            for (int e = 0; e < 4; e++) d += P[o * 80 + idx[v * 4 + e]];
            float s = (float)d;
            s = s != s ? s : fmaxf(s, 0.0f);
            H[vl][o] = s;
            HT[((size_t)t * NV + v) * C1 + o] = s;
        }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < nv * 4 * C2; q += 256) {  // T2 rows 4 v + j
        const int vl = q / (4 * C2), r = q - vl * 4 * C2, j = r / C2, co = r - j * C2;
        const float *w = Ws + j * C1 * WSP + co;
        double acc = 0.0;
#pragma unroll 8
        for (int o = 0; o < C1; o++) acc += (double)H[vl][o] * (double)w[o * WSP];
        T2[((size_t)t * NROW + 4 * (v0 + vl) + j) * C2 + co] = (float)acc;
    }
}

// grid (NCH, T): dH[t][v][o] = [HT > 0] * sum_{j, co} dT2[4 v + j][co] * W2[co][o][tap(type, j)]
__global__ __launch_bounds__(256) void k_stage_bwd_h(const float *__restrict__ W2, const float *__restrict__ HT,
                                                     const float *__restrict__ dT2, float *__restrict__ dH) {
    __shared__ float G[VB][4 * C2], Ws[C2 * 4 * C1];
    const int t = blockIdx.y;
    int p, v0, nv;
    chunk_of(blockIdx.x, p, v0, nv);
    load_w2_slice(W2 + (size_t)t * C2 * C1 * 16, p, Ws);
    for (int q = threadIdx.x; q < nv * 4 * C2; q += 256)
        G[q / (4 * C2)][q % (4 * C2)] = dT2[((size_t)t * NROW + 4 * v0) * C2 + q];
    __syncthreads();
    const int vl = threadIdx.x / C1, o = threadIdx.x - vl * C1;
    if (vl >= nv) return;
    double acc = 0.0;
    for (int j = 0; j < 4; j++)
#pragma unroll 8
        for (int co = 0; co < C2; co++) acc += (double)G[vl][j * C2 + co] * (double)Ws[(co * 4 + j) * C1 + o];
    const size_t hi = ((size_t)t * NV + v0 + vl) * C1 + o;
    dH[hi] = HT[hi] > 0.0f ? (float)acc : 0.0f;
}

constexpr int VS = 64;      // combinations per LDS stage of the dW2 blocks
constexpr int NP3 = 10;  // the 625-combination type's dW2 sums split over this many blocks (63 combinations each)
constexpr int NI = 12 + 4 * NP3;  // dW2 work items per tower: (type < 3, j), then (j, part) of type 3
constexpr int WT = 1024;    // threads of k_stage_bwd_w
constexpr int WQ = WT / 256;  // combination groups of a dW2 block (each thread of a group: 8 outputs)

// blocks [0, T * NI): work item (tower, type, j[, part]): dW2[co][o][tap] = sum over the type's combinations of
// HT[v][o] * dT2[4 v + j][co]; group g of the block's four thread groups sums the combinations v with (v - va) % 4 ==
// g in order (8 outputs per thread), the four partials join in a fixed order -- a type-3 block walked 625
// combinations, 10 dependent load-and-sum stages, the kernel's time: type 3's sums are split into NP3 blocks of
// 63 combinations whose f64 partials k_stage_fold adds in part order;  blocks [T * NI, T * NI + T * C1): tower t,
// conv1 channel o: db1[o] = sum_v dH[v][o] (strided partial sums, then a fixed tree), dP[o][k]
// for the 80 k (combinations in (v, e) order through the CSR kinv), then dW1[o][c][ky][kx]
__global__ __launch_bounds__(WT) void k_stage_bwd_w(const float *__restrict__ HT, const float *__restrict__ dT2,
                                                    const float *__restrict__ dH, const float *__restrict__ atlas,
                                                    const int16_t *__restrict__ koff, const int16_t *__restrict__ kv,
                                                    int T, float *__restrict__ dW1, float *__restrict__ db1,
                                                    float *__restrict__ dW2, double *__restrict__ ws) {
    __shared__ float Hs[VS][C1], Gs[VS][C2];
    __shared__ double part[WQ - 1][256 * 8], red[WT], dP[80];
    if ((int)blockIdx.x < T * NI) {
        const int t = blockIdx.x / NI, it = blockIdx.x % NI;
        const int p = it < 12 ? it >> 2 : 3, j = it < 12 ? it & 3 : (it - 12) / NP3, q = it < 12 ? 0 : (it - 12) % NP3;
        const int tap = (2 * (j >> 1) + (p >> 1)) * 4 + 2 * (j & 1) + (p & 1);
        constexpr int CH3 = (625 + NP3 - 1) / NP3;
        const int va = p < 3 ? part_off(p) : part_off(3) + q * CH3, vb = p < 3 ? part_off(p + 1) : min(va + CH3, NV);
        const int g = threadIdx.x >> 8, l = threadIdx.x & 255;
        const int o = l & (C1 - 1), cq = l >> 5;  // outputs (co = cq + 8 i, o)
        double acc[8];
#pragma unroll
        for (int i = 0; i < 8; i++) acc[i] = 0.0;
        // the next stage's values are loaded into registers while this stage is summed (one stage of HT and dT2
        // rows: VS * C1 / WT = 2 and VS * C2 / WT = 4 values per thread; rows past the type's end read as 0)
        constexpr int NH = VS * C1 / WT, NG = VS * C2 / WT;
        float rh[NH], rg[NG];
        auto load = [&](int vs) {
#pragma unroll
            for (int u = 0; u < NH; u++) {  // (loads unconditional -- rows clamped into the type -- then masked)
                const int q = threadIdx.x + u * WT, vl = q / C1, in = vs + vl < vb;
                const float x = HT[((size_t)t * NV + (in ? vs : vb - 1 - vl)) * C1 + q];
                rh[u] = in ? x : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < NG; u++) {
                const int q = threadIdx.x + u * WT, vl = q / C2, co = q - vl * C2, in = vs + vl < vb;
                const float x = dT2[((size_t)t * NROW + 4 * (in ? vs + vl : vb - 1) + j) * C2 + co];
                rg[u] = in ? x : 0.0f;
            }
        };
        load(va);
        for (int vs = va; vs < vb; vs += VS) {
            const int n = min(VS, vb - vs);
            __syncthreads();
#pragma unroll
            for (int u = 0; u < NH; u++) {
                const int q = threadIdx.x + u * WT;
                Hs[q / C1][q % C1] = rh[u];
            }
#pragma unroll
            for (int u = 0; u < NG; u++) {
                const int q = threadIdx.x + u * WT;
                Gs[q / C2][q % C2] = rg[u];
            }
            __syncthreads();
            if (vs + VS < vb) load(vs + VS);
            for (int vl = g; vl < n; vl += WQ) {  // VS % WQ == 0: group g keeps its residue across stages
                const double h = Hs[vl][o];
#pragma unroll
                for (int i = 0; i < 8; i++) acc[i] += h * (double)Gs[vl][cq + 8 * i];
            }
        }
        if (g > 0) {
#pragma unroll
            for (int i = 0; i < 8; i++) part[g - 1][i * 256 + l] = acc[i];
        }
        __syncthreads();
        if (g == 0) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const double s = (acc[i] + part[0][i * 256 + l]) + (part[1][i * 256 + l] + part[2][i * 256 + l]);
                if (p < 3)
                    dW2[(((size_t)t * C2 + cq + 8 * i) * C1 + o) * 16 + tap] = (float)s;
                else
                    ws[(((size_t)t * 4 + j) * NP3 + q) * 2048 + i * 256 + l] = s;
            }
        }
        return;
    }
    const int b = blockIdx.x - T * NI, t = b / C1, o = b - t * C1;
    const float *d = dH + (size_t)t * NV * C1 + o;
    {  // db1: thread i sums combinations i, i + WT, ... in order, then a fixed tree
        double s = 0.0;
        for (int v = threadIdx.x; v < NV; v += WT) s += d[(size_t)v * C1];
        red[threadIdx.x] = s;
    }
    {  // dP[o][k]: the sum over the (v, e) entries with idx[v][e] = k.  One wave per k (five k per wave): lane l adds
       // entries l, l + 64, ... in order (one round of loads for most k; a bin of the 625-combination type has ~125
       // entries, which one thread walked as ~16 dependent rounds of two loads: the kernel's critical path), then a
       // fixed butterfly over the lanes -- the same order on every call
        const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
        for (int k = wv; k < 80; k += WT / 64) {
            const int i0 = koff[k], i1 = koff[k + 1];
            double acc = 0.0;
            for (int i = i0 + ln; i < i1; i += 64) acc += d[(size_t)kv[i] * C1];
#pragma unroll
            for (int m = 32; m > 0; m >>= 1) acc += __shfl_xor(acc, m);
            if (ln == 0) dP[k] = acc;
        }
    }
    __syncthreads();
    for (int w = WT / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) db1[t * C1 + o] = (float)red[0];
    for (int q = threadIdx.x; q < 3 * 64; q += WT) {  // dW1[t][o][c][ky][kx]
        const int c = q >> 6, ky = (q >> 3) & 7, kx = q & 7;
        const int dy = ky >> 2, kk = ky & 3, dx = kx >> 2, l = kx & 3, slot = 2 * dy + dx;
        double acc = 0.0;
        for (int bin = 0; bin < 20; bin++) {
            const int z = bin >> 2, qy = (bin >> 1) & 1, qx = bin & 1;
            acc += dP[slot * 20 + bin] * (double)atlas[((z * 3 + c) * 8 + 4 * qy + kk) * 8 + 4 * qx + l];
        }
        dW1[(((size_t)t * C1 + o) * 3 + c) * 64 + ky * 8 + kx] = (float)acc;
    }
}

// grid (T * 4): type 3's dW2 at tap j from its NP3 partial sums, added in part order
__global__ __launch_bounds__(256) void k_stage_fold(const double *__restrict__ ws, float *__restrict__ dW2) {
    const int t = blockIdx.x >> 2, j = blockIdx.x & 3, l = threadIdx.x, o = l & (C1 - 1), cq = l >> 5;
    const int tap = (2 * (j >> 1) + 1) * 4 + 2 * (j & 1) + 1;
    const double *w = ws + ((size_t)t * 4 + j) * NP3 * 2048;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        double s = w[i * 256 + l];
        for (int q = 1; q < NP3; q++) s += w[q * 2048 + i * 256 + l];
        dW2[(((size_t)t * C2 + cq + 8 * i) * C1 + o) * 16 + tap] = (float)s;
    }
}

}  // namespace

hipError_t launch_stage_fwd(const float *W1, const float *b1, const float *W2, const float *atlas, const int16_t *idx,
                            int T, float *HT, float *T2, hipStream_t s) {
    hipLaunchKernelGGL(k_stage_fwd, dim3(NCH, T), dim3(256), 0, s, W1, b1, W2, atlas, idx, HT, T2);
    return hipGetLastError();
}

hipError_t launch_stage_bwd(const float *W2, const float *HT, const float *dT2, const float *atlas,
                            const int16_t *koff, const int16_t *kv, int T, float *dH, float *dW1, float *db1,
                            float *dW2, double *ws, hipStream_t s) {
    hipLaunchKernelGGL(k_stage_bwd_h, dim3(NCH, T), dim3(256), 0, s, W2, HT, dT2, dH);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_stage_bwd_w, dim3(T * NI + T * C1), dim3(WT), 0, s, HT, dT2, dH, atlas, koff, kv, T, dW1,
                       db1, dW2, ws);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_stage_fold, dim3(T * 4), dim3(256), 0, s, ws, dW2);
    return hipGetLastError();
}

}  // namespace merlin
