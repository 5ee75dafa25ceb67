// merlin_winbwd.hip -- the window GEMM Q = a2w W3r (k_winfwd) and its backward (conv3 seen per window: a2w [T][nw][64] the
// relu(conv2) rows of the update's windows, W3r [T][64][576] conv3's weights as (ci) x (tap, co), src/actor_critic.py
// :13 conv3) in one launch plus an ordered fold, replacing hipBLASLt's input-gradient GEMM, the split-K weight
// gradient's batched GEMMs + torch sum, and the ReLU backward with its bias-gradient column sums (merlin/fast_step.py;
// 137.6 us standalone at nw = 6,571, scripts/probe_window_bwd.py):
//
//   da2w[w][c] = [a2w[w][c] > 0] * sum_j dQ[w][j] W3r[c][j]     db2[c] = sum_w da2w[w][c]
//   dW3r[c][j] = sum_w a2w[w][c] dQ[w][j]          (optionally db3[c] = sum_w dQ[w][c], tap 0: conv3's bias gradient)
//
// On the exact-f32 MFMA (v_mfma_f32_32x32x2_f32: every product and sum an f32 fmaf, fp32 GEMM arithmetic), one wave per
// 32 x 32 (input gradient) or 32 x 64 (weight gradient, K split over the windows) output tile, operands straight from
// L2 (the 30-MB dQ and the 0.3-MB W3r stay cache-resident): the input gradient loads 16-B runs of k per lane and
// pairs MFMA k slot h of step s with k = k0 + 4 h + s (the same permutation for both operands); the weight gradient's
// k is the window index, so each step's operands are one coalesced row of a2w / dQ per lane half.  Loads run P steps
// ahead in registers.  Every sum has a fixed order: the column sums per wave (rows in MFMA order, then the two lane
// halves), the weight gradient's splits, then k_winbwd_fold adds the partials in index order (bitwise reproducible).
#include <algorithm>

#include "merlin_internal.h"

namespace merlin {
namespace {

typedef float wb_f32x16 __attribute__((ext_vector_type(16)));
constexpr int WB_CI = 64, WB_CJ = 576;
constexpr int WB_PD = 4;        // input gradient: 8-k iterations loaded ahead
constexpr int WB_PW = 8;        // weight gradient: window steps loaded ahead
constexpr int WB_SPLIT = 256;   // weight gradient: windows per split

__device__ __forceinline__ wb_f32x16 wb_mfma(float a, float b, wb_f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// blocks [0, nd): input-gradient tiles (tower, 32-row tile, 32-column half); [nd, nd + nwg): weight-gradient tiles
// (tower, split, c half, 64-column j tile).  One wave per block.
__global__ __launch_bounds__(64) void k_winbwd(const float *__restrict__ a2w, const float *__restrict__ dQ,
                                               const float *__restrict__ W3r, int64_t nw, int T, int nd, int splits,
                                               float *__restrict__ da2w, float *__restrict__ colpart,
                                               float *__restrict__ wpart, float *__restrict__ tpart) {
    const int lane = threadIdx.x, fr = lane & 31, fh = lane >> 5;
    const int64_t rt = (nw + 31) / 32;
    wb_f32x16 acc = {};
    if ((int)blockIdx.x < nd) {
        const int b = blockIdx.x, t = b / (int)(rt * 2), rem = b - t * (int)(rt * 2), tile = rem >> 1, ch = rem & 1;
        const int64_t w0 = (int64_t)tile * 32;
        const int64_t wr = std::min<int64_t>(w0 + fr, nw - 1);  // clamped: rows past nw are computed, never stored
        const float4 *A = reinterpret_cast<const float4 *>(dQ + ((size_t)t * nw + wr) * WB_CJ) + fh;
        const float4 *B = reinterpret_cast<const float4 *>(W3r + ((size_t)t * WB_CI + ch * 32 + fr) * WB_CJ) + fh;
        constexpr int NI = WB_CJ / 8;  // 72 iterations of 8 k (4 MFMAs)
        float4 ra[WB_PD], rb[WB_PD];
#pragma unroll
        for (int i = 0; i < WB_PD; i++) {
            ra[i] = A[2 * i];
            rb[i] = B[2 * i];
        }
        for (int i0 = 0; i0 < NI; i0 += WB_PD) {
#pragma unroll
            for (int u = 0; u < WB_PD; u++) {
                const float4 a = ra[u], bb = rb[u];
                if (i0 + u + WB_PD < NI) {
                    ra[u] = A[2 * (i0 + u + WB_PD)];
                    rb[u] = B[2 * (i0 + u + WB_PD)];
                }
                acc = wb_mfma(a.x, bb.x, acc);
                acc = wb_mfma(a.y, bb.y, acc);
                acc = wb_mfma(a.z, bb.z, acc);
                acc = wb_mfma(a.w, bb.w, acc);
            }
        }
        // mask, store, the column sums of this wave's rows (rows past nw add 0)
        const int col = ch * 32 + fr;
        float cs = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; r++) {
            const int64_t row = w0 + (r & 3) + 8 * (r >> 2) + 4 * fh;
            if (row < nw) {
                const size_t o = ((size_t)t * nw + row) * WB_CI + col;
                const float v = a2w[o] > 0.0f ? acc[r] : 0.0f;
                da2w[o] = v;
                cs += v;
            }
        }
        cs += __shfl_xor(cs, 32);
        if (fh == 0) colpart[((size_t)t * rt + tile) * WB_CI + col] = cs;
        return;
    }
    // weight gradient: tile (t, s, c half ch, j tile jt of 64): rows [s * WB_SPLIT, ...) of a2w^T dQ
    const int b = blockIdx.x - nd, per_t = splits * 2 * 9, t = b / per_t, r0 = b - t * per_t;
    const int s = r0 / 18, ch = (r0 / 9) & 1, jt = r0 % 9;
    const int64_t k0 = (int64_t)s * WB_SPLIT, k1 = std::min<int64_t>(nw, k0 + WB_SPLIT);
    const float *Aw = a2w + (size_t)t * nw * WB_CI + ch * 32 + fr;        // A[c][w] = a2w[w][c]
    const float *Bw = dQ + (size_t)t * nw * WB_CJ + jt * 64 + fr;         // B[w][j] = dQ[w][j]
    wb_f32x16 acc2 = {};
    float ts0 = 0.0f, ts1 = 0.0f;  // tap 0's column sums (j < 64: the conv3 bias gradient), in the (j0 = 0, c half 0) waves
    const bool tap0 = tpart && jt == 0 && ch == 0;
    const int64_t nst = (k1 - k0 + 1) / 2;  // MFMA steps: rows k0 + 2 st + fh
    float pa[WB_PW], pb0[WB_PW], pb1[WB_PW];
    auto ld = [&](int64_t st, float &a, float &b0, float &b1) __attribute__((always_inline)) {
        const int64_t w = k0 + 2 * st + fh, wc = std::min<int64_t>(w, nw - 1);
        const bool ok = w < k1;
        const float va = Aw[wc * WB_CI], vb0 = Bw[wc * WB_CJ], vb1 = Bw[wc * WB_CJ + 32];
        a = ok ? va : 0.0f;
        b0 = ok ? vb0 : 0.0f;
        b1 = ok ? vb1 : 0.0f;
    };
#pragma unroll
    for (int i = 0; i < WB_PW; i++) ld(i, pa[i], pb0[i], pb1[i]);
    for (int64_t st0 = 0; st0 < nst; st0 += WB_PW) {
#pragma unroll
        for (int u = 0; u < WB_PW; u++) {
            const float a = pa[u], b0 = pb0[u], b1 = pb1[u];
            ld(st0 + u + WB_PW, pa[u], pb0[u], pb1[u]);  // past the end: clamped rows, zeroed
            if (st0 + u < nst) {
                acc = wb_mfma(a, b0, acc);
                acc2 = wb_mfma(a, b1, acc2);
                if (tap0) {
                    ts0 += b0;
                    ts1 += b1;
                }
            }
        }
    }
    if (tap0) {  // the two row parities, then one store per column
        ts0 += __shfl_xor(ts0, 32);
        ts1 += __shfl_xor(ts1, 32);
        if (fh == 0) {
            tpart[((size_t)t * splits + s) * WB_CI + fr] = ts0;
            tpart[((size_t)t * splits + s) * WB_CI + 32 + fr] = ts1;
        }
    }
    float *P = wpart + (((size_t)s * T + t) * WB_CI) * WB_CJ;
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int c = ch * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
        P[(size_t)c * WB_CJ + jt * 64 + fr] = acc[r];
        P[(size_t)c * WB_CJ + jt * 64 + 32 + fr] = acc2[r];
    }
}

// blocks [0, nb): dW3r = the splits' partials added in split order; then one wave per (tower, column): db2 = the
// column partials, lane q adding tiles q, q + 64, ... in order, then a fixed butterfly
__global__ __launch_bounds__(256) void k_winbwd_fold(const float *__restrict__ colpart, const float *__restrict__ wpart,
                                                     const float *__restrict__ tpart, int T, int64_t rt, int splits,
                                                     int nb, float *__restrict__ db2, float *__restrict__ dW3r,
                                                     float *__restrict__ db3) {
    if ((int)blockIdx.x < nb) {
        const int64_t n = (int64_t)T * WB_CI * WB_CJ, i = (int64_t)blockIdx.x * 256 + threadIdx.x;
        if (i >= n) return;
        float s = wpart[i];
#pragma unroll 8
        for (int q = 1; q < splits; q++) s += wpart[(size_t)q * n + i];
        dW3r[i] = s;
        return;
    }
    if ((int)blockIdx.x == nb + (T * WB_CI + 3) / 4) {  // db3 = tap 0's split sums in split order
        if (!db3 || (int)threadIdx.x >= T * WB_CI) return;
        const int t = threadIdx.x / WB_CI, c = threadIdx.x - t * WB_CI;
        float s = 0.0f;
        for (int q = 0; q < splits; q++) s += tpart[((size_t)t * splits + q) * WB_CI + c];
        db3[threadIdx.x] = s;
        return;
    }
    const int k = ((int)blockIdx.x - nb) * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (k >= T * WB_CI) return;
    const int t = k / WB_CI, c = k - t * WB_CI;
    float s = 0.0f;
    for (int64_t q = lane; q < rt; q += 64) s += colpart[((size_t)t * rt + q) * WB_CI + c];
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) s += __shfl_xor(s, m);
    if (lane == 0) db2[k] = s;
}

// The forward Q = a2w W3r [T][nw][576] (hipBLASLt's fp32 GEMM before, 22.7 us in the r05h step sequence): one wave per
// 32 x 64 output tile, K = 64: A = a2w rows by 16-B runs of k, B[k][j] = W3r[k][j] one coalesced row per lane half;
// k slot h of step s of an 8-k iteration is k = k0 + 4 h + s for both operands (as the input gradient above)
__global__ __launch_bounds__(64) void k_winfwd(const float *__restrict__ a2w, const float *__restrict__ W3r, int64_t nw,
                                               float *__restrict__ Q) {
    const int lane = threadIdx.x, fr = lane & 31, fh = lane >> 5;
    const int64_t rt = (nw + 31) / 32;
    const int b = blockIdx.x, per_t = (int)rt * 9, t = b / per_t, rem = b - t * per_t;
    const int64_t tile = rem / 9;
    const int jt = rem % 9;
    const int64_t w0 = tile * 32, wr = std::min<int64_t>(w0 + fr, nw - 1);
    const float4 *A = reinterpret_cast<const float4 *>(a2w + ((size_t)t * nw + wr) * WB_CI) + fh;
    const float *B = W3r + (size_t)t * WB_CI * WB_CJ + jt * 64 + fr;
    float4 ra[8];
#pragma unroll
    for (int i = 0; i < 8; i++) ra[i] = A[2 * i];
    float rb[8][4][2];
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int k = 8 * i + 4 * fh + u;
            rb[i][u][0] = B[(size_t)k * WB_CJ];
            rb[i][u][1] = B[(size_t)k * WB_CJ + 32];
        }
    wb_f32x16 acc = {}, acc2 = {};
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const float av[4] = {ra[i].x, ra[i].y, ra[i].z, ra[i].w};
#pragma unroll
        for (int u = 0; u < 4; u++) {
            acc = wb_mfma(av[u], rb[i][u][0], acc);
            acc2 = wb_mfma(av[u], rb[i][u][1], acc2);
        }
    }
    float *Qt = Q + (size_t)t * nw * WB_CJ + jt * 64 + fr;
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int64_t row = w0 + (r & 3) + 8 * (r >> 2) + 4 * fh;
        if (row < nw) {
            Qt[(size_t)row * WB_CJ] = acc[r];
            Qt[(size_t)row * WB_CJ + 32] = acc2[r];
        }
    }
}

}  // namespace

hipError_t launch_winfwd(const float *a2w, const float *W3r, int T, int64_t nw, float *Q, hipStream_t s) {
    if (nw <= 0 || T < 1) return nw == 0 ? hipSuccess : hipErrorInvalidValue;
    const int64_t nb = (int64_t)T * ((nw + 31) / 32) * 9;
    if (nb > INT32_MAX) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_winfwd, dim3((unsigned)nb), dim3(64), 0, s, a2w, W3r, nw, Q);
    return hipGetLastError();
}

int64_t winbwd_work_floats(int T, int64_t nw) {
    const int64_t rt = (nw + 31) / 32, splits = (nw + WB_SPLIT - 1) / WB_SPLIT;
    return (int64_t)T * rt * WB_CI + splits * T * WB_CI * WB_CJ + splits * T * WB_CI;
}

hipError_t launch_winbwd(const float *a2w, const float *dQ, const float *W3r, int T, int64_t nw, float *da2w,
                         float *db2, float *dW3r, float *work, hipStream_t s, float *db3) {
    if (nw <= 0 || T < 1) return hipErrorInvalidValue;
    const int64_t rt = (nw + 31) / 32, splits = (nw + WB_SPLIT - 1) / WB_SPLIT;
    const int64_t nd = (int64_t)T * rt * 2, nwg = (int64_t)T * splits * 18;
    if (nd + nwg > INT32_MAX) return hipErrorInvalidValue;
    float *colpart = work, *wpart = work + (size_t)T * rt * WB_CI, *tpart = wpart + (size_t)splits * T * WB_CI * WB_CJ;
    hipLaunchKernelGGL(k_winbwd, dim3((unsigned)(nd + nwg)), dim3(64), 0, s, a2w, dQ, W3r, nw, T, (int)nd, (int)splits,
                       da2w, colpart, wpart, db3 ? tpart : nullptr);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int nb = (T * WB_CI * WB_CJ + 255) / 256;
    hipLaunchKernelGGL(k_winbwd_fold, dim3((unsigned)(nb + (T * WB_CI + 3) / 4 + 1)), dim3(256), 0, s, colpart, wpart,
                       tpart, T, rt, (int)splits, nb, db2, dW3r, db3);
    return hipGetLastError();
}

}  // namespace merlin
