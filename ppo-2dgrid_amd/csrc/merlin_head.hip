// merlin_head.hip -- the memory-bound epilogues around the towers' conv3 / fc1 GEMMs and the
// heads' backward (src/actor_critic.py:14-18 conv3 + ReLU, :30-41 Linear(576, 512) -> ReLU ->
// Linear(512, act_dim | 1)), so that no full-size activation is touched more than once per
// direction outside the GEMMs:
//   k_bias_relu        Z = relu(Z + b) in place after a plain GEMM (instead of baddbmm's
//                      bias broadcast copy + a separate relu_ pass)
//   k_relu_bwd_colsum  dZ = [Y > 0] * dY and the bias gradient (column sums) in one pass
//   k_head_bwd         fc1's ReLU mask applied to the heads' input gradient, fused with the
//                      heads' weight gradients and fc1's bias gradient: one read of h, one
//                      write of dz per tower (instead of two select-backward zero fills, an
//                      add, a where and a reduction over [2, n, 512])
// Column sums are per-block partials folded in a fixed order (bitwise reproducible).
#include <algorithm>

#include "merlin_internal.h"

namespace merlin {
namespace {

constexpr int EBLK = 256;
constexpr int MAXA = 8;  // act_dim limit of the fused head backward

__device__ __forceinline__ float relu_nan(float v) { return v != v ? v : fmaxf(v, 0.0f); }  // torch.relu keeps NaN
__device__ __forceinline__ float4 f4_zero() { return make_float4(0.0f, 0.0f, 0.0f, 0.0f); }
__device__ __forceinline__ void f4_add(float4 &a, const float4 b) {
    a.x += b.x;
    a.y += b.y;
    a.z += b.z;
    a.w += b.w;
}
__device__ __forceinline__ float4 f4_mask(const float4 y, const float4 g) {
    return make_float4(y.x > 0.0f ? g.x : 0.0f, y.y > 0.0f ? g.y : 0.0f, y.z > 0.0f ? g.z : 0.0f,
                       y.w > 0.0f ? g.w : 0.0f);
}

// Z[t][r][:] = relu(Z[t][r][:] + b[t][:]), c4 = cols / 4
__global__ __launch_bounds__(EBLK) void k_bias_relu(float4 *__restrict__ Z, const float4 *__restrict__ b,
                                                    int64_t rows, int c4, int64_t total4) {
    for (int64_t e = (int64_t)blockIdx.x * EBLK + threadIdx.x; e < total4; e += (int64_t)gridDim.x * EBLK) {
        const int64_t tr = e / c4;
        const int c = (int)(e - tr * c4), t = (int)(tr / rows);
        const float4 bb = b[t * c4 + c];
        float4 v = Z[e];
        v.x = relu_nan(v.x + bb.x);
        v.y = relu_nan(v.y + bb.y);
        v.z = relu_nan(v.z + bb.z);
        v.w = relu_nan(v.w + bb.w);
        Z[e] = v;
    }
}

// Block (b, t): rows [b*per, min(rows, (b+1)*per)) of tower t.  Thread = (row lane r0, column
// group c); c4 divides EBLK, so EBLK / c4 rows are in flight per iteration and every wave
// load is a run of whole rows.  partials[t][b][c4] = the block's column sums of dZ.
__global__ __launch_bounds__(EBLK) void k_relu_bwd_colsum(const float4 *__restrict__ Y, const float4 *dY,
                                                          float4 *dZ, int64_t rows, int c4, int64_t per,
                                                          float4 *__restrict__ partials) {
    __shared__ float4 red[EBLK];
    const int t = blockIdx.y, R = EBLK / c4;
    const int c = threadIdx.x % c4, r0 = threadIdx.x / c4;
    const int64_t lo = (int64_t)blockIdx.x * per, hi = std::min<int64_t>(rows, lo + per);
    const size_t base = (size_t)t * rows * c4;
    float4 acc = f4_zero();
#pragma unroll 4
    for (int64_t r = lo + r0; r < hi; r += R) {
        const size_t e = base + (size_t)r * c4 + c;
        const float4 d = f4_mask(Y[e], dY[e]);
        dZ[e] = d;
        f4_add(acc, d);
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x < c4) {
        float4 s = red[threadIdx.x];
        for (int k = 1; k < R; k++) f4_add(s, red[threadIdx.x + k * c4]);
        partials[((size_t)t * gridDim.x + blockIdx.x) * c4 + threadIdx.x] = s;
    }
}

// partials[t][b][c4] = sum over the block's rows r of X[t][r * stride4 + c] (column sums of strided rows)
__global__ __launch_bounds__(EBLK) void k_colsum(const float4 *__restrict__ X, int64_t rows, int c4, int64_t stride4,
                                                 int64_t tstride4, int64_t per, float4 *__restrict__ partials) {
    __shared__ float4 red[EBLK];
    const int t = blockIdx.y, R = EBLK / c4;
    const int c = threadIdx.x % c4, r0 = threadIdx.x / c4;
    const int64_t lo = (int64_t)blockIdx.x * per, hi = std::min<int64_t>(rows, lo + per);
    const float4 *Xt = X + (size_t)t * tstride4 + c;
    float4 acc = f4_zero();
#pragma unroll 4
    for (int64_t r = lo + r0; r < hi; r += R) f4_add(acc, Xt[(size_t)r * stride4]);
    red[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x < c4) {
        float4 s = red[threadIdx.x];
        for (int k = 1; k < R; k++) f4_add(s, red[threadIdx.x + k * c4]);
        partials[((size_t)t * gridDim.x + blockIdx.x) * c4 + threadIdx.x] = s;
    }
}

// Fold of per-block partials: output k (< total) is the sum over blocks b of
// partials[(t * nblk + b) * S + off] with (t, off) = locate(k).  A block takes 32 outputs; its
// 8 slices of 32 threads each sum every 8th block (8 loads in flight), then slice 0 adds the
// 8 slice sums in order: fixed order, and no thread walks all nblk partials serially.
constexpr int FOLD_COLS = 32, FOLD_SLICES = 8;
template <typename Locate, typename Store>
__device__ __forceinline__ void fold_partials(const float *__restrict__ partials, int nblk, int S, int total,
                                              Locate locate, Store store) {
    __shared__ float red[FOLD_SLICES][FOLD_COLS];
    const int c = threadIdx.x % FOLD_COLS, z = threadIdx.x / FOLD_COLS;
    const int k = blockIdx.x * FOLD_COLS + c;
    float acc = 0.0f;
    if (k < total) {
        int t, off;
        locate(k, t, off);
        const float *p = partials + (size_t)t * nblk * S + off;
#pragma unroll 8
        for (int b = z; b < nblk; b += FOLD_SLICES) acc += p[(size_t)b * S];
    }
    red[z][c] = acc;
    __syncthreads();
    if (z == 0 && k < total) {
        float sum = red[0][c];
        for (int q = 1; q < FOLD_SLICES; q++) sum += red[q][c];
        store(k, sum);
    }
}

// out[t][c] = sum over blocks of partials[t][b][c]
__global__ __launch_bounds__(FOLD_COLS * FOLD_SLICES) void k_fold_cols(const float *__restrict__ partials, int nblk,
                                                                       int cols, int T, float *__restrict__ out) {
    fold_partials(
        partials, nblk, cols, T * cols, [&](int k, int &t, int &off) { t = k / cols; off = k - t * cols; },
        [&](int k, float v) { out[k] = v; });
}

// Heads backward with fc1's ReLU mask, h [2][n][H] = relu(fc1) of the actor / critic tower:
//   tower 0: dz[0][k] = [h0 > 0] * (sum_j dlogits[k][j] * Wa[j]),  dWa[j] += dlogits[k][j] * h0[k]
//   tower 1: dz[1][k] = [h1 > 0] * (dvalue[k] * wc),               dwc    += dvalue[k] * h1[k]
//   db4[t] += dz[t][k]
// partials[t][b][(1 + A) * H4] (float4): tower 0 = (db4_0, dWa rows 0..A-1), tower 1 = (db4_1, dwc).
// NA: the register arrays' size (A <= NA; the bench's A = 3 instance keeps 4 waves per SIMD resident)
//
// PL (dz as h3 planes, merlin_h3.hip's operand form, for fc1's input- and weight-gradient GEMMs): dz is not written
// as fp32 but as its planes dzp [2][n][H/8][2][8] f16, scaled by 2^e from a BOUND on max |dz| instead of its max --
// |dz[r][k]| <= sum_j max_r' |dlogits[r'][j]| |Wa[j][k]| (tower 0; tower 1: max |dvalue| |wc[k]|), the maxima from
// the loss (k_ppo_loss_fix's dmax, float bits: [0, A) the logits, [DMAX_VALUE] the value) -- so the scale is known
// before any dz value is, and the split costs no pass of its own.  Every block computes the same bound (the same
// operations in the same order); block 0 of tower t stores it to amax[t] (bits), from which the GEMMs derive the same
// e.  A bound above the max only shifts where the planes' 2^26 dynamic range starts (below 2^-26 of the bound).
constexpr int DMAX_VALUE = 8;
template <int NA, bool PL>
__global__ __launch_bounds__(EBLK) void k_head_bwd(const float4 *__restrict__ h, const float *__restrict__ dlogits,
                                                   const float *__restrict__ dvalue, const float4 *__restrict__ wa,
                                                   const float4 *__restrict__ wc, int64_t n, int H4, int A,
                                                   int64_t per, float4 *__restrict__ dz,
                                                   float4 *__restrict__ partials, uint32_t *__restrict__ amax,
                                                   const uint32_t *__restrict__ dmax, uint2 *__restrict__ dzp) {
    __shared__ float4 red[EBLK];
    const int t = blockIdx.y, R = EBLK / H4;
    const int c = threadIdx.x % H4, r0 = threadIdx.x / H4;
    const int nw = t == 0 ? A : 1;
    float4 w[NA], accw[NA];
    // the head-gradient source of this tower (actor: dlogits [n][A], critic: dvalue [n]): every load below is issued
    // unconditionally from it (index clamped into [0, nw)) and masked after, so no load waits behind a branch
    const float *dsrc = t == 0 ? dlogits : dvalue;
    const int dstride = t == 0 ? A : 1;
    const float4 *wsrc = t == 0 ? wa : wc;
#pragma unroll
    for (int j = 0; j < NA; j++) {
        const float4 x = wsrc[(j < nw ? j : 0) * H4 + c];
        w[j] = j < nw ? x : f4_zero();
        accw[j] = f4_zero();
    }
    float sc = 1.0f, sc2 = H3_LO_SCALE;
    if constexpr (PL) {
        float4 b = f4_zero();
#pragma unroll
        for (int j = 0; j < NA; j++) {
            if (j < nw) {
                const float D = __uint_as_float(__hip_atomic_load(dmax + (t == 0 ? j : DMAX_VALUE), __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_AGENT));
                b.x += D * fabsf(w[j].x);
                b.y += D * fabsf(w[j].y);
                b.z += D * fabsf(w[j].z);
                b.w += D * fabsf(w[j].w);
            }
        }
        uint32_t m = max(max(__float_as_uint(b.x), __float_as_uint(b.y)), max(__float_as_uint(b.z), __float_as_uint(b.w)));
        for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
        __shared__ uint32_t bred[EBLK / 64];
        if ((threadIdx.x & 63) == 0) bred[threadIdx.x >> 6] = m;
        __syncthreads();
        m = bred[0];
#pragma unroll
        for (int q = 1; q < EBLK / 64; q++) m = max(m, bred[q]);
        if (blockIdx.x == 0 && threadIdx.x == 0) amax[t] = m;
        const int e = h3_exp(m);
        sc = pow2f(e);
        sc2 = pow2f(e + 11);
    }
    float4 acc = f4_zero();
    uint32_t mz = 0u;  // max |dz| of the block as float bits (merlin_h3.hip's operand scale)
    const int64_t lo = (int64_t)blockIdx.x * per, hi = std::min<int64_t>(n, lo + per);
    const size_t base = (size_t)t * n * H4;
    // HEAD_ROWS rows per thread per round, all their loads issued before any is used (rows past the
    // block's range read its last row and are dropped): 64 B of h in flight per thread instead of 32 --
    // the pass is HBM-bound (h in, dz out) and 16 waves per CU kept too little in flight
    constexpr int HEAD_ROWS = 4;
    for (int64_t r = lo + r0; r < hi; r += HEAD_ROWS * R) {
        float4 hv[HEAD_ROWS];
        float d[HEAD_ROWS][NA];
#pragma unroll
        for (int k = 0; k < HEAD_ROWS; k++) {
            const int64_t rk = std::min<int64_t>(r + k * R, hi - 1);
            hv[k] = h[base + (size_t)rk * H4 + c];
#pragma unroll
            for (int j = 0; j < NA; j++) {
                const float x = dsrc[rk * dstride + (j < nw ? j : 0)];
                d[k][j] = j < nw ? x : 0.0f;
            }
        }
#pragma unroll
        for (int k = 0; k < HEAD_ROWS; k++) {
            if (r + k * R >= hi) break;
            float4 g = f4_zero();
#pragma unroll
            for (int j = 0; j < NA; j++) {
                if (j < nw) {
                    g.x += d[k][j] * w[j].x;
                    g.y += d[k][j] * w[j].y;
                    g.z += d[k][j] * w[j].z;
                    g.w += d[k][j] * w[j].w;
                    accw[j].x += d[k][j] * hv[k].x;
                    accw[j].y += d[k][j] * hv[k].y;
                    accw[j].z += d[k][j] * hv[k].z;
                    accw[j].w += d[k][j] * hv[k].w;
                }
            }
            const float4 o = f4_mask(hv[k], g);
            if constexpr (PL)
                h3_store4_pair(reinterpret_cast<uint4 *>(dzp) + base + (size_t)(r + k * R) * H4, c, o, sc, sc2);
            else
                dz[base + (size_t)(r + k * R) * H4 + c] = o;
            f4_add(acc, o);
            if constexpr (!PL) mz = std::max(mz, std::max(std::max(__float_as_uint(o.x) & 0x7fffffffu, __float_as_uint(o.y) & 0x7fffffffu),
                                       std::max(__float_as_uint(o.z) & 0x7fffffffu, __float_as_uint(o.w) & 0x7fffffffu)));
        }
    }
    if (!PL && amax) {  // block-uniform
        const uint32_t mx[2] = {t == 0 ? mz : 0u, t == 1 ? mz : 0u};
        block_amax2(mx, 2, amax);
    }
    float4 *dst = partials + ((size_t)t * gridDim.x + blockIdx.x) * (size_t)(1 + A) * H4;
#pragma unroll
    for (int q = 0; q < 1 + NA; q++) {
        if (q <= nw) {  // block-uniform
            __syncthreads();
            red[threadIdx.x] = q == 0 ? acc : accw[q > 0 ? q - 1 : 0];
            __syncthreads();
            if (threadIdx.x < H4) {
                float4 s = red[threadIdx.x];
                for (int k = 1; k < R; k++) f4_add(s, red[threadIdx.x + k * H4]);
                dst[(size_t)q * H4 + threadIdx.x] = s;
            }
        }
    }
}

// Heads forward (src/actor_critic.py:41-46, Linear(512, act_dim) and Linear(512, 1) on h = relu(fc1) of the
// actor / critic tower): logits[r][j] = sum_k h[0][r][k] Wa[j][k] (+ ba[j]), value[r] = sum_k h[1][r][k] wc[k]
// (+ bc).  One wave per row, HEADS_ROWS rows per round with all their loads issued first (both towers' rows:
// 4 KB); lane l holds columns 4 l .. 4 l + 3 and 256 + 4 l .. + 3 of the weights in registers, sums its eight
// products in column order, then the lanes' partials are added by a fixed xor butterfly.  Replaces the two
// skinny GEMMs (2 x ~55 us at the update's shape, both reading h).
constexpr int HEADS_ROWS = 4;
template <int NA>
__global__ __launch_bounds__(256) void k_heads_fwd(const float4 *__restrict__ h, int64_t n, const float4 *__restrict__ wa,
                                                   int A, const float4 *__restrict__ wc, const float *__restrict__ ba,
                                                   const float *__restrict__ bc, float *__restrict__ logits,
                                                   float *__restrict__ value) {
    constexpr int H4 = 128;  // hidden 512
    const int lane = threadIdx.x & 63;
    float4 w[NA][2], v[2];
#pragma unroll
    for (int q = 0; q < 2; q++) {
#pragma unroll
        for (int j = 0; j < NA; j++) w[j][q] = j < A ? wa[j * H4 + q * 64 + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
        v[q] = wc[q * 64 + lane];
    }
    auto dot = [](const float4 a, const float4 b, float s) {
        s += a.x * b.x;
        s += a.y * b.y;
        s += a.z * b.z;
        s += a.w * b.w;
        return s;
    };
    const int64_t waves = (int64_t)gridDim.x * 4;
    for (int64_t r0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r0 < n; r0 += waves * HEADS_ROWS) {
        float4 x[HEADS_ROWS][2][2];  // [row][tower][half]
#pragma unroll
        for (int k = 0; k < HEADS_ROWS; k++) {
            const int64_t r = std::min<int64_t>(r0 + k * waves, n - 1);
#pragma unroll
            for (int t = 0; t < 2; t++)
#pragma unroll
                for (int q = 0; q < 2; q++) x[k][t][q] = h[((size_t)t * n + r) * H4 + q * 64 + lane];
        }
#pragma unroll
        for (int k = 0; k < HEADS_ROWS; k++) {
            const int64_t r = r0 + k * waves;
            if (r >= n) break;  // wave-uniform
            float s[NA + 1];
#pragma unroll
            for (int j = 0; j < NA; j++) s[j] = dot(x[k][0][1], w[j][1], dot(x[k][0][0], w[j][0], 0.0f));
            s[NA] = dot(x[k][1][1], v[1], dot(x[k][1][0], v[0], 0.0f));
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
                for (int j = 0; j <= NA; j++) s[j] += __shfl_xor(s[j], off);
            if (lane == 0) {
#pragma unroll
                for (int j = 0; j < NA; j++)
                    if (j < A) logits[r * A + j] = ba ? s[j] + ba[j] : s[j];
                value[r] = bc ? s[NA] + bc[0] : s[NA];
            }
        }
    }
}

// db4[2][H], dWa[A][H], dwc[H] from the head partials: tower 0's rows are (db4_0, dWa), tower
// 1's (db4_1, dwc)
__global__ __launch_bounds__(FOLD_COLS * FOLD_SLICES) void k_head_fold(const float *__restrict__ partials, int nblk,
                                                                       int H, int A, float *__restrict__ db4,
                                                                       float *__restrict__ dwa,
                                                                       float *__restrict__ dwc) {
    const int S = (1 + A) * H;
    fold_partials(
        partials, nblk, S, S + 2 * H,
        [&](int k, int &t, int &off) {
            t = k < S ? 0 : 1;
            off = k < S ? k : k - S;
        },
        [&](int k, float v) {
            const int t = k < S ? 0 : 1, off = k < S ? k : k - S;
            if (off < H)
                db4[t * H + off] = v;
            else if (t == 0)
                dwa[off - H] = v;
            else
                dwc[off - H] = v;
        });
}

int blocks_for(int64_t rows) {
    return (int)std::max<int64_t>(1, std::min<int64_t>(EPI_MAX_BLOCKS, (rows + 31) / 32));
}

}  // namespace

size_t epilogue_work_floats() { return (size_t)2 * EPI_MAX_BLOCKS * (1 + MAXA) * 1024; }

bool epilogue_cols_ok(int cols) { return cols > 0 && cols % 4 == 0 && cols / 4 <= EBLK && EBLK % (cols / 4) == 0; }

int epilogue_max_act() { return MAXA; }

hipError_t launch_bias_relu(float *Z, const float *b, int64_t rows, int cols, int T, hipStream_t s) {
    const int64_t total4 = (int64_t)T * rows * (cols / 4);
    if (total4 <= 0) return hipSuccess;
    const int grid = (int)std::min<int64_t>((total4 + EBLK - 1) / EBLK, 256 * 16);
    hipLaunchKernelGGL(k_bias_relu, dim3(grid), dim3(EBLK), 0, s, reinterpret_cast<float4 *>(Z),
                       reinterpret_cast<const float4 *>(b), rows, cols / 4, total4);
    return hipGetLastError();
}

hipError_t launch_relu_bwd_colsum(const float *Y, const float *dY, float *dZ, int64_t rows, int cols, int T,
                                  float *dbias, float *work, hipStream_t s) {
    if (rows <= 0) return zero_async(dbias, sizeof(float) * T * cols, s);
    const int nblk = blocks_for(rows);
    const int64_t per = (rows + nblk - 1) / nblk;
    hipLaunchKernelGGL(k_relu_bwd_colsum, dim3(nblk, T), dim3(EBLK), 0, s, reinterpret_cast<const float4 *>(Y),
                       reinterpret_cast<const float4 *>(dY), reinterpret_cast<float4 *>(dZ), rows, cols / 4, per,
                       reinterpret_cast<float4 *>(work));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_fold_cols, dim3((T * cols + FOLD_COLS - 1) / FOLD_COLS), dim3(FOLD_COLS * FOLD_SLICES), 0, s,
                       work, nblk, cols, T, dbias);
    return hipGetLastError();
}

hipError_t launch_colsum(const float *X, int64_t rows, int cols, int64_t row_stride, int64_t tower_stride, int T,
                         float *out, float *work, hipStream_t s) {
    if (rows <= 0) return zero_async(out, sizeof(float) * T * cols, s);
    const int nblk = blocks_for(rows);
    const int64_t per = (rows + nblk - 1) / nblk;
    hipLaunchKernelGGL(k_colsum, dim3(nblk, T), dim3(EBLK), 0, s, reinterpret_cast<const float4 *>(X), rows, cols / 4,
                       row_stride / 4, tower_stride / 4, per, reinterpret_cast<float4 *>(work));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_fold_cols, dim3((T * cols + FOLD_COLS - 1) / FOLD_COLS), dim3(FOLD_COLS * FOLD_SLICES), 0, s,
                       work, nblk, cols, T, out);
    return hipGetLastError();
}

hipError_t launch_head_bwd(const float *h, const float *dlogits, const float *dvalue, const float *wa,
                           const float *wc, int64_t n, int H, int A, float *dz, float *db4, float *dwa, float *dwc,
                           float *work, uint32_t *amax, hipStream_t s, const uint32_t *dmax, void *dz_planes) {
    if (dz_planes && (!dmax || !amax || A > DMAX_VALUE)) return hipErrorInvalidValue;
    if (n <= 0) {
        hipError_t e = zero_async(db4, sizeof(float) * 2 * H, s);
        if (e == hipSuccess) e = zero_async(dwa, sizeof(float) * A * H, s);
        return e == hipSuccess ? zero_async(dwc, sizeof(float) * H, s) : e;
    }
    const int nblk = blocks_for(n);
    const int64_t per = (n + nblk - 1) / nblk;
    const auto kern = dz_planes ? (A <= 3 ? k_head_bwd<3, true> : k_head_bwd<MAXA, true>)
                                : (A <= 3 ? k_head_bwd<3, false> : k_head_bwd<MAXA, false>);
    hipLaunchKernelGGL(kern, dim3(nblk, 2), dim3(EBLK), 0, s,
                       reinterpret_cast<const float4 *>(h), dlogits, dvalue, reinterpret_cast<const float4 *>(wa),
                       reinterpret_cast<const float4 *>(wc), n, H / 4, A, per, reinterpret_cast<float4 *>(dz),
                       reinterpret_cast<float4 *>(work), amax, dmax, static_cast<uint2 *>(dz_planes));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int total = (1 + A) * H + 2 * H;
    hipLaunchKernelGGL(k_head_fold, dim3((total + FOLD_COLS - 1) / FOLD_COLS), dim3(FOLD_COLS * FOLD_SLICES), 0, s,
                       work, nblk, H, A, db4, dwa, dwc);
    return hipGetLastError();
}

hipError_t launch_heads_fwd(const float *h, int64_t n, int H, const float *wa, int A, const float *wc, const float *ba,
                            const float *bc, float *logits, float *value, hipStream_t s) {
    if (H != 512 || A < 1 || A > MAXA) return hipErrorInvalidValue;
    if (n <= 0) return hipSuccess;
    const int grid = (int)std::min<int64_t>((n + 4 * HEADS_ROWS - 1) / (4 * HEADS_ROWS), 256 * 8);
    const float4 *h4 = reinterpret_cast<const float4 *>(h), *wa4 = reinterpret_cast<const float4 *>(wa),
                 *wc4 = reinterpret_cast<const float4 *>(wc);
    if (A <= 3)
        hipLaunchKernelGGL(k_heads_fwd<3>, dim3(grid), dim3(256), 0, s, h4, n, wa4, A, wc4, ba, bc, logits, value);
    else
        hipLaunchKernelGGL(k_heads_fwd<MAXA>, dim3(grid), dim3(256), 0, s, h4, n, wa4, A, wc4, ba, bc, logits, value);
    return hipGetLastError();
}

}  // namespace merlin
