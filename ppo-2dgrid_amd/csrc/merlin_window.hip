// merlin_window.hip -- conv2 and conv3 of both CNN towers evaluated once per distinct
// receptive-field window of an update's frames (src/actor_critic.py:11-14), and the
// fixed-order segmented sums of their backward passes.
//
// conv2 output (py, px) of a frame depends only on the frame's 3x3 tile-class window at
// (py, px) (its 16 conv2 table rows, merlin_conv2lut.hip), and convolution + ReLU are
// translation invariant, so merlin/windows.py numbers the distinct windows of a rollout once
// per update and each minibatch runs
//   Z2w[t][w]     = sum over the 16 taps of T2[t][rows[w][tap]]                    k_window_lut
//   Q[t][w][tap]  = relu(Z2w[t][w] + b2[t]) . W3[t][:, :, tap]        (a small GEMM in torch)
//   Y3[t][u*9+p3] = relu(b3[t] + sum over the 9 taps of Q[t][wid[g_u][p3+tap]][tap])  k_window_conv3
// instead of building conv3's 576-wide im2col rows (3.3 GB per minibatch) and their GEMM.
// Backward:
//   dQ[t][w*9+tap] = sum of dZ3[t][u*9+p3] over the (u, p3) that read Q[t][w][tap]
//   dT2[t][row]    = sum of dZ2w[t][w] over the (w, tap) that read T2[t][row]
// are segmented sums over entry lists sorted by destination once per update: k_seg_sum cuts a
// list into items of L entries, one wave per item, adding each destination's entries in list
// order; a destination whose entries span items gets the items' partial sums added in item
// order by k_seg_fix.  No atomics: bitwise reproducible.
#include <algorithm>

#include "merlin_internal.h"

namespace merlin {
namespace {

constexpr int NROW = 2720;  // conv2 table rows per tower (merlin_conv2lut.hip)

__device__ __forceinline__ void f4_add(float4 &a, const float4 b) {
    a.x += b.x;
    a.y += b.y;
    a.z += b.z;
    a.w += b.w;
}
__device__ __forceinline__ float relu_nan(float v) { return v != v ? v : fmaxf(v, 0.0f); }  // torch.relu keeps NaN

// Z2w[t][w][c4] = sum_{k<16} T2[t][rows[w][k]][c4], taps in k_conv2_lut_fwd's order
__global__ __launch_bounds__(256) void k_window_lut(const int32_t *__restrict__ rows, int64_t nw,
                                                    const float4 *__restrict__ tab, int T,
                                                    float4 *__restrict__ Z2w) {
    const int64_t total = (int64_t)T * nw * 16;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
        const int c = (int)(e & 15);
        const int64_t tw = e >> 4;
        const int t = (int)(tw / nw);
        const int32_t *r = rows + (tw - (int64_t)t * nw) * 16;
        const float4 *tt = tab + (size_t)t * NROW * 16 + c;
        float4 v[16];
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = tt[r[k] * 16];
        float4 acc = v[0];
#pragma unroll
        for (int k = 1; k < 16; k++) f4_add(acc, v[k]);
        Z2w[e] = acc;
    }
}

// Y3[t][u*9 + p3][c4] = relu(b3[t][c4] + sum_tap Q[t][wid[g*25 + p2(p3, tap)]][tap][c4]); 16
// consecutive lanes read one 256-B row of Q per tap
__global__ __launch_bounds__(256) void k_window_conv3(const float4 *__restrict__ Q, int64_t nw,
                                                      const int32_t *__restrict__ wid,
                                                      const int64_t *__restrict__ groups, int64_t n,
                                                      const float4 *__restrict__ b3, int T,
                                                      float4 *__restrict__ Y3) {
    const int64_t total = (int64_t)T * n * 9 * 16;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
        const int c = (int)(e & 15);
        const int64_t r = e >> 4, tu = r / 9;
        const int p3 = (int)(r - tu * 9), t = (int)(tu / n);
        const int64_t u = tu - (int64_t)t * n;
        const int32_t *wr = wid + (groups ? groups[u] : u) * 25;
        const int oy = p3 / 3, ox = p3 - 3 * (p3 / 3);
        const float4 *qt = Q + (size_t)t * nw * 9 * 16 + c;
        float4 v[9];
#pragma unroll
        for (int tap = 0; tap < 9; tap++) {
            const int ky = tap / 3, kx = tap - 3 * (tap / 3);
            v[tap] = qt[((size_t)wr[(oy + ky) * 5 + ox + kx] * 9 + tap) * 16];
        }
        float4 acc = v[0];
#pragma unroll
        for (int tap = 1; tap < 9; tap++) f4_add(acc, v[tap]);
        const float4 b = b3[t * 16 + c];
        Y3[e] = make_float4(relu_nan(acc.x + b.x), relu_nan(acc.y + b.y), relu_nan(acc.z + b.z),
                            relu_nan(acc.w + b.w));
    }
}

// One wave per item of L entries; lane = (tower t, float2 column c2), so one wave load reads
// one entry's 256-B row of each tower.  The wave loads 64 entries' (idx, key) at a time,
// resolves their source rows (through slot[] when given: -1 = not in this minibatch), and
// walks the valid ones in order, SEG_UNROLL row loads in flight (issued unconditionally:
// a select around a load would make hipcc wait for each load in turn), flushing a
// destination's sum when the key changes.  The item's first / last destination, when it
// continues in the neighbouring item, goes to carry[t][item][0 / 1] instead of out.  With
// acc_out the sums are added to out (one writer per destination per launch), so a list split
// by source block into several launches (merlin/windows.py) accumulates in block order.
constexpr int SEG_WAVES = 4, SEG_UNROLL = 8;
__global__ __launch_bounds__(64 * SEG_WAVES) void k_seg_sum(const float2 *__restrict__ src, int64_t src_rows,
                                                           const int32_t *__restrict__ idx,
                                                           const int32_t *__restrict__ key, int64_t nnz,
                                                           const int32_t *__restrict__ slot, int S, int64_t L,
                                                           int64_t nitems, int T, float2 *__restrict__ out,
                                                           int64_t out_rows, float2 *__restrict__ carry,
                                                           int acc_out) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int t = lane >> 5, c2 = lane & 31;
    const bool live = t < T;
    const float2 *srct = src + (size_t)(live ? t : 0) * src_rows * 32 + c2;
    const float2 zero = make_float2(0.0f, 0.0f);
    for (int64_t it = (int64_t)blockIdx.x * SEG_WAVES + wv; it < nitems; it += (int64_t)gridDim.x * SEG_WAVES) {
        const int64_t e0 = it * L, e1 = std::min<int64_t>(nnz, e0 + L);
        const int kfirst = key[e0], klast = key[e1 - 1];
        const bool xfirst = e0 > 0 && key[e0 - 1] == kfirst;
        const bool xlast = e1 < nnz && key[e1] == klast;
        const bool to_head_last = kfirst == klast && xlast;
        float2 head = zero, tail = zero, acc = zero;
        int cur = -1;
        auto flush = [&]() {
            if (cur == kfirst && (xfirst || to_head_last))
                head = acc;
            else if (cur == klast && xlast)
                tail = acc;
            else if (live) {
                float2 *o = out + ((size_t)t * out_rows + cur) * 32 + c2;
                if (acc_out) {
                    const float2 p = *o;
                    *o = make_float2(p.x + acc.x, p.y + acc.y);
                } else {
                    *o = acc;
                }
            }
        };
        for (int64_t base = e0; base < e1; base += 64) {
            int row = -1, k = -1;
            if (base + lane < e1) {
                const int v = idx[base + lane];
                k = key[base + lane];
                if (slot) {
                    const int q = v / S;
                    const int s = slot[q];
                    row = s >= 0 ? s * S + (v - q * S) : -1;
                } else {
                    row = v;
                }
            }
            unsigned long long m = __ballot(row >= 0);
            while (m) {
                int rq[SEG_UNROLL], kq[SEG_UNROLL];
#pragma unroll
                for (int q = 0; q < SEG_UNROLL; q++) {
                    const int j = m ? __builtin_ctzll(m) : -1;  // wave-uniform
                    if (m) m &= m - 1;
                    rq[q] = j >= 0 ? __shfl(row, j) : 0;
                    kq[q] = j >= 0 ? __shfl(k, j) : -1;
                }
                float2 vq[SEG_UNROLL];
#pragma unroll
                for (int q = 0; q < SEG_UNROLL; q++) vq[q] = srct[(size_t)rq[q] * 32];
#pragma unroll
                for (int q = 0; q < SEG_UNROLL; q++) {
                    if (kq[q] < 0) break;
                    if (kq[q] != cur) {
                        if (cur >= 0) flush();
                        cur = kq[q];
                        acc = vq[q];
                    } else {
                        acc.x += vq[q].x;
                        acc.y += vq[q].y;
                    }
                }
            }
        }
        if (cur >= 0) flush();
        if (live) {
            float2 *cr = carry + ((size_t)t * nitems + it) * 64 + c2;
            cr[0] = head;
            cr[32] = tail;
        }
    }
}

// fix rows (dst, j0, j1, slot0): out[t][dst] = carry[t][j0][slot0] + sum_{j0 < j <= j1} carry[t][j][0]
__global__ __launch_bounds__(256) void k_seg_fix(const float2 *__restrict__ carry, int64_t nitems,
                                                 const int4 *__restrict__ fix, int64_t nfix, int T,
                                                 float2 *__restrict__ out, int64_t out_rows, int acc_out) {
    const int lane = threadIdx.x & 63, t = lane >> 5, c2 = lane & 31;
    for (int64_t f = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); f < nfix; f += (int64_t)gridDim.x * 4) {
        if (t >= T) continue;
        const int4 x = fix[f];
        const float2 *ct = carry + (size_t)t * nitems * 64 + c2;
        float2 acc = ct[(size_t)x.y * 64 + x.w * 32];
#pragma unroll 8
        for (int j = x.y + 1; j <= x.z; j++) {
            const float2 v = ct[(size_t)j * 64];
            acc.x += v.x;
            acc.y += v.y;
        }
        float2 *o = out + ((size_t)t * out_rows + x.x) * 32 + c2;
        if (acc_out) {
            const float2 p = *o;
            *o = make_float2(p.x + acc.x, p.y + acc.y);
        } else {
            *o = acc;
        }
    }
}

// ---- dQ of the hot windows: scatter into LDS accumulators ------------------------------------
// The dQ gather above reads each 256-B dZ3 row once per tap (9x), from a table far larger than L2;
// the windows are very skewed (a bench rollout: the 192 most-entered of ~6k windows take ~85 % of
// the entries), so their dQ rows are accumulated in LDS instead, each dZ3 row read once:
//   workgroup = (tower t, channel slice c of DQH_SC channels, chunk of frames), one wave per tap;
//   the workgroup stages DQH_STEP dZ3 rows (its slice) and their frames' hot slots in LDS, and wave
//   `tap` adds row (u, p3) into acc[tap][hot slot of window wid(u, p3 + tap)] when that window is
//   hot.  Each accumulator has one writer wave, which adds in row order: the partial sums are
//   reproducible.  Partials per chunk go to `part` and k_dq_hot_reduce sums them in chunk order
//   into the hot windows' dQ rows.  Blocks are numbered so that the DQH_NS slice workgroups of one
//   (tower, chunk) share an XCD (block b runs on XCD b % 8): each dZ3 row is fetched into that
//   XCD's L2 once and read by the slices from there.
constexpr int DQH_SC = 16;                // channels per workgroup
constexpr int DQH_NS = 64 / DQH_SC;       // slices
constexpr int DQH_C4 = DQH_SC / 4;        // float4 per row slice
constexpr int DQH_STEP = 64;              // dZ3 rows per staged step
constexpr int DQH_FR = 8;                 // frames a step can touch (64 rows of 9)
constexpr int DQH_HSW = 32;               // int16 hot slots per frame row (25 used)
constexpr int DQH_THREADS = 9 * 64;
constexpr int DQH_MAXHOT = 192;

__global__ __launch_bounds__(DQH_THREADS) void k_dq_hot(const float4 *__restrict__ dZ3, int64_t U,
                                                      const int16_t *__restrict__ hs, int nhot, int chunks, int T,
                                                      float4 *__restrict__ part) {
    __shared__ float4 acc[9 * DQH_MAXHOT * DQH_C4];
    __shared__ float4 stg[2][DQH_STEP * DQH_C4];
    __shared__ int16_t hsl[2][DQH_FR * DQH_HSW];
    const int b = blockIdx.x;
    const int slice = (b >> 3) % DQH_NS;
    const int r = (b / (8 * DQH_NS)) * 8 + (b & 7);
    if (r >= T * chunks) return;  // grid padding: whole workgroup, before any barrier
    const int t = r % T, chunk = r / T;
    const int tid = threadIdx.x, lane = tid & 63, tap = tid >> 6;
    for (int i = tid; i < 9 * nhot * DQH_C4; i += DQH_THREADS) acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int64_t u0 = U * chunk / chunks, u1 = U * (chunk + 1) / chunks;
    const int64_t r0 = u0 * 9, r1 = u1 * 9;
    const int nsteps = (int)((r1 - r0 + DQH_STEP - 1) / DQH_STEP);
    const float4 *src = dZ3 + (size_t)t * U * 9 * 16 + slice * DQH_C4;
    // staging roles: threads [0, 256) one float4 of the rows, [256, 288) 16 B of hot slots
    float4 vreg = make_float4(0.f, 0.f, 0.f, 0.f);
    int4 hreg = make_int4(-1, -1, -1, -1);
    auto gload = [&](int k) {
        const int64_t s0 = r0 + (int64_t)k * DQH_STEP;
        if (tid < DQH_STEP * DQH_C4) {
            const int64_t row = s0 + tid / DQH_C4;
            vreg = row < r1 ? src[row * 16 + tid % DQH_C4] : make_float4(0.f, 0.f, 0.f, 0.f);
        } else if (tid < DQH_STEP * DQH_C4 + DQH_FR * DQH_HSW / 8) {
            const int j = tid - DQH_STEP * DQH_C4;
            const int64_t u = s0 / 9 + j / (DQH_HSW / 8);
            hreg = u < u1 ? reinterpret_cast<const int4 *>(hs + u * DQH_HSW)[j % (DQH_HSW / 8)]
                          : make_int4(-1, -1, -1, -1);
        }
    };
    auto swrite = [&](int buf) {
        if (tid < DQH_STEP * DQH_C4)
            stg[buf][tid] = vreg;
        else if (tid < DQH_STEP * DQH_C4 + DQH_FR * DQH_HSW / 8)
            reinterpret_cast<int4 *>(hsl[buf])[tid - DQH_STEP * DQH_C4] = hreg;
    };
    // per-lane constants: 16 rows per wave-instruction, lane = (row q, float4 c4 of the slice)
    const int q = lane / DQH_C4, c4 = lane % DQH_C4;
    const int ky = tap / 3, kx = tap - 3 * ky;
    float *accw = reinterpret_cast<float *>(acc) + (size_t)tap * nhot * DQH_SC + c4 * 4;
    if (nsteps > 0) {
        gload(0);
        swrite(0);
    }
    __syncthreads();
    for (int k = 0; k < nsteps; k++) {
        const int buf = k & 1;
        if (k + 1 < nsteps) gload(k + 1);
        const int64_t s0 = r0 + (int64_t)k * DQH_STEP;
        const int64_t ulo = s0 / 9;
#pragma unroll
        for (int it = 0; it < DQH_STEP / 16; it++) {
            const int lr = it * 16 + q;
            const int64_t row = s0 + lr;
            const int64_t u = row / 9;
            const int p3 = (int)(row - u * 9);
            const int p2 = (p3 / 3 + ky) * 5 + (p3 - 3 * (p3 / 3)) + kx;
            const int s = row < r1 ? hsl[buf][(int)(u - ulo) * DQH_HSW + p2] : -1;
            if (s >= 0) {
                const float4 v = stg[buf][lr * DQH_C4 + c4];
                float *a = accw + s * DQH_SC;
                atomicAdd(a + 0, v.x);
                atomicAdd(a + 1, v.y);
                atomicAdd(a + 2, v.z);
                atomicAdd(a + 3, v.w);
            }
        }
        if (k + 1 < nsteps) swrite(buf ^ 1);
        __syncthreads();
    }
    // partial sums of this (tower, chunk, slice): part[t][chunk][tap][slot][64 channels]
    for (int i = tid; i < 9 * nhot * DQH_C4; i += DQH_THREADS) {
        const int row = i / DQH_C4;  // tap * nhot + slot
        part[(((size_t)t * chunks + chunk) * 9 * nhot + row) * 16 + slice * DQH_C4 + i % DQH_C4] = acc[i];
    }
}

// dQ[t][hot_w[s] * 9 + tap] = sum over chunks (in order) of part[t][chunk][tap][s]
__global__ __launch_bounds__(256) void k_dq_hot_reduce(const float4 *__restrict__ part, int chunks, int nhot,
                                                       const int32_t *__restrict__ hot_w, int T,
                                                       float4 *__restrict__ out, int64_t out_rows) {
    const int64_t total = (int64_t)T * 9 * nhot * 16;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
        const int c = (int)(e & 15);
        const int64_t rr = e >> 4;  // (t, tap, s)
        const int s = (int)(rr % nhot), tap = (int)((rr / nhot) % 9), t = (int)(rr / (9 * nhot));
        const float4 *p = part + (((size_t)t * chunks * 9 + tap) * nhot + s) * 16 + c;
        float4 a = p[0];
        for (int ch = 1; ch < chunks; ch++) f4_add(a, p[(size_t)ch * 9 * nhot * 16]);
        out[((size_t)t * out_rows + (int64_t)hot_w[s] * 9 + tap) * 16 + c] = a;
    }
}

}  // namespace

int dq_hot_chunks(int64_t U, int T) {
    // one workgroup per CU: T * DQH_NS * chunks ~ 256, at least a few steps per chunk
    int c = 256 / (T * DQH_NS);
    while (c > 1 && U * 9 / c < 4 * DQH_STEP) c >>= 1;
    return c;
}
size_t dq_hot_part_floats(int64_t U, int T, int nhot) { return (size_t)T * dq_hot_chunks(U, T) * 9 * nhot * 64; }
int dq_hot_max() { return DQH_MAXHOT; }

hipError_t launch_dq_hot(const float *dZ3, int64_t U, const int16_t *hs, const int32_t *hot_w, int nhot, int T,
                         float *part, float *out, int64_t out_rows, hipStream_t s) {
    if (U <= 0 || nhot <= 0) return hipSuccess;
    const int chunks = dq_hot_chunks(U, T);
    const int work = T * chunks * DQH_NS;  // workgroups doing work
    const int grid = ((work + 8 * DQH_NS - 1) / (8 * DQH_NS)) * 8 * DQH_NS;
    hipLaunchKernelGGL(k_dq_hot, dim3(grid), dim3(DQH_THREADS), 0, s, reinterpret_cast<const float4 *>(dZ3), U, hs,
                       nhot, chunks, T, reinterpret_cast<float4 *>(part));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int64_t total = (int64_t)T * 9 * nhot * 16;
    const int g2 = (int)std::min<int64_t>((total + 255) / 256, 256 * 8);
    hipLaunchKernelGGL(k_dq_hot_reduce, dim3(g2), dim3(256), 0, s, reinterpret_cast<const float4 *>(part), chunks,
                       nhot, hot_w, T, reinterpret_cast<float4 *>(out), out_rows);
    return hipGetLastError();
}

hipError_t launch_window_lut(const int32_t *rows, int64_t nw, const float *tab, int T, float *Z2w, hipStream_t s) {
    const int64_t total = (int64_t)T * nw * 16;
    if (total <= 0) return hipSuccess;
    const int grid = (int)std::min<int64_t>((total + 255) / 256, 256 * 16);
    hipLaunchKernelGGL(k_window_lut, dim3(grid), dim3(256), 0, s, rows, nw, reinterpret_cast<const float4 *>(tab), T,
                       reinterpret_cast<float4 *>(Z2w));
    return hipGetLastError();
}

hipError_t launch_window_conv3(const float *Q, int64_t nw, const int32_t *wid, const int64_t *groups, int64_t n,
                               const float *b3, int T, float *Y3, hipStream_t s) {
    const int64_t total = (int64_t)T * n * 9 * 16;
    if (total <= 0) return hipSuccess;
    const int grid = (int)std::min<int64_t>((total + 255) / 256, 256 * 32);
    hipLaunchKernelGGL(k_window_conv3, dim3(grid), dim3(256), 0, s, reinterpret_cast<const float4 *>(Q), nw, wid,
                       groups, n, reinterpret_cast<const float4 *>(b3), T, reinterpret_cast<float4 *>(Y3));
    return hipGetLastError();
}

hipError_t launch_seg_sum(const float *src, int64_t src_rows, const int32_t *idx, const int32_t *key, int64_t nnz,
                          const int32_t *slot, int S, int64_t L, const int32_t *fix, int64_t nfix, int T, float *out,
                          int64_t out_rows, float *carry, int acc_out, hipStream_t s) {
    hipError_t e = acc_out ? hipSuccess : hipMemsetAsync(out, 0, sizeof(float) * 64 * (size_t)T * out_rows, s);
    if (e != hipSuccess || nnz <= 0) return e;
    const int64_t nitems = (nnz + L - 1) / L;
    const int grid = (int)std::min<int64_t>((nitems + SEG_WAVES - 1) / SEG_WAVES, 256 * 8);
    hipLaunchKernelGGL(k_seg_sum, dim3(grid), dim3(64 * SEG_WAVES), 0, s, reinterpret_cast<const float2 *>(src),
                       src_rows, idx, key, nnz, slot, S, L, nitems, T, reinterpret_cast<float2 *>(out), out_rows,
                       reinterpret_cast<float2 *>(carry), acc_out);
    e = hipGetLastError();
    if (e != hipSuccess || nfix <= 0) return e;
    const int gfix = (int)std::min<int64_t>((nfix + 3) / 4, 256 * 8);
    hipLaunchKernelGGL(k_seg_fix, dim3(gfix), dim3(256), 0, s, reinterpret_cast<const float2 *>(carry), nitems,
                       reinterpret_cast<const int4 *>(fix), nfix, T, reinterpret_cast<float2 *>(out), out_rows,
                       acc_out);
    return hipGetLastError();
}

}  // namespace merlin
