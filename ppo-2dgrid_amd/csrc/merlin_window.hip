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
#include <cstdlib>
#include <type_traits>

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
// ReLU backward (threshold_backward): g where y > 0, else 0
__device__ __forceinline__ float4 f4_mask(const float4 y, const float4 g) {
    return make_float4(y.x > 0.0f ? g.x : 0.0f, y.y > 0.0f ? g.y : 0.0f, y.z > 0.0f ? g.z : 0.0f,
                       y.w > 0.0f ? g.w : 0.0f);
}

// Z2w[t][w][c4] = sum_{k<16} T2[t][rows[w][k]][c4], taps in k_conv2_lut_fwd's order.  ALL only names the
// instantiation: 1 for the rollout's table over every possible window (5^9 rows, once per rollout), 0 for an
// update's windows (every minibatch) -- so a profile tells the two apart
// b2 (optional): relu(Z2w + b2[t]) written instead (conv2's bias and ReLU, as k_bias_relu computes them)
template <int ALL>
__global__ __launch_bounds__(256) void k_window_lut(const int32_t *__restrict__ rows, int64_t nw,
                                                    const float4 *__restrict__ tab, int T,
                                                    float4 *__restrict__ Z2w, const float4 *__restrict__ b2) {
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
        if (b2) {
            const float4 b = b2[t * 16 + c];
            acc = make_float4(relu_nan(acc.x + b.x), relu_nan(acc.y + b.y), relu_nan(acc.z + b.z),
                              relu_nan(acc.w + b.w));
        }
        Z2w[e] = acc;
    }
}

// Y3[t][u*9 + p3][c4] = relu(b3[t][c4] + sum_tap Q[t][wid[g*25 + p2(p3, tap)]][tap][c4]); 16
// consecutive lanes read one 256-B row of Q per tap.  bits (optional): bit ch of bits[t][u*9 + p3]
// = (Y3 channel ch > 0), the row's ReLU mask for the backward (16 lanes OR their nibbles together
// with xor shuffles inside the row's 16-lane group; the caller keeps the groups whole and converged).
// mx: max |Y3| per tower as float bits (merlin_h3.hip's operand scale), reduced by block_amax2.
// pl (h3 planes, round 5): the row is written as its h3 planes (merlin_internal.h h3_store4_pair; 256 B like the fp32
// row) scaled by psc = (2^e0, 2^e1, 2^(e0 + 11), 2^(e1 + 11)) of the two towers
__device__ __forceinline__ void conv3_row(const float4 *__restrict__ Q, int64_t nw, const int32_t *__restrict__ wid,
                                          const int64_t *__restrict__ groups, int64_t n,
                                          const float4 *__restrict__ b3, float4 *__restrict__ Y3,
                                          uint64_t *__restrict__ bits, bool amax, int64_t r, int c,
                                          uint32_t (&mx)[2], bool pl = false, float4 psc = float4{}) {
    const int64_t tu = r / 9;
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
    const float4 y = make_float4(relu_nan(acc.x + b.x), relu_nan(acc.y + b.y), relu_nan(acc.z + b.z),
                                 relu_nan(acc.w + b.w));
    if (pl)
        h3_store4_pair(reinterpret_cast<uint4 *>(Y3) + r * 16, c, y, t == 0 ? psc.x : psc.y, t == 0 ? psc.z : psc.w);
    else
        Y3[r * 16 + c] = y;
    if (amax) {
        const uint32_t m = std::max(std::max(__float_as_uint(y.x) & 0x7fffffffu, __float_as_uint(y.y) & 0x7fffffffu),
                                    std::max(__float_as_uint(y.z) & 0x7fffffffu, __float_as_uint(y.w) & 0x7fffffffu));
        if (t == 0) mx[0] = std::max(mx[0], m);
        else mx[1] = std::max(mx[1], m);
    }
    if (bits) {
        uint64_t w = (uint64_t)((y.x > 0.0f ? 1u : 0u) | (y.y > 0.0f ? 2u : 0u) | (y.z > 0.0f ? 4u : 0u) |
                                (y.w > 0.0f ? 8u : 0u))
                     << (4 * c);
#pragma unroll
        for (int off = 8; off >= 1; off >>= 1) w |= __shfl_xor(w, off);
        if (c == 0) bits[r] = w;
    }
}

// Every row: 16 lanes per row (rows are 16-lane aligned, so the groups are whole and converged).
__global__ __launch_bounds__(256) void k_window_conv3(const float4 *__restrict__ Q, int64_t nw,
                                                      const int32_t *__restrict__ wid,
                                                      const int64_t *__restrict__ groups, int64_t n,
                                                      const float4 *__restrict__ b3, int T,
                                                      float4 *__restrict__ Y3, uint64_t *__restrict__ bits,
                                                      uint32_t *__restrict__ amax) {
    const int64_t total = (int64_t)T * n * 9 * 16;
    uint32_t mx[2] = {0u, 0u};
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256)
        conv3_row(Q, nw, wid, groups, n, b3, Y3, bits, amax != nullptr, e >> 4, (int)(e & 15), mx);
    if (amax) block_amax2(mx, T, amax);
}

// Patch reuse: rows (u, p3) whose frames hold the same 5x5-tile patch at p3 read the same 9 windows at the same
// taps, so their outputs are bit-identical; rrow[u*9 + p3] names one row of the minibatch holding that patch (its
// representative, rrow[rep] = rep; merlin/windows.py builds it per minibatch).  Only the representatives are
// computed (~a third of the rows at the bench state): each wave takes 64 consecutive rows of the tower-major row
// space, packs its representatives into an LDS queue (ballot + prefix count) and computes them 4 at a time, 16
// lanes per row, so no lane idles on a copied row.  The block walks its 256-row spans in step (block-uniform trip
// count: the queue barriers are block barriers).
// bound (nullable, round 5): the rows are written as h3 planes scaled by the exponent of bound[t] (k_q_bound's bound
// on max Y3, known before any row is), amax unused
__global__ __launch_bounds__(256) void k_window_conv3_reps(const float4 *__restrict__ Q, int64_t nw,
                                                           const int32_t *__restrict__ wid,
                                                           const int64_t *__restrict__ groups, int64_t n,
                                                           const float4 *__restrict__ b3, int T,
                                                           float4 *__restrict__ Y3, uint64_t *__restrict__ bits,
                                                           uint32_t *__restrict__ amax,
                                                           const int32_t *__restrict__ rrow,
                                                           const uint32_t *__restrict__ bound) {
    __shared__ int64_t queue[4][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, q = lane >> 4, c = lane & 15;
    const unsigned long long below = (1ull << lane) - 1ull;
    const int64_t rows = n * 9, total = (int64_t)T * rows;
    uint32_t mx[2] = {0u, 0u};
    const bool pl = bound != nullptr;
    float4 psc = float4{};
    if (pl) {
        const int e0 = h3_exp(__hip_atomic_load(bound, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        const int e1 = T > 1 ? h3_exp(__hip_atomic_load(bound + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) : 0;
        psc = make_float4(pow2f(e0), pow2f(e1), pow2f(e0 + 11), pow2f(e1 + 11));
    }
    for (int64_t base = (int64_t)blockIdx.x * 256; base < total; base += (int64_t)gridDim.x * 256) {
        const int64_t i = base + threadIdx.x;
        bool rep = false;
        if (i < total) {
            const int64_t r = i - (i >= rows ? rows : 0);  // T <= 2 (the launcher checks)
            rep = rrow[r] == (int32_t)r;
        }
        const unsigned long long m = __ballot(rep);
        if (rep) queue[wv][__popcll(m & below)] = i;
        __syncthreads();
        const int cnt = __popcll(m);
        for (int p = q; p < cnt; p += 4) conv3_row(Q, nw, wid, groups, n, b3, Y3, bits, !pl && amax != nullptr,
                                                   queue[wv][p], c, mx, pl, psc);
        __syncthreads();
    }
    if (!pl && amax) block_amax2(mx, T, amax);
}

// A bound on max Y3 per tower before conv3 runs, so its representatives can be written as h3 planes directly (the
// plane scale must be known when a value is stored): Y3[u, p3][c] = relu(b3[c] + sum over taps of Q[w][tap][c]) <=
// relu(b3[c] + sum over taps of max_w Q[w][tap][c]), the maxima summed in conv3_row's order (fp32 addition is
// monotonic, so the bound holds for the rounded sums too).  A bound above the max only moves the planes' 2^26 dynamic
// range up by the ratio.
// ordered-uint image of a float: monotonic over all floats, NaN above +inf (so a NaN column max propagates)
__device__ __forceinline__ uint32_t f2ord(float f) {
    const uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t o) {
    return o == 0u ? -INFINITY : __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}
// part[t][b][k] = max over block b's windows of Q[t][w][k] (ordered images; k = tap * 64 + c): QB_BLOCKS blocks per
// tower over contiguous window ranges, 2 x 144 threads each (a half takes every other row, 8 rows' loads in flight),
// plain stores -- k_q_bound reduces over the blocks (same-address atomics from every block serialised: 152 us)
constexpr int QB_BLOCKS = 64;
__global__ __launch_bounds__(288) void k_q_colmax(const float4 *__restrict__ Q, int64_t nw, uint4 *__restrict__ part) {
    const int t = blockIdx.y, j = threadIdx.x % 144, h = threadIdx.x / 144;
    const int64_t per = (nw + QB_BLOCKS - 1) / QB_BLOCKS;
    const int64_t w0 = (int64_t)blockIdx.x * per, w1 = std::min<int64_t>(nw, w0 + per);
    const float4 *q = Q + (size_t)t * nw * 144 + j;
    uint32_t m[4] = {0u, 0u, 0u, 0u};
    for (int64_t w = w0 + h; w < w1; w += 16) {
        float4 v[8];
#pragma unroll
        for (int i = 0; i < 8; i++) v[i] = q[(size_t)std::min<int64_t>(w + 2 * i, w1 - 1) * 144];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            m[0] = max(m[0], f2ord(v[i].x));
            m[1] = max(m[1], f2ord(v[i].y));
            m[2] = max(m[2], f2ord(v[i].z));
            m[3] = max(m[3], f2ord(v[i].w));
        }
    }
    __shared__ uint4 hm[144];
    if (h == 1) hm[j] = make_uint4(m[0], m[1], m[2], m[3]);
    __syncthreads();
    if (h == 0) {
        const uint4 o = hm[j];
        part[((size_t)t * QB_BLOCKS + blockIdx.x) * 144 + j] =
            make_uint4(max(m[0], o.x), max(m[1], o.y), max(m[2], o.z), max(m[3], o.w));
    }
}
// bound[t] = float bits of max over c of relu(sum_tap colmax[t][tap][c] + b3[t][c]), colmax[t][k] the max over the
// blocks' partials (one block of 576 threads per tower)
__global__ __launch_bounds__(576) void k_q_bound(const uint32_t *__restrict__ part, const float *__restrict__ b3,
                                                 uint32_t *__restrict__ bound) {
    const int t = blockIdx.x, k = threadIdx.x;
    uint32_t m = 0u;
#pragma unroll 8
    for (int b = 0; b < QB_BLOCKS; b++) m = max(m, part[((size_t)t * QB_BLOCKS + b) * 576 + k]);
    __shared__ float col[576];
    col[k] = ord2f(m);
    __syncthreads();
    if (k < 64) {
        float acc = col[k];
#pragma unroll
        for (int tap = 1; tap < 9; tap++) acc += col[tap * 64 + k];
        uint32_t y = __float_as_uint(relu_nan(acc + b3[t * 64 + k])) & 0x7fffffffu;
        for (int o = 32; o > 0; o >>= 1) y = max(y, (uint32_t)__shfl_xor((int)y, o));
        if (k == 0) bound[t] = y;
    }
}

// The other rows from their representatives (after k_window_conv3_reps): with Y (16 lanes per row) the Y3 row and
// the mask word, without (one lane per row) the mask word only.
template <bool Y>
__global__ __launch_bounds__(256) void k_window_conv3_copy(float4 *Y3, uint64_t *bits, int64_t n, int T,
                                                           const int32_t *__restrict__ rrow) {
    const int64_t rows = n * 9, total = (int64_t)T * rows * (Y ? 16 : 1);
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
        const int64_t i = Y ? e >> 4 : e;
        const int64_t t0 = i >= rows ? rows : 0, r = i - t0;
        const int32_t src = rrow[r];
        if (src == (int32_t)r) continue;
        if (Y) Y3[e] = Y3[(t0 + src) * 16 + (e & 15)];
        if (bits && (!Y || (e & 15) == 0)) bits[i] = bits[t0 + src];
    }
}

// The acting path's conv3 from a table over every 3x3 tile window an observation can hold (built once per rollout
// from the fixed weights): Y3[t][u*9 + p3][c4] = relu(b3[t][c4] + sum_tap Qall[t][key(u, p2(p3, tap))][tap][c4]),
// computed from the frame's 49 class nibbles in registers, so conv2's lookups, conv3's im2col and its GEMM all drop
// out.  The agent's tile (class 4) is always at view cell (3, 6) (minigrid's egocentric view: the agent at the bottom
// centre), so a window holds it exactly when it covers that cell -- conv2 position (4, 1..3), the tile at local (2,
// 3 - wx) -- and nowhere else; every other tile is one of the four classes 0..3.  Keys (merlin/windows.py
// compact_window_keys): a window away from the agent = its 9 classes in base 4 (tile (0, 0) most significant,
// 4^9 keys); a window over the agent = 4^9 + (wx - 1) 4^8 + its other 8 classes in base 4.  458,752 keys instead of
// all 5^9 = 1,953,125 class patterns: a 4.3x smaller table (2.1 GB for both towers), built in that fraction of the
// time.  (Valid observations only: a class-4 tile elsewhere is read as class 3, so a frame that is not an observation
// -- no agent tile at (3, 6), or one elsewhere -- raises MERLIN_DEVERR_BAD_TILE in `err`, merlin_tower_errors.)
constexpr int64_t ALL_WINDOWS = 458752;  // 4^9 + 3 * 4^8
// The 25 window keys of a frame are computed once per block (CC_F frames per block, keys in LDS), not by each of the
// 16 lanes of each of the 9 output rows that read them: round 4's per-lane key arithmetic (81 class lookups per lane)
// made the kernel VALU-bound (35 us per 4096-frame step; 57 us once the compact key's slot skipping was added).
constexpr int CC_F = 4;  // 1,024 blocks of 256 threads at 4,096 frames: ~4.5 outputs (9 row gathers each) per thread
template <int CC_U>
__global__ __launch_bounds__(256) void k_codes_conv3(const uint32_t *__restrict__ codes, int64_t n,
                                                     const float4 *__restrict__ Q, const float4 *__restrict__ b3,
                                                     int T, float4 *__restrict__ Y3, uint32_t *__restrict__ amax,
                                                     uint32_t *__restrict__ err) {
    __shared__ uint32_t keys[CC_F][25];
    bool bad = false;  // a tile this compact table cannot hold (see above)
    uint32_t mx[2] = {0u, 0u};  // max |Y3| per tower as float bits (fc1's h3 operand scale), when amax != null
    for (int64_t f0 = (int64_t)blockIdx.x * CC_F; f0 < n; f0 += (int64_t)gridDim.x * CC_F) {
        const int nf = (int)std::min<int64_t>(CC_F, n - f0);
        for (int e = threadIdx.x; e < nf * 25; e += 256) {
            const int f = e / 25, p = e - f * 25, wy = p / 5, wx = p - wy * 5;
            const uint4 w0 = *reinterpret_cast<const uint4 *>(codes + (f0 + f) * 8);
            const uint4 w1 = *reinterpret_cast<const uint4 *>(codes + (f0 + f) * 8 + 4);
            const uint32_t w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
            const bool agent = wy == 4 && wx >= 1 && wx <= 3;
            const int skip = agent ? 9 - wx : -1;  // local slot 3 * 2 + (3 - wx) of the agent's tile
            uint32_t key = 0;
#pragma unroll
            for (int a = 0; a < 3; a++)
#pragma unroll
                for (int b = 0; b < 3; b++) {
                    const int cell = (wy + a) * 7 + wx + b;
                    const uint32_t raw = (w[cell >> 3] >> (4 * (cell & 7))) & 15u;
                    bad |= cell == 45 ? raw != 4u : raw > 3u;  // the agent at view cell (3, 6), nowhere else
                    const uint32_t c = min(raw, 3u);  // 0..3: see above
                    if (3 * a + b != skip) key = key * 4u + c;
                }
            if (agent) key += 262144u + (uint32_t)(wx - 1) * 65536u;
            keys[f][p] = key;
        }
        __syncthreads();
        const int per_t = nf * 9 * 16;
        // CC_U outputs per thread and round, all their 9 CC_U row gathers issued before any is summed (outputs past
        // the block's end gather the round's first output's rows and are dropped): ~4.5 outputs per thread took 4-5
        // dependent gather round trips one after the other
        for (int e0 = threadIdx.x; e0 < T * per_t; e0 += CC_U * 256) {
            float4 v[CC_U][9];
            int tt[CC_U], cc[CC_U], ff[CC_U], pp[CC_U];
#pragma unroll
            for (int h = 0; h < CC_U; h++) {
                const int e = e0 + h * 256 < T * per_t ? e0 + h * 256 : e0;
                const int t = e / per_t, r = e - t * per_t, c = r & 15, fp = r >> 4, f = fp / 9, p3 = fp - f * 9;
                const int oy = p3 / 3, ox = p3 - oy * 3;
                const float4 *qt = Q + (size_t)t * ALL_WINDOWS * 9 * 16 + c;
#pragma unroll
                for (int tap = 0; tap < 9; tap++) {
                    const int ky = tap / 3, kx = tap - ky * 3;
                    v[h][tap] = qt[((size_t)keys[f][(oy + ky) * 5 + ox + kx] * 9 + tap) * 16];
                }
                tt[h] = t;
                cc[h] = c;
                ff[h] = f;
                pp[h] = p3;
            }
#pragma unroll
            for (int h = 0; h < CC_U; h++) {
                if (e0 + h * 256 >= T * per_t) break;
                const int t = tt[h], c = cc[h];
                float4 acc = v[h][0];
#pragma unroll
                for (int tap = 1; tap < 9; tap++) f4_add(acc, v[h][tap]);
                const float4 b = b3[t * 16 + c];
                const float4 y = make_float4(relu_nan(acc.x + b.x), relu_nan(acc.y + b.y), relu_nan(acc.z + b.z),
                                             relu_nan(acc.w + b.w));
                Y3[(((size_t)t * n + f0 + ff[h]) * 9 + pp[h]) * 16 + c] = y;
                if (amax) {
                    const uint32_t m = std::max(std::max(__float_as_uint(y.x) & 0x7fffffffu, __float_as_uint(y.y) & 0x7fffffffu),
                                                std::max(__float_as_uint(y.z) & 0x7fffffffu, __float_as_uint(y.w) & 0x7fffffffu));
                    if (t == 0) mx[0] = std::max(mx[0], m);
                    else mx[1] = std::max(mx[1], m);
                }
            }
        }
        __syncthreads();
    }
    if (amax) block_amax2(mx, T, amax);
    if (bad && err) atomicOr(err, MERLIN_DEVERR_BAD_TILE);
}

// One wave per item of L entries; lane = (tower t, entry parity q, float4 column c): one wave
// load reads the 256-B rows of two entries in both towers (1 KB, 16 B per lane).  The wave loads
// 64 entries' (idx, key) at a time, resolves their source rows (through slot[] when given: -1 = not
// in this minibatch) and walks the valid ones in order in rounds of two, SEG_UNROLL rounds of row
// loads in flight (issued unconditionally: a select around a load would make hipcc wait for each
// load in turn).  Lanes q = 0 / 1 keep partial sums of the even / odd entries of the current
// destination; when the key changes the two are added (a fixed xor-16 exchange) and the
// destination's sum is flushed.  The item's first / last destination, when it continues in the
// neighbouring item, goes to carry[t][item][0 / 1] instead of out.  With acc_out the sums are
// added to out (one writer per destination per launch), so a list split by source block into
// several launches accumulates in block order.  MASK: each source row is first multiplied by the
// ReLU mask of the same row of `mask` (the forward's output), i.e. the sums are of
// threshold_backward(src, mask) rows, never materialised.  MASK 2: the same mask as one 64-bit
// word per row (bit ch = mask channel ch > 0, as k_window_conv3 writes it): 8 B per row instead
// of 256.
// mark (optional): mark[key] = key for every entry not skipped -- the destinations this launch sums into, as a
// slot map for a following pass over them (the caller presets -1).
// ROLE only names the instantiation (rocprofv3 tells the passes of conv3's backward apart by it):
// 0 generic, 1 R (patch sums), 2 S (band sums), 3 dQ (window sums), 4 dT2 (table rows)
constexpr int SEG_WAVES = 4, SEG_UNROLL = 8;

// A carry word: 8 bytes (a float2 of a row), read at agent scope (sc1, past this CU's L1) when the carries were
// published inside the same launch by other workgroups, plainly otherwise.
template <bool SC1>
__device__ __forceinline__ float2 carry_load(const float2 *p) {
    if constexpr (SC1) {
        const uint64_t v = __hip_atomic_load(reinterpret_cast<const uint64_t *>(p), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        return __builtin_bit_cast(float2, v);
    } else {
        return *p;
    }
}

// one fix row (dst, j0, j1, slot0) by one wave, lane = (tower t, float2 column c2):
// out[t][dst] (+)= carry[t][j0][slot0] + sum_{j0 < j <= j1} carry[t][j][0], in that order
template <bool SC1>
__device__ __forceinline__ void seg_fix_row(const float2 *__restrict__ carry, int64_t nitems, int4 x, int T,
                                            float2 *__restrict__ out, int64_t out_rows, int acc_out, int lane) {
    const int t = lane >> 5, c2 = lane & 31;
    if (t >= T) return;
    const float2 *ct = carry + (size_t)t * nitems * 64 + c2;
    float2 acc = carry_load<SC1>(ct + (size_t)x.y * 64 + x.w * 32);
    // a hot destination spans hundreds of items: four independent partial sums (items
    // j0+1+4i+q go to partial q) keep 16 loads in flight instead of one dependent chain;
    // the partials join in a fixed order, so the result stays bitwise reproducible
    float2 a[4] = {make_float2(0.f, 0.f), make_float2(0.f, 0.f), make_float2(0.f, 0.f), make_float2(0.f, 0.f)};
    int j = x.y + 1;
    for (; j + 15 <= x.z; j += 16) {
        float2 v[16];
#pragma unroll
        for (int u = 0; u < 16; u++) v[u] = carry_load<SC1>(ct + (size_t)(j + u) * 64);
#pragma unroll
        for (int u = 0; u < 16; u++) {
            a[u & 3].x += v[u].x;
            a[u & 3].y += v[u].y;
        }
    }
    for (; j <= x.z; j += 4) {  // static partial indices (a dynamic a[q] would live in scratch)
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (j + u <= x.z) {
                const float2 v = carry_load<SC1>(ct + (size_t)(j + u) * 64);
                a[u].x += v.x;
                a[u].y += v.y;
            }
        }
    }
    acc.x += (a[0].x + a[1].x) + (a[2].x + a[3].x);
    acc.y += (a[0].y + a[1].y) + (a[2].y + a[3].y);
    float2 *o = out + ((size_t)t * out_rows + x.x) * 32 + c2;
    if (acc_out) {
        const float2 p = *o;
        *o = make_float2(p.x + acc.x, p.y + acc.y);
    } else {
        *o = acc;
    }
}
// A64 (opt-in, MERLIN_SEG_F64=1): the per-destination partial sums of an item accumulate in f64 and are rounded to
// fp32 once, when flushed (the carries are then added in fp32, k_seg_fix's order).  Measured in round 6: the benched
// update's first-step gradient is within ~3e-7 of float64 either way (tests/test_gpu_update_grad.py, both runs in
// profiles/r06c_grad*.log), and the f64 adds cost the R pass 16 us per minibatch (profiles/r06c_ab*.log), so fp32
// accumulation stays the default.
struct SegAcc64 {
    double x, y, z, w;
};
__device__ __forceinline__ void seg_zero(float4 &a) { a = make_float4(0.0f, 0.0f, 0.0f, 0.0f); }
__device__ __forceinline__ void seg_zero(SegAcc64 &a) { a = SegAcc64{0.0, 0.0, 0.0, 0.0}; }
__device__ __forceinline__ void seg_add(float4 &a, const float4 v) { f4_add(a, v); }
__device__ __forceinline__ void seg_add(SegAcc64 &a, const float4 v) {
    a.x += (double)v.x;
    a.y += (double)v.y;
    a.z += (double)v.z;
    a.w += (double)v.w;
}
// the two parity lanes' partials of a destination added (lanes q and q ^ 1 compute the same sum), as fp32
__device__ __forceinline__ float4 seg_pair(const float4 a) {
    return make_float4(a.x + __shfl_xor(a.x, 16), a.y + __shfl_xor(a.y, 16), a.z + __shfl_xor(a.z, 16),
                       a.w + __shfl_xor(a.w, 16));
}
__device__ __forceinline__ float4 seg_pair(const SegAcc64 a) {
    return make_float4((float)(a.x + __shfl_xor(a.x, 16)), (float)(a.y + __shfl_xor(a.y, 16)),
                       (float)(a.z + __shfl_xor(a.z, 16)), (float)(a.w + __shfl_xor(a.w, 16)));
}

template <int MASK, int ROLE, bool A64 = true>
__global__ __launch_bounds__(64 * SEG_WAVES) void k_seg_sum(const float4 *__restrict__ src,
                                                           const void *__restrict__ mask, int64_t src_rows,
                                                           const int32_t *__restrict__ idx,
                                                           const int32_t *__restrict__ key, int64_t nnz,
                                                           const int32_t *__restrict__ slot, int S, int64_t L,
                                                           int64_t nitems, int T, float4 *__restrict__ out,
                                                           int64_t out_rows, float4 *__restrict__ carry,
                                                           int acc_out, int32_t *__restrict__ mark,
                                                           const int4 *__restrict__ fix,
                                                           const int32_t *__restrict__ hfix,
                                                           int32_t *__restrict__ cnt,
                                                           const int32_t *__restrict__ mrow) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int t = lane >> 5, q = (lane >> 4) & 1, c = lane & 15;
    const bool live = t < T;
    const float4 *srct = src + (size_t)(live ? t : 0) * src_rows * 16 + c;
    const float4 *maskt =
        MASK == 1 ? static_cast<const float4 *>(mask) + (size_t)(live ? t : 0) * src_rows * 16 + c : nullptr;
    // MASK 3: the bit words of MASK 2 read through a row map, bits[mrow[row]] (conv3's patch representatives: rows of
    // one patch share their ReLU mask, only the representatives' words are written)
    const uint64_t *bitst = MASK >= 2 ? static_cast<const uint64_t *>(mask) + (size_t)(live ? t : 0) * src_rows
                                      : nullptr;
    const float4 zero = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    for (int64_t it = (int64_t)blockIdx.x * SEG_WAVES + wv; it < nitems; it += (int64_t)gridDim.x * SEG_WAVES) {
        const int64_t e0 = it * L, e1 = std::min<int64_t>(nnz, e0 + L);
        const int kfirst = key[e0], klast = key[e1 - 1];
        const bool xfirst = e0 > 0 && key[e0 - 1] == kfirst;
        const bool xlast = e1 < nnz && key[e1] == klast;
        const bool to_head_last = kfirst == klast && xlast;
        float4 head = zero, tail = zero;
        std::conditional_t<A64, SegAcc64, float4> acc;
        seg_zero(acc);
        int cur = -1;
        auto flush = [&]() {  // wave-uniform call sites (keys are uniform)
            const float4 o = seg_pair(acc);
            if (cur == kfirst && (xfirst || to_head_last))
                head = o;
            else if (cur == klast && xlast)
                tail = o;
            else if (live && q == 0) {
                float4 *d = out + ((size_t)t * out_rows + cur) * 16 + c;
                if (acc_out) {
                    const float4 p = *d;
                    *d = make_float4(p.x + o.x, p.y + o.y, p.z + o.z, p.w + o.w);
                } else {
                    *d = o;
                }
            }
        };
        // the item's entries in chunks of 64 (one per lane), software-pipelined: while chunk c's rows are summed,
        // chunk c+1's slot lookups and chunk c+2's (idx, key) are in flight (a chunk's three dependent reads --
        // entry, slot, row -- used to run back to back).  Reads are clamped into the item, never branched around.
        // (the lane's validity is kept apart from the loaded key and applied where the key is used: a select
        // right behind a load makes the wave wait for it there)
        auto fetch = [&](int64_t b, int &v, int &k) {
            const int64_t e = std::min<int64_t>(b + lane, e1 - 1);
            v = idx[e];
            k = key[e];
        };
        int v0, kc0, v1 = 0, kc1 = 0;
        fetch(e0, v0, kc0);
        int sl0 = slot ? slot[v0 / S] : 0;
        if (e0 + 64 < e1) fetch(e0 + 64, v1, kc1);
        for (int64_t base = e0; base < e1; base += 64) {
            const int k = base + lane < e1 ? kc0 : -1;
            const int row = k < 0 ? -1 : !slot ? v0 : sl0 >= 0 ? sl0 * S + (v0 - (v0 / S) * S) : -1;
            if (mark && row >= 0) mark[k] = k;  // destinations that receive a sum (same-value stores)
            const int sl1 = slot ? slot[v1 / S] : 0;
            int v2 = 0, kc2 = 0;
            if (base + 128 < e1) fetch(base + 128, v2, kc2);
            v0 = v1;
            kc0 = kc1;
            sl0 = sl1;
            v1 = v2;
            kc1 = kc2;
            unsigned long long m = __ballot(row >= 0);
            while (m) {
                int rq[SEG_UNROLL], k0[SEG_UNROLL], k1[SEG_UNROLL];
#pragma unroll
                for (int u = 0; u < SEG_UNROLL; u++) {
                    const int j0 = m ? __builtin_ctzll(m) : -1;  // wave-uniform
                    if (m) m &= m - 1;
                    const int j1 = m ? __builtin_ctzll(m) : -1;
                    if (m) m &= m - 1;
                    const int r0 = j0 >= 0 ? __shfl(row, j0) : 0;
                    const int r1 = j1 >= 0 ? __shfl(row, j1) : 0;
                    k0[u] = j0 >= 0 ? __shfl(k, j0) : -1;
                    k1[u] = j1 >= 0 ? __shfl(k, j1) : -1;
                    rq[u] = q ? r1 : r0;
                }
                float4 vq[SEG_UNROLL];
#pragma unroll
                for (int u = 0; u < SEG_UNROLL; u++) vq[u] = srct[(size_t)rq[u] * 16];
                if constexpr (MASK == 1) {
                    float4 mq[SEG_UNROLL];
#pragma unroll
                    for (int u = 0; u < SEG_UNROLL; u++) mq[u] = maskt[(size_t)rq[u] * 16];
#pragma unroll
                    for (int u = 0; u < SEG_UNROLL; u++) vq[u] = f4_mask(mq[u], vq[u]);
                } else if constexpr (MASK >= 2) {
                    uint32_t mb[SEG_UNROLL];
#pragma unroll
                    for (int u = 0; u < SEG_UNROLL; u++)
                        mb[u] = (uint32_t)(bitst[MASK == 3 ? mrow[rq[u]] : rq[u]] >> (4 * c));
#pragma unroll
                    for (int u = 0; u < SEG_UNROLL; u++)
                        vq[u] = make_float4(mb[u] & 1u ? vq[u].x : 0.0f, mb[u] & 2u ? vq[u].y : 0.0f,
                                            mb[u] & 4u ? vq[u].z : 0.0f, mb[u] & 8u ? vq[u].w : 0.0f);
                }
#pragma unroll
                for (int u = 0; u < SEG_UNROLL; u++) {
                    if (k0[u] < 0) break;
                    if (k0[u] != cur) {
                        if (cur >= 0) flush();
                        cur = k0[u];
                        seg_zero(acc);
                    }
                    if (q == 0) seg_add(acc, vq[u]);
                    if (k1[u] < 0) break;
                    if (k1[u] != cur) {
                        flush();
                        cur = k1[u];
                        seg_zero(acc);
                    }
                    if (q == 1) seg_add(acc, vq[u]);
                }
            }
        }
        if (cur >= 0) flush();
        if (!cnt) {
            if (live && q == 0) {
                float4 *cr = carry + ((size_t)t * nitems + it) * 32 + c;
                cr[0] = head;
                cr[16] = tail;
            }
            continue;
        }
        // in-launch fix-up (cnt != null): publish the carries write-through (8-byte agent-scope stores: sc1, no
        // release fence), drain, then count this item in at the fix rows it takes part in -- the one its first
        // destination started at (hfix, when that destination continues from an earlier item) and its own (when
        // its last destination starts here and continues).  The item that completes a row's count sums the row's
        // carries in k_seg_fix's order with agent-scope loads, so the result does not depend on which item is
        // last, and resets the counter for the next launch.
        if (live && q == 0) {
            uint64_t *cr = reinterpret_cast<uint64_t *>(carry + ((size_t)t * nitems + it) * 32 + c);
            __hip_atomic_store(cr, __builtin_bit_cast(uint64_t, make_float2(head.x, head.y)), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(cr + 1, __builtin_bit_cast(uint64_t, make_float2(head.z, head.w)), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(cr + 32, __builtin_bit_cast(uint64_t, make_float2(tail.x, tail.y)), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(cr + 33, __builtin_bit_cast(uint64_t, make_float2(tail.z, tail.w)), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        // Memory-model note: the publish / count pair is relaxed on purpose.  Its ordering rests on two
        // gfx950 facts -- vector stores are counted by vmcnt, so the wait below retires the carry stores before the
        // counter's fetch_add issues, and agent-scope (sc1) stores and loads go through to the coherence point that
        // every XCD's L2 sees -- not on a release / acquire pair: an agent-scope release here is an L2 write-back per
        // item (buffer_wbl2), measured in round 3 at 265 -> 495 ms per update.  Other targets are refused below.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "k_seg_sum's in-launch fix-ups rely on gfx950's vmcnt-counted stores and sc1 write-through (see above)"
#endif
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int f0 = hfix[it];
        const int f1 = fix[it].x >= 0 ? (int)it : -1;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int f = k == 0 ? f0 : f1;  // wave-uniform
            if (f < 0) continue;
            const int4 x = fix[f];
            int old = 0;
            if (lane == 0) old = __hip_atomic_fetch_add(cnt + f, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            old = __shfl(old, 0);
            if (old != x.z - x.y) continue;  // not the last of the row's j1 - j0 + 1 items
            if (lane == 0) __hip_atomic_store(cnt + f, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            seg_fix_row<true>(reinterpret_cast<const float2 *>(carry), nitems, x, T, reinterpret_cast<float2 *>(out),
                              out_rows, acc_out, lane);
        }
    }
}

// fix rows (dst, j0, j1, slot0): out[t][dst] = carry[t][j0][slot0] + sum_{j0 < j <= j1} carry[t][j][0];
// rows with dst < 0 hold nothing (merlin/windows.py SegmentPlan: one row per item)
template <int ROLE>
__global__ __launch_bounds__(256) void k_seg_fix(const float2 *__restrict__ carry, int64_t nitems,
                                                 const int4 *__restrict__ fix, int64_t nfix, int T,
                                                 float2 *__restrict__ out, int64_t out_rows, int acc_out) {
    const int lane = threadIdx.x & 63;
    for (int64_t f = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); f < nfix; f += (int64_t)gridDim.x * 4) {
        const int4 x = fix[f];
        if (x.x < 0) continue;
        seg_fix_row<false>(carry, nitems, x, T, out, out_rows, acc_out, lane);
    }
}

// The minibatches' live-patch maps for a whole update (merlin/windows.py WindowPlan._bulk_minibatches): group g
// (minibatch m = key / F, frame key % F, position j = g - goff[m] in its minibatch), position p3 -> patch k =
// kid[frame][p3]: kmap[m][k] = k (the S pass's slot map; racing writers store the same value) and rmap[m][k] = j*9 +
// p3 (one row of the minibatch holding k: any writer wins, they compute the same bits); then, after that launch,
// rep_row[g*9 + p3] = rmap[m][k].  One thread per (group, position), 32-bit indices throughout.
template <int PASS>
__global__ __launch_bounds__(256) void k_patch_maps(const int32_t *__restrict__ kid, const int64_t *__restrict__ gkey,
                                                    int64_t G, int64_t F, const int64_t *__restrict__ goff, int K,
                                                    int32_t *__restrict__ kmap, int32_t *__restrict__ rmap,
                                                    int32_t *__restrict__ rep_row) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= G * 9) return;
    const int64_t g = e / 9;
    const int p3 = (int)(e - g * 9);
    const int64_t key = gkey[g], m = key / F, frame = key - m * F;
    const int32_t k = kid[frame * 9 + p3];
    const int64_t at = m * K + k;
    if (PASS == 0) {  // (reading kmap first and writing only unmarked slots: 2,041 vs 1,283 us, profiles/r05i_*)
        kmap[at] = k;
        rmap[at] = (int32_t)((g - goff[m]) * 9 + p3);
    } else {
        rep_row[e] = rmap[at];
    }
}

}  // namespace

hipError_t launch_patch_maps(const int32_t *kid, const int64_t *gkey, int64_t G, int64_t F, const int64_t *goff, int K,
                             int32_t *kmap, int32_t *rmap, int32_t *rep_row, hipStream_t s) {
    if (G <= 0) return hipSuccess;
    const dim3 grid((unsigned)((G * 9 + 255) / 256));
    hipLaunchKernelGGL(k_patch_maps<0>, grid, dim3(256), 0, s, kid, gkey, G, F, goff, K, kmap, rmap, rep_row);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_patch_maps<1>, grid, dim3(256), 0, s, kid, gkey, G, F, goff, K, kmap, rmap, rep_row);
    return hipGetLastError();
}

hipError_t launch_window_lut(const int32_t *rows, int64_t nw, const float *tab, int T, float *Z2w, hipStream_t s,
                             const float *b2) {
    const int64_t total = (int64_t)T * nw * 16;
    if (total <= 0) return hipSuccess;
    const int grid = (int)std::min<int64_t>((total + 255) / 256, 256 * 16);
    if (nw == ALL_WINDOWS)  // merlin_tower_all_windows(): the acting path's table
        hipLaunchKernelGGL(k_window_lut<1>, dim3(grid), dim3(256), 0, s, rows, nw, reinterpret_cast<const float4 *>(tab),
                           T, reinterpret_cast<float4 *>(Z2w), reinterpret_cast<const float4 *>(b2));
    else
        hipLaunchKernelGGL(k_window_lut<0>, dim3(grid), dim3(256), 0, s, rows, nw, reinterpret_cast<const float4 *>(tab),
                           T, reinterpret_cast<float4 *>(Z2w), reinterpret_cast<const float4 *>(b2));
    return hipGetLastError();
}

hipError_t launch_window_conv3(const float *Q, int64_t nw, const int32_t *wid, const int64_t *groups, int64_t n,
                               const float *b3, int T, float *Y3, uint64_t *bits, uint32_t *amax, const int32_t *rrow,
                               int copy, hipStream_t s, uint32_t *colmax, uint32_t *bound) {
    const int64_t total = (int64_t)T * n * 9 * 16;
    if (total <= 0) return hipSuccess;
    const int grid = (int)std::min<int64_t>((total + 255) / 256, 256 * 32);
    const float4 *q = reinterpret_cast<const float4 *>(Q), *b = reinterpret_cast<const float4 *>(b3);
    float4 *y = reinterpret_cast<float4 *>(Y3);
    if (!rrow) {
        hipLaunchKernelGGL(k_window_conv3, dim3(grid), dim3(256), 0, s, q, nw, wid, groups, n, b, T, y, bits, amax);
        return hipGetLastError();
    }
    if (T > 2) return hipErrorInvalidValue;
    const int rgrid = (int)std::min<int64_t>((total / 16 + 255) / 256, 256 * 32);
    if (bound) {  // planes: the representatives only, scaled by the bound from Q's column maxima
        if (!colmax || (copy & 7) || nw <= 0) return hipErrorInvalidValue;
        hipLaunchKernelGGL(k_q_colmax, dim3(QB_BLOCKS, T), dim3(288), 0, s, q, nw, reinterpret_cast<uint4 *>(colmax));
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_q_bound, dim3(T), dim3(576), 0, s, colmax, b3, bound);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_window_conv3_reps, dim3(rgrid), dim3(256), 0, s, q, nw, wid, groups, n, b, T, y, bits,
                           nullptr, rrow, bound);
        return hipGetLastError();
    }
    if (!(copy & 4)) {  // copy bit 2: the copies only (the representatives were computed by an earlier call)
        hipLaunchKernelGGL(k_window_conv3_reps, dim3(rgrid), dim3(256), 0, s, q, nw, wid, groups, n, b, T, y, bits,
                           amax, rrow, nullptr);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (!(copy & 3)) return hipSuccess;
    if (copy & 1)
        hipLaunchKernelGGL(k_window_conv3_copy<true>, dim3(grid), dim3(256), 0, s, y, (copy & 2) ? bits : nullptr, n,
                           T, rrow);
    else if (bits)
        hipLaunchKernelGGL(k_window_conv3_copy<false>, dim3(rgrid), dim3(256), 0, s, y, bits, n, T, rrow);
    return hipGetLastError();
}

hipError_t launch_codes_conv3(const uint32_t *codes, int64_t n, const float *Q, const float *b3, int T, float *Y3,
                              uint32_t *amax, uint32_t *err, hipStream_t s) {
    const int64_t total = (int64_t)T * n * 9 * 16;
    if (total <= 0) return hipSuccess;
    const int grid = (int)std::min<int64_t>((n + CC_F - 1) / CC_F, 256 * 32);
    // 3 outputs per thread and gather round: at the bench state 20.85 ms per rollout against 21.85 for one output's
    // gathers at a time, 21.4 for 2 and 21.7 for 5 (scripts/probe_rollout.py, profiles/r06ab_ccu*.log)
#define CC_GO(U)                                                                                                  \
    hipLaunchKernelGGL(k_codes_conv3<U>, dim3(grid), dim3(256), 0, s, codes, n, reinterpret_cast<const float4 *>(Q), \
                       reinterpret_cast<const float4 *>(b3), T, reinterpret_cast<float4 *>(Y3), amax, err)
    CC_GO(3);
#undef CC_GO
    return hipGetLastError();
}

namespace {
bool seg_f32() {  // fp32 accumulation unless MERLIN_SEG_F64=1 (read once per process)
    static const bool v = [] {
        const char *e = getenv("MERLIN_SEG_F64");
        return !(e && e[0] == '1');
    }();
    return v;
}
template <int ROLE>
hipError_t seg_launch(const float *src, const void *mask, int mask_bits, int64_t src_rows, const int32_t *idx,
                      const int32_t *key, int64_t nnz, const int32_t *slot, int S, int64_t L, const int32_t *fix,
                      int64_t nfix, int T, float *out, int64_t out_rows, float *carry, int acc_out, int32_t *mark,
                      const int32_t *hfix, int32_t *cnt, const int32_t *mrow, hipStream_t s) {
    const int64_t nitems = (nnz + L - 1) / L;
    if (cnt && nfix != nitems) return hipErrorInvalidValue;  // in-launch fix-ups: one fix row per item
    const int grid = (int)std::min<int64_t>((nitems + SEG_WAVES - 1) / SEG_WAVES, 256 * 8);
    const int4 *fx = cnt ? reinterpret_cast<const int4 *>(fix) : nullptr;
    const int32_t *hf = cnt ? hfix : nullptr;
    const float4 *s4 = reinterpret_cast<const float4 *>(src);
    float4 *o4 = reinterpret_cast<float4 *>(out), *c4 = reinterpret_cast<float4 *>(carry);
#define SEG_GO(MASK_, A64_, MP_, RP_)                                                                                \
    hipLaunchKernelGGL((k_seg_sum<MASK_, ROLE, A64_>), dim3(grid), dim3(64 * SEG_WAVES), 0, s, s4, MP_, src_rows, idx, \
                       key, nnz, slot, S, L, nitems, T, o4, out_rows, c4, acc_out, mark, fx, hf, cnt, RP_)
#define SEG_GO2(MASK_, MP_, RP_)       \
    do {                               \
        if (seg_f32())                 \
            SEG_GO(MASK_, false, MP_, RP_); \
        else                           \
            SEG_GO(MASK_, true, MP_, RP_);  \
    } while (0)
    if (mask && mask_bits && mrow)
        SEG_GO2(3, mask, mrow);
    else if (mask && mask_bits)
        SEG_GO2(2, mask, nullptr);
    else if (mask)
        SEG_GO2(1, mask, nullptr);
    else
        SEG_GO2(0, nullptr, nullptr);
#undef SEG_GO2
#undef SEG_GO
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || nfix <= 0 || cnt) return e;
    const int gfix = (int)std::min<int64_t>((nfix + 3) / 4, 256 * 8);
    hipLaunchKernelGGL(k_seg_fix<ROLE>, dim3(gfix), dim3(256), 0, s, reinterpret_cast<const float2 *>(carry), nitems,
                       reinterpret_cast<const int4 *>(fix), nfix, T, reinterpret_cast<float2 *>(out), out_rows,
                       acc_out);
    return hipGetLastError();
}
}  // namespace

hipError_t launch_seg_sum(const float *src, const void *mask, int mask_bits, int64_t src_rows, const int32_t *idx,
                          const int32_t *key, int64_t nnz, const int32_t *slot, int S, int64_t L, const int32_t *fix,
                          int64_t nfix, int T, float *out, int64_t out_rows, float *carry, int acc_out, int fill,
                          int role, int32_t *mark, const int32_t *hfix, int32_t *cnt, hipStream_t s,
                          const int32_t *mrow) {
    hipError_t e = (acc_out || !fill) ? hipSuccess
                                      : zero_async(out, sizeof(float) * 64 * (size_t)T * out_rows, s);
    if (e != hipSuccess || nnz <= 0) return e;
#define SEG_ROLE(R) \
    seg_launch<R>(src, mask, mask_bits, src_rows, idx, key, nnz, slot, S, L, fix, nfix, T, out, out_rows, carry, \
                  acc_out, mark, hfix, cnt, mrow, s)
    switch (role) {
        case 1: return SEG_ROLE(1);
        case 2: return SEG_ROLE(2);
        case 3: return SEG_ROLE(3);
        case 4: return SEG_ROLE(4);
        default: return SEG_ROLE(0);
    }
#undef SEG_ROLE
}

}  // namespace merlin
