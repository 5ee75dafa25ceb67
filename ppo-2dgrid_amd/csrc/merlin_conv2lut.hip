// merlin_conv2lut.hip -- conv1 + conv2 of both CNN towers as table lookups over the tile codes.
//
// Why this is exact arithmetic on the same function (src/actor_critic.py:9-14,20-21):
// every observation is a 7x7 blit of 5 atlas tiles (8x8 px), and conv1 (k8, s4) windows
// cover 2x2 quarter-tile blocks, so relu(conv1) at position (y, x) of the 13x13 map is one
// of a few vectors: it depends only on the classes of the tiles its blocks fall in and on
// the parity of (y, x):
//   y even, x even: 1 tile            -> 5 possible 32-vectors       (type ee)
//   y even, x odd : 2 tiles (row)     -> 25                          (type eo)
//   y odd,  x even: 2 tiles (column)  -> 25                          (type oe)
//   y odd,  x odd : 2x2 tiles         -> 625                         (type oo)
// conv2 (k4, s2) tap (ky, kx) of output (py, px) reads conv1 position (2py+ky, 2px+kx),
// whose parity is (ky&1, kx&1): so
//   Z2[py][px][co] = sum over 16 taps of  T[tap][v(tap, py, px)][co]
// with T[tap][v] = W2[:, :, ky, kx] . relu(conv1)[type(tap)][v]: 2,720 rows x 64 floats per
// tower (ee 5x4 taps, eo 25x4, oe 25x4, oo 625x4), built from the weights by a few small
// differentiable torch ops (merlin/actor_critic.py::conv2_tables) once per optimizer step.
// Row layout: type blocks at bases 0 / 20 / 120 / 220, row = base + 4*v + j with
// j = 2*(ky>>1) + (kx>>1); v = the type's tile classes in base 5, lexicographic over
// (row, col) of the tiles, top-left tile = (py + (ky>>1), px + (kx>>1)).
//
// Forward (k_conv2_lut_fwd): per output 16 float4 row loads from the L2-resident tables and
// a sum -- 102 KB of table reads instead of 819k MACs per frame per tower.
// Backward (k_conv2_lut_hist): dT[row] = sum of dZ2 over the (frame, position) pairs whose
// tap reads that row: a histogram, accumulated in 64-bit fixed point with LDS integer
// atomics in a block-private copy of one 4-channel slice of the table, then folded across
// blocks (k_conv2_lut_fold).
// dW2, the conv1 weight/bias gradient and db2 follow from dT by autograd through the table
// construction (db2 = sum of tap 0's rows, since each output position reads exactly one
// row of every tap).
#include <algorithm>

#include "merlin_internal.h"

namespace merlin {
namespace {

constexpr int NROW = 2720;        // table rows per tower
constexpr int C2 = 64, P2 = 25;   // conv2 output channels / positions

// 16 table rows of output position (py, px) from its 3x3 tile-class window w[a*3 + b]
__device__ __forceinline__ void tap_rows(const int w[9], int rows[16]) {
#pragma unroll
    for (int ky = 0; ky < 4; ky++)
#pragma unroll
        for (int kx = 0; kx < 4; kx++) {
            const int a = ky >> 1, b = kx >> 1, j = 2 * a + b;
            const int c00 = w[a * 3 + b];
            int row;
            if (!(ky & 1) && !(kx & 1)) {
                row = 4 * c00 + j;
            } else if (!(ky & 1)) {
                row = 20 + 4 * (5 * c00 + w[a * 3 + b + 1]) + j;
            } else if (!(kx & 1)) {
                row = 120 + 4 * (5 * c00 + w[(a + 1) * 3 + b]) + j;
            } else {
                row = 220 + 4 * (125 * c00 + 25 * w[a * 3 + b + 1] + 5 * w[(a + 1) * 3 + b] + w[(a + 1) * 3 + b + 1]) + j;
            }
            rows[ky * 4 + kx] = row;
        }
}

__device__ __forceinline__ void window(const uint8_t *cls, int p, int w[9]) {
    const int py = p / 5, px = p - (p / 5) * 5;
    const uint8_t *c = cls + py * 7 + px;
#pragma unroll
    for (int a = 0; a < 3; a++)
#pragma unroll
        for (int b = 0; b < 3; b++) w[a * 3 + b] = c[a * 7 + b];
}

// wave-private staging of nf frames' 49 tile classes (bytes) into cls
__device__ __forceinline__ void stage_classes(const uint32_t *__restrict__ codes, const int64_t *__restrict__ index,
                                              int64_t s0, int nf, int lane, uint8_t *cls) {
    for (int e = lane; e < nf * 49; e += 64) {
        const int f = e / 49, cell = e - f * 49;
        const int64_t row = index ? index[s0 + f] : s0 + f;
        const uint32_t word = codes[row * MERLIN_OBS_WORDS + (cell >> 3)];
        // classes are 0..4 by construction; the clamp keeps a corrupt code inside the tables
        cls[e] = (uint8_t)min((word >> ((cell & 7) * 4)) & 0xfu, 4u);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS writes are visible to it
    __builtin_amdgcn_wave_barrier();
}

// ---------------------------------------------------------------------------
constexpr int FWD_WAVES = 4, FWD_G = 4;  // frames per wave group
// gstride > 0 (grouped): frame s belongs to group g = s / gstride and is evaluated only by that group's
// two towers 2g, 2g+1 (their own tables: one weight set per group, e.g. FOMAML's per-task policies);
// Z2 is then [towers][gstride*25][16 float4] with the frame at its index within the group.
__global__ __launch_bounds__(64 * FWD_WAVES) void k_conv2_lut_fwd(const uint32_t *__restrict__ codes,
                                                                 const int64_t *__restrict__ index, int64_t n,
                                                                 const float4 *__restrict__ tab, int towers,
                                                                 float4 *__restrict__ Z2, int64_t gstride) {
    __shared__ uint8_t cls_all[FWD_WAVES][FWD_G * 49 + 4];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint8_t *cls = cls_all[wv];
    const int64_t groups = (n + FWD_G - 1) / FWD_G;
    for (int64_t g = (int64_t)blockIdx.x * FWD_WAVES + wv; g < groups; g += (int64_t)gridDim.x * FWD_WAVES) {
        const int64_t s0 = g * FWD_G;
        const int nf = (int)std::min<int64_t>(FWD_G, n - s0);
        stage_classes(codes, index, s0, nf, lane, cls);
        const int tasks = (gstride > 0 ? 2 : towers) * nf * P2 * 16;
        for (int tid = lane; tid < tasks; tid += 64) {
            const int q = tid & 15, r = tid >> 4;
            const int p = r % P2, tf = r / P2, f = tf % nf;
            int t = tf / nf;
            int64_t orow = s0 + f, rows_per_t = n;  // output row of the frame within its tower's block
            if (gstride > 0) {
                const int64_t gi = (s0 + f) / gstride;
                t += 2 * (int)gi;
                orow = s0 + f - gi * gstride;
                rows_per_t = gstride;
            }
            int w[9], rows[16];
            window(cls + f * 49, p, w);
            tap_rows(w, rows);
            const float4 *tt = tab + (size_t)t * NROW * 16 + q;
            float4 v[16];
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = tt[rows[k] * 16];
            float4 acc = v[0];
#pragma unroll
            for (int k = 1; k < 16; k++) {
                acc.x += v[k].x;
                acc.y += v[k].y;
                acc.z += v[k].z;
                acc.w += v[k].w;
            }
            Z2[((size_t)t * rows_per_t + orow) * (P2 * 16) + p * 16 + q] = acc;
        }
        __builtin_amdgcn_wave_barrier();  // this group's classes consumed before restaging
    }
}

// ---------------------------------------------------------------------------
// Histogram.  Block = (tower, 4-channel chunk, frame range); dZ2c is chunk-major
// [towers][16][n*25][4] (k_col2im3_bwd, chunked), so a block streams contiguous bytes.
// Lane = (tap k = lane/4, channel c = lane%4): one wave instruction adds one entry
// (frame, position) into its 16 rows (distinct: rows of different taps never coincide)
// x 4 channels.  Accumulation is in 64-bit fixed point with LDS integer atomics
// (ds_add_u64): LDS float atomics run ~44x slower than integer ones on gfx950
// (scripts/micro/lds_atomics.hip: 193 vs 4.4 cycles per wave instruction), and integer
// sums are exact and order-independent, so the result is bitwise reproducible.
// Scale 2^K with K = 62 - ceil(log2(n*25 + 1)) - e, max|dZ2| < 2^e (from k_col2im3_bwd):
// no partial or total sum of a row can overflow, and each term is rounded to 2^-K.
constexpr int HIST_WAVES = 16, HIST_G = 4, HCH = 4, NHCHUNK = C2 / HCH;
constexpr int HSLICE = NROW * HCH;  // u64 per slice table (87,040 B)

__device__ __forceinline__ int fixed_exp(uint32_t absmax_bits, int64_t n) {
    const float M = __uint_as_float(absmax_bits);
    int e = 0;
    frexpf(M, &e);  // M < 2^e (M == 0: e = 0)
    int lg = 0;
    while ((int64_t(1) << lg) < n * P2 + 1) lg++;
    return 62 - lg - e;
}

// round(g * 2^K) from the float's bits (|g| * 2^K < 2^38 by the choice of K)
__device__ __forceinline__ long long to_fixed(float g, int K) {
    const uint32_t bits = __float_as_uint(g);
    int E = (bits >> 23) & 0xff;
    uint32_t m = bits & 0x7fffffu;
    if (E) m |= 0x800000u; else E = 1;
    const int sh = E - 150 + K;
    long long q;
    if (sh >= 0) q = (long long)m << sh;
    else if (sh > -26) q = (long long)((m + (1u << (-sh - 1))) >> (-sh));
    else q = 0;
    return (bits >> 31) ? -q : q;
}

// codes here are the minibatch's own rows (the caller gathers them once), so a wave's group
// of frames is one contiguous 128-B read; the next group's dZ2 slice and code words are
// loaded into registers while the current group is accumulated.
// grouped (gstride > 0): n = frames per tower, and tower t's frames are codes rows (t / 2) * gstride + [0, n)
__global__ __launch_bounds__(64 * HIST_WAVES) void k_conv2_lut_hist(const uint32_t *__restrict__ codes, int64_t n,
                                                                   const float *__restrict__ dZ2c,
                                                                   const uint32_t *__restrict__ absmax, int fblocks,
                                                                   unsigned long long *__restrict__ slabs,
                                                                   int64_t gstride) {
    __shared__ unsigned long long tab[HSLICE];
    __shared__ uint32_t words_all[HIST_WAVES][HIST_G * MERLIN_OBS_WORDS];
    // per frame, per parity type and 2x2-tile window origin (r, c) in 0..5: the type's table
    // row base + 4 v (rows of tap j are that + j)
    __shared__ uint16_t rb_all[HIST_WAVES][HIST_G * 4 * 36];
    // the group's dZ2 slice already in fixed point: [frame][position][channel] as int64
    __shared__ __align__(16) long long q_all[HIST_WAVES][HIST_G * P2 * HCH];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tc = blockIdx.x / fblocks, fb = blockIdx.x - tc * fblocks;  // tc = tower*16 + chunk
    if (gstride > 0) codes += (size_t)(tc / NHCHUNK / 2) * gstride * MERLIN_OBS_WORDS;
    uint32_t *words = words_all[wv];
    uint16_t *rb = rb_all[wv];
    long long *qs = q_all[wv];
    for (int k = threadIdx.x; k < HSLICE; k += blockDim.x) tab[k] = 0ull;
    const int K = fixed_exp(*absmax, n);
    __syncthreads();
    // this lane's tap: type (yp, xp), tap index j within the type, tile offset (a, b)
    const int k = lane >> 2, c = lane & 3, ky = k >> 2, kx = k & 3;
    const int type = 2 * (ky & 1) + (kx & 1), a = ky >> 1, b = kx >> 1, j = 2 * a + b;
    int64_t per = (n + fblocks - 1) / fblocks;
    per = (per + HIST_G - 1) / HIST_G * HIST_G;
    const int64_t f0 = (int64_t)fb * per, f1 = std::min<int64_t>(n, f0 + per);
    const float4 *src0 = reinterpret_cast<const float4 *>(dZ2c) + (size_t)tc * n * P2;
    const int64_t stride = (int64_t)HIST_WAVES * HIST_G;
    float4 pg0 = make_float4(0.f, 0.f, 0.f, 0.f), pg1 = pg0;
    uint32_t pw = 0u;
    auto prefetch = [&](int64_t gg) {
        const int nf = (int)std::min<int64_t>(HIST_G, f1 - gg);
        const float4 *src = src0 + (size_t)gg * P2;
        if (lane < nf * P2) pg0 = src[lane];
        if (lane + 64 < nf * P2) pg1 = src[lane + 64];
        if (lane < nf * MERLIN_OBS_WORDS) pw = codes[gg * MERLIN_OBS_WORDS + lane];
    };
    int64_t g = f0 + (int64_t)wv * HIST_G;
    if (g < f1) prefetch(g);
    for (; g < f1; g += stride) {
        const int nf = (int)std::min<int64_t>(HIST_G, f1 - g);
        if (lane < nf * P2) {
            longlong2 *d = reinterpret_cast<longlong2 *>(qs + lane * HCH);
            d[0] = make_longlong2(to_fixed(pg0.x, K), to_fixed(pg0.y, K));
            d[1] = make_longlong2(to_fixed(pg0.z, K), to_fixed(pg0.w, K));
        }
        if (lane + 64 < nf * P2) {
            longlong2 *d = reinterpret_cast<longlong2 *>(qs + (lane + 64) * HCH);
            d[0] = make_longlong2(to_fixed(pg1.x, K), to_fixed(pg1.y, K));
            d[1] = make_longlong2(to_fixed(pg1.z, K), to_fixed(pg1.w, K));
        }
        if (lane < nf * MERLIN_OBS_WORDS) words[lane] = pw;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS writes are visible to it
        __builtin_amdgcn_wave_barrier();
        if (g + stride < f1) prefetch(g + stride);
        for (int e = lane; e < nf * 4 * 36; e += 64) {
            const int f = e / 144, r = e - f * 144, ty = r / 36, w = r - ty * 36, wr = w / 6, wc = w - wr * 6;
            const uint32_t *fw = words + f * MERLIN_OBS_WORDS;
            auto cls = [&](int cell) { return (int)min((fw[cell >> 3] >> ((cell & 7) * 4)) & 0xfu, 4u); };
            const int cell = wr * 7 + wc;
            const int c00 = cls(cell);
            int v, base;
            if (ty == 0) { v = c00; base = 0; }
            else if (ty == 1) { v = 5 * c00 + cls(cell + 1); base = 20; }
            else if (ty == 2) { v = 5 * c00 + cls(cell + 7); base = 120; }
            else { v = 125 * c00 + 25 * cls(cell + 1) + 5 * cls(cell + 7) + cls(cell + 8); base = 220; }
            rb[e] = (uint16_t)(base + 4 * v);
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        for (int f = 0; f < nf; f++) {
            const uint16_t *rf = rb + f * 144 + type * 36 + a * 6 + b;
            const long long *qf = qs + f * (P2 * HCH) + c;
            unsigned long long *tc0 = tab + j * HCH + c;
#pragma unroll
            for (int p = 0; p < P2; p++) {
                const long long q = qf[p * HCH];  // constant offsets: immediate ds_read fields
                const int row = rf[(p / 5) * 6 + p % 5];
                if (q != 0) atomicAdd(tc0 + row * HCH, (unsigned long long)q);
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    ulonglong2 *dst = reinterpret_cast<ulonglong2 *>(slabs + (size_t)blockIdx.x * HSLICE);
    const ulonglong2 *t2 = reinterpret_cast<const ulonglong2 *>(tab);
    for (int e = threadIdx.x; e < HSLICE / 2; e += blockDim.x) dst[e] = t2[e];
}

// dT[t][row][chunk*4 + c] = (sum over the fblocks slabs of slice (t, chunk)) * 2^-K
__global__ __launch_bounds__(256) void k_conv2_lut_fold(const unsigned long long *__restrict__ slabs,
                                                        const uint32_t *__restrict__ absmax, int64_t n, int towers,
                                                        int fblocks, float *__restrict__ dT) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= towers * NROW * C2) return;
    const int t = k / (NROW * C2), r = k - t * (NROW * C2), row = r >> 6, co = r & 63;
    const int tc = t * NHCHUNK + (co >> 2);
    const unsigned long long *s = slabs + (size_t)tc * fblocks * HSLICE + row * HCH + (co & 3);
    unsigned long long acc = 0ull;
    for (int b = 0; b < fblocks; b++) acc += s[(size_t)b * HSLICE];
    const float M = __uint_as_float(*absmax);
    dT[k] = (M - M != 0.0f) ? __int_as_float(0x7fc00000)  // non-finite gradient in: NaN out
                            : (float)ldexp((double)(long long)acc, -fixed_exp(*absmax, n));
}

}  // namespace

int conv2_lut_rows() { return NROW; }

size_t conv2_lut_slab_bytes(int towers, int fblocks) {
    return sizeof(unsigned long long) * (size_t)towers * NHCHUNK * fblocks * HSLICE;
}

hipError_t launch_conv2_lut_fwd(const uint32_t *codes, const int64_t *index, int64_t n, const float *tables,
                                int towers, float *Z2, hipStream_t s, int64_t gstride) {
    if (n <= 0) return hipSuccess;
    const int64_t groups = (n + FWD_G - 1) / FWD_G;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((groups + FWD_WAVES - 1) / FWD_WAVES, 256 * 8));
    hipLaunchKernelGGL(k_conv2_lut_fwd, dim3(grid), dim3(64 * FWD_WAVES), 0, s, codes, index, n,
                       reinterpret_cast<const float4 *>(tables), towers, reinterpret_cast<float4 *>(Z2), gstride);
    return hipGetLastError();
}

int conv2_lut_fblocks(int64_t n) {
    // one block (16 waves, 87 KB LDS slice) per CU: 2 towers x 16 chunks x fblocks frame ranges
    return (int)std::max<int64_t>(1, std::min<int64_t>(8, (n + 255) / 256));
}

hipError_t launch_conv2_lut_bwd(const uint32_t *codes, int64_t n, const float *dZ2c, const uint32_t *absmax,
                                int towers, float *dT, void *slabs, hipStream_t s, int64_t gstride) {
    if (n <= 0) return zero_async(dT, sizeof(float) * towers * NROW * C2, s);
    const int fblocks = conv2_lut_fblocks(n);
    auto *sl = reinterpret_cast<unsigned long long *>(slabs);
    hipLaunchKernelGGL(k_conv2_lut_hist, dim3(towers * NHCHUNK * fblocks), dim3(64 * HIST_WAVES), 0, s, codes,
                       n, dZ2c, absmax, fblocks, sl, gstride);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_conv2_lut_fold, dim3((towers * NROW * C2 + 255) / 256), dim3(256), 0, s, sl, absmax, n,
                       towers, fblocks, dT);
    return hipGetLastError();
}

}  // namespace merlin
