// merlin_gemm.hip -- fc1 of both towers (src/actor_critic.py:31-41, Linear(576, 512) -> ReLU) in
// fp32 on the bf16 matrix cores: forward with the bias + ReLU epilogue, the input gradient and the
// split-K weight gradient of PPO.update's minibatch step (src/ppo.py:141-156).
//
// gfx950 has no reduced-precision f32 MFMA (no xf32) and its f32-input MFMA runs at 1/16 of the
// bf16 rate.  An fp32 value x is stored as three bf16 planes x = x0 + x1 + x2, EXACTLY: x0 =
// bf16(x) (round to nearest), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1); each subtraction is exact
// in fp32 and each plane takes the next 8 of the 24 significand bits, so nothing is lost.  A
// product a*b is then sum_{i+j<=2} a_i*b_j, six bf16 MFMAs with fp32 accumulation; the three terms
// left out (a1 b2, a2 b1, a2 b2) are below 2^-24 |a b| together at worst, the size of one fp32
// rounding, and every bf16 x bf16 product is exact in fp32.  Each 32-deep k step is summed in its
// own accumulator and added to the running sum once (mma6), so the small plane products never round
// at the running sum's scale.  So these GEMMs compute fp32 products
// at 16/6 of the f32 MFMA rate (tests/test_gpu_gemm.py measures the error against float64 beside
// hipBLASLt's fp32 GEMM on the same operands).
//
// Plane layout ("x6 planes") of a logical fp32 matrix X[R][C], C % 8 == 0: bf16 [R][C/8][3][8],
// i.e. per row and per group of 8 columns three 16-B chunks (planes 0, 1, 2).  The producers
// write it directly (k_window_conv3: fc1's input rows; k_head_bwd: fc1's output gradient), so no
// fp32 copy of either operand exists on the update path.
//
//   k_x6_nt  C[t][m][n] = epi(sum_k A[t][m][k] B[t][n][k]) (both operands K-contiguous: forward
//            with B = W4, input gradient with B = W4^T); block tile BM x BN, K steps of 32, the
//            next step's chunks prefetched into registers while the current one is multiplied
//            from LDS; LDS rows of 64 B with the 16-B chunk index XORed by (row >> 2) & 3 so each
//            16-lane ds_read_b128 group hits 16 distinct bank slots.
//   k_x6_tn  slab[s][t][m][n] = sum_{k in split s} A[t][k][m] B[t][k][n] (weight gradient: both
//            operands row-major over the long reduction dimension k = the minibatch's frames);
//            LDS images [k][m] read with ds_read_b64_tr_b16 (the hardware transposed read) so the
//            MFMA fragments come out k-contiguous; k_x6_fold sums the slabs in split order.
#include <algorithm>

#include "merlin_internal.h"
#include "merlin_x6.h"

namespace merlin {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
typedef __attribute__((address_space(3))) char lds_char;

constexpr int BK = 32;       // k per step: 4 groups of 8
constexpr int CPR = 12;      // 16-B chunks per row and k step (4 groups x 3 planes)

__global__ __launch_bounds__(256) void k_x6_split(const float4 *__restrict__ x, int64_t n4,
                                                  uint2 *__restrict__ planes) {
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n4; e += (int64_t)gridDim.x * 256)
        x6_store4(planes, e, x[e]);
}

// planes -> fp32 (tests: the planes must add back to the input exactly)
__global__ __launch_bounds__(256) void k_x6_join(const uint2 *__restrict__ planes, int64_t n4,
                                                 float4 *__restrict__ x) {
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n4; e += (int64_t)gridDim.x * 256) {
        const uint2 *s = planes + (e >> 1) * 6 + (e & 1);
        const uint2 a = s[0], b = s[2], c = s[4];
        x[e] = make_float4(x6_lo(a.x) + x6_lo(b.x) + x6_lo(c.x), x6_hi(a.x) + x6_hi(b.x) + x6_hi(c.x),
                           x6_lo(a.y) + x6_lo(b.y) + x6_lo(c.y), x6_hi(a.y) + x6_hi(b.y) + x6_hi(c.y));
    }
}

__device__ __forceinline__ f32x4 mfma(const u32x4 a, const u32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma(const bf16x8 a, const bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// acc + the six plane products with i + j <= 2 of one k step.  The step's products are summed on
// their own (smallest first, into a fresh accumulator) and the step's total is added to acc with one
// rounding: the five small products never round at the running sum's scale, so the error is that of
// a blocked fp32 sum (the matrix cores' own bf16 x bf16 products are exact).
template <typename F>
__device__ __forceinline__ f32x4 mma6(const F a[3], const F b[3], f32x4 acc) {
    f32x4 c = mfma(a[2], b[0], f32x4{0.0f, 0.0f, 0.0f, 0.0f});
    c = mfma(a[1], b[1], c);
    c = mfma(a[0], b[2], c);
    c = mfma(a[1], b[0], c);
    c = mfma(a[0], b[1], c);
    c = mfma(a[0], b[0], c);
    return acc + c;
}

__device__ __forceinline__ float relu_nan(float v) { return v != v ? v : fmaxf(v, 0.0f); }

// block id -> tile id so that each XCD (blocks b % 8 share one) takes a contiguous run of tiles:
// the BN-column tiles of one BM-row panel run back to back on one L2 (bijective for any count)
__device__ __forceinline__ int xcd_tile(int b, int nb) {
    const int xcd = b & 7, q = nb >> 3, r = nb & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

// ---------------------------------------------------------------------------------------------
// NT: C[t][m][n] = epi(sum_k A[t][m][k] B[t][n][k]); A, B in x6 planes (K % 32 == 0, N % BN == 0);
// EPI 1: relu(. + bias[t][n]).  grid (tiles_m * tiles_n, T).
template <int BM, int BN, int WGM, int WGN, int EPI>
__global__ __launch_bounds__(64 * WGM * WGN) void k_x6_nt(const u32x4 *__restrict__ A, const u32x4 *__restrict__ B,
                                                          int64_t M, int N, int K, int64_t sA, int64_t sB,
                                                          const float *__restrict__ bias, float *__restrict__ C,
                                                          int64_t sC, int tiles_n) {
    constexpr int NT = 64 * WGM * WGN;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int FM = WTM / 16, FN = WTN / 16;
    constexpr int CA = (BM * CPR + NT - 1) / NT, CB = (BN * CPR + NT - 1) / NT;
    static_assert(WTM % 16 == 0 && WTN % 16 == 0, "wave tile");
    // two LDS stages: step kt+1 is written into the other stage while step kt is multiplied, one
    // barrier per step; the registers hold step kt+2 in flight (issued a whole step before use)
    // plane p of the A / B image at p * PSA / 3 * PSA + p * PSB chunks: the 12-chunk pad per plane
    // (plus the chunk order of the staging loads, planes major within a row) makes every 16-lane
    // group of the staging writes, and of the fragment reads, hit 16 distinct bank slots
    constexpr int PSA = BM * 4 + 12, PSB = BN * 4 + 12;
    constexpr int STAGE = 3 * (PSA + PSB);
    __shared__ u32x4 lds[2 * STAGE];

    const int t = blockIdx.y;
    const int L = xcd_tile(blockIdx.x, gridDim.x);
    const int tm = L / tiles_n, tn = L - tm * tiles_n;
    const int64_t m0 = (int64_t)tm * BM;
    const int n0 = tn * BN;
    const int64_t rowA = (int64_t)(K / 8) * 3;  // chunks per row
    A += t * sA;
    B += t * sB;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WGN, wn = w - (w / WGN) * WGN;

    const u32x4 *ga[CA];
    int la[CA];
#pragma unroll
    for (int i = 0; i < CA; i++) {
        const int q = tid + i * NT;
        const int row = q / CPR, rem = q - (q / CPR) * CPR, p = rem >> 2, g = rem & 3;
        const int64_t grow = std::min<int64_t>(m0 + std::min(row, BM - 1), M - 1);
        ga[i] = A + grow * rowA + g * 3 + p;
        la[i] = p * PSA + row * 4 + (g ^ ((row >> 2) & 3));
    }
    const u32x4 *gb[CB];
    int lb[CB];
#pragma unroll
    for (int i = 0; i < CB; i++) {
        const int q = tid + i * NT;
        const int row = q / CPR, rem = q - (q / CPR) * CPR, p = rem >> 2, g = rem & 3;
        gb[i] = B + (int64_t)(n0 + std::min(row, BN - 1)) * rowA + g * 3 + p;
        lb[i] = 3 * PSA + p * PSB + row * 4 + (g ^ ((row >> 2) & 3));
    }
    u32x4 ra[CA], rb[CB];
    auto load = [&](int kt) {
#pragma unroll
        for (int i = 0; i < CA; i++) ra[i] = ga[i][(int64_t)kt * CPR];
#pragma unroll
        for (int i = 0; i < CB; i++) rb[i] = gb[i][(int64_t)kt * CPR];
    };
    auto store = [&](int buf) {
        u32x4 *st = lds + buf * STAGE;
#pragma unroll
        for (int i = 0; i < CA; i++)
            if ((BM * CPR) % NT == 0 || i + 1 < CA || tid + i * NT < BM * CPR) st[la[i]] = ra[i];
#pragma unroll
        for (int i = 0; i < CB; i++)
            if ((BN * CPR) % NT == 0 || i + 1 < CB || tid + i * NT < BN * CPR) st[lb[i]] = rb[i];
    };

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

    // fragment read offsets: row (base + lane & 15), chunk (lane >> 4) XOR ((lane & 15) >> 2)
    const int fr = lane & 15, fc = (lane >> 4) ^ ((lane & 15) >> 2);
    const int nk = K / BK;
    load(0);
    store(0);
    if (nk > 1) load(1);
    __syncthreads();
    for (int kt = 0; kt < nk; kt++) {
        const int buf = kt & 1;
        if (kt + 1 < nk) store(buf ^ 1);
        if (kt + 2 < nk) load(kt + 2);
        const u32x4 *sAl = lds + buf * STAGE, *sBl = sAl + 3 * PSA;
        if constexpr (FM <= FN) {  // A fragments resident, B streamed
            u32x4 af[FM][3];
#pragma unroll
            for (int i = 0; i < FM; i++)
#pragma unroll
                for (int p = 0; p < 3; p++) af[i][p] = sAl[p * PSA + (wm * WTM + i * 16 + fr) * 4 + fc];
#pragma unroll
            for (int j = 0; j < FN; j++) {
                u32x4 bf[3];
#pragma unroll
                for (int p = 0; p < 3; p++) bf[p] = sBl[p * PSB + (wn * WTN + j * 16 + fr) * 4 + fc];
#pragma unroll
                for (int i = 0; i < FM; i++) acc[i][j] = mma6(af[i], bf, acc[i][j]);
            }
        } else {
            u32x4 bf[FN][3];
#pragma unroll
            for (int j = 0; j < FN; j++)
#pragma unroll
                for (int p = 0; p < 3; p++) bf[j][p] = sBl[p * PSB + (wn * WTN + j * 16 + fr) * 4 + fc];
#pragma unroll
            for (int i = 0; i < FM; i++) {
                u32x4 af[3];
#pragma unroll
                for (int p = 0; p < 3; p++) af[p] = sAl[p * PSA + (wm * WTM + i * 16 + fr) * 4 + fc];
#pragma unroll
                for (int j = 0; j < FN; j++) acc[i][j] = mma6(af, bf[j], acc[i][j]);
            }
        }
        __syncthreads();
    }

    float *Ct = C + t * sC;
#pragma unroll
    for (int j = 0; j < FN; j++) {
        const int col = n0 + wn * WTN + j * 16 + fr;
        const float bv = EPI == 1 ? bias[(int64_t)t * N + col] : 0.0f;
#pragma unroll
        for (int i = 0; i < FM; i++) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int64_t row = m0 + wm * WTM + i * 16 + 4 * (lane >> 4) + r;
                if (row < M) {
                    const float v = acc[i][j][r];
                    Ct[row * N + col] = EPI == 1 ? relu_nan(v + bv) : v;
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// The same product as a persistent kernel: one block per CU walks its tiles (tile j*G + base, tiles
// numbered (t, tm, tn) with tn fastest; base puts G/8 consecutive tiles on each XCD per round, so
// the BN-column tiles of one A panel run together on one L2) as one flat stream of k steps: the
// loads of the next tile's first steps are in flight while the current tile finishes, and the
// epilogue's stores overlap the next tile's multiplies.  G % 8 == 0.
template <int BM, int BN, int WGM, int WGN, int EPI>
__global__ __launch_bounds__(64 * WGM * WGN) void k_x6_ntp(const u32x4 *__restrict__ A, const u32x4 *__restrict__ B,
                                                           int64_t M, int N, int K, int64_t sA, int64_t sB,
                                                           const float *__restrict__ bias, float *__restrict__ C,
                                                           int64_t sC, int tiles_m, int tiles_n, int T) {
    constexpr int NT = 64 * WGM * WGN;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int FM = WTM / 16, FN = WTN / 16;
    constexpr int CA = (BM * CPR + NT - 1) / NT, CB = (BN * CPR + NT - 1) / NT;
    static_assert(WTM % 16 == 0 && WTN % 16 == 0, "wave tile");
    constexpr int PSA = BM * 4 + 12, PSB = BN * 4 + 12;
    constexpr int STAGE = 3 * (PSA + PSB);
    __shared__ u32x4 lds[2 * STAGE];

    const int G = gridDim.x, b = blockIdx.x;
    const int base = (b & 7) * (G >> 3) + (b >> 3);
    const int per_t = tiles_m * tiles_n, total = T * per_t;
    const int nk = K / BK;
    const int ntl = base < total ? (total - base + G - 1) / G : 0;
    const int steps = ntl * nk;
    if (steps == 0) return;
    const int64_t rowA = (int64_t)(K / 8) * 3;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WGN, wn = w - (w / WGN) * WGN;

    int rA[CA], oA[CA], la[CA];
#pragma unroll
    for (int i = 0; i < CA; i++) {
        const int q = tid + i * NT;
        const int row = q / CPR, rem = q - (q / CPR) * CPR, p = rem >> 2, g = rem & 3;
        rA[i] = std::min(row, BM - 1);
        oA[i] = g * 3 + p;
        la[i] = p * PSA + row * 4 + (g ^ ((row >> 2) & 3));
    }
    int oB[CB], lb[CB];
#pragma unroll
    for (int i = 0; i < CB; i++) {
        const int q = tid + i * NT;
        const int row = q / CPR, rem = q - (q / CPR) * CPR, p = rem >> 2, g = rem & 3;
        oB[i] = std::min(row, BN - 1) * (int)rowA + g * 3 + p;
        lb[i] = 3 * PSA + p * PSB + row * 4 + (g ^ ((row >> 2) & 3));
    }
    auto tile_of = [&](int j, int &t, int &tm, int &tn) {
        const int id = j * G + base;
        t = id / per_t;
        const int r = id - t * per_t;
        tm = r / tiles_n;
        tn = r - tm * tiles_n;
    };
    u32x4 ra[CA], rb[CB];
    auto load = [&](int s) {
        const int j = s / nk, kt = s - j * nk;
        int t, tm, tn;
        tile_of(j, t, tm, tn);
        const u32x4 *Ab = A + t * sA + kt * CPR;
        const u32x4 *Bb = B + t * sB + (int64_t)tn * BN * rowA + kt * CPR;
        const int64_t m0 = (int64_t)tm * BM;
#pragma unroll
        for (int i = 0; i < CA; i++) ra[i] = Ab[std::min<int64_t>(m0 + rA[i], M - 1) * rowA + oA[i]];
#pragma unroll
        for (int i = 0; i < CB; i++) rb[i] = Bb[oB[i]];
    };
    auto store = [&](int buf) {
        u32x4 *st = lds + buf * STAGE;
#pragma unroll
        for (int i = 0; i < CA; i++)
            if ((BM * CPR) % NT == 0 || i + 1 < CA || tid + i * NT < BM * CPR) st[la[i]] = ra[i];
#pragma unroll
        for (int i = 0; i < CB; i++)
            if ((BN * CPR) % NT == 0 || i + 1 < CB || tid + i * NT < BN * CPR) st[lb[i]] = rb[i];
    };

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

    const int fr = lane & 15, fc = (lane >> 4) ^ ((lane & 15) >> 2);
    load(0);
    store(0);
    if (steps > 1) load(1);
    __syncthreads();
    int kt = 0, jt = 0;
    for (int s = 0; s < steps; s++) {
        const int buf = s & 1;
        if (s + 1 < steps) store(buf ^ 1);
        if (s + 2 < steps) load(s + 2);
        const u32x4 *sAl = lds + buf * STAGE, *sBl = sAl + 3 * PSA;
        if constexpr (FM <= FN) {
            u32x4 af[FM][3];
#pragma unroll
            for (int i = 0; i < FM; i++)
#pragma unroll
                for (int p = 0; p < 3; p++) af[i][p] = sAl[p * PSA + (wm * WTM + i * 16 + fr) * 4 + fc];
#pragma unroll
            for (int j = 0; j < FN; j++) {
                u32x4 bf[3];
#pragma unroll
                for (int p = 0; p < 3; p++) bf[p] = sBl[p * PSB + (wn * WTN + j * 16 + fr) * 4 + fc];
#pragma unroll
                for (int i = 0; i < FM; i++) acc[i][j] = mma6(af[i], bf, acc[i][j]);
            }
        } else {
            u32x4 bf[FN][3];
#pragma unroll
            for (int j = 0; j < FN; j++)
#pragma unroll
                for (int p = 0; p < 3; p++) bf[j][p] = sBl[p * PSB + (wn * WTN + j * 16 + fr) * 4 + fc];
#pragma unroll
            for (int i = 0; i < FM; i++) {
                u32x4 af[3];
#pragma unroll
                for (int p = 0; p < 3; p++) af[p] = sAl[p * PSA + (wm * WTM + i * 16 + fr) * 4 + fc];
#pragma unroll
                for (int j = 0; j < FN; j++) acc[i][j] = mma6(af, bf[j], acc[i][j]);
            }
        }
        if (++kt == nk) {  // tile done: epilogue, fresh accumulators
            int t, tm, tn;
            tile_of(jt, t, tm, tn);
            float *Ct = C + t * sC;
            const int64_t m0 = (int64_t)tm * BM;
#pragma unroll
            for (int j = 0; j < FN; j++) {
                const int col = tn * BN + wn * WTN + j * 16 + fr;
                const float bv = EPI == 1 ? bias[(int64_t)t * N + col] : 0.0f;
#pragma unroll
                for (int i = 0; i < FM; i++) {
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int64_t row = m0 + wm * WTM + i * 16 + 4 * (lane >> 4) + r;
                        if (row < M) {
                            const float v = acc[i][j][r];
                            Ct[row * N + col] = EPI == 1 ? relu_nan(v + bv) : v;
                        }
                    }
                    acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
                }
            }
            kt = 0;
            jt++;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// TN: slab[s][t][m][n] = sum_{k in [s*kc, min(Kd, (s+1)*kc))} A[t][k][m] B[t][k][n]; A = x6 planes
// [Kd][M/8][3][8], B = [Kd][N/8][3][8]; M % BM == 0, N % BN == 0, kc % 32 == 0.
// grid (tiles_m * tiles_n, splits, T).
// LDS image of one plane: [32 k rows][BM / 8 chunks], chunk index XOR sw(row) so that a 32-lane
// half of a transposed read (rows r..r+3 and r+8..r+11, two adjacent chunks each) hits 16
// distinct 16-B bank slots (rows of 16k chunks or of 16k + 8 chunks).
template <int RC>
__device__ __forceinline__ int tr_swz(int row) {
    static_assert(RC % 8 == 0, "row chunks");
    if constexpr (RC % 16 == 0)
        return ((row & 3) << 1) | (((row >> 3) & 1) << 3);
    else
        return (((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2);
}

template <int RC>
__device__ __forceinline__ bf16x8 tr_frag(const u32x4 *img, int col0, int lane) {
    // rows 8G + 4h + q, columns col0 + 4 * pp .. + 3 (G = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3)
    const int G = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    const int chunk = (col0 >> 3) + (pp >> 1);
    bf16x4 v[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int row = 8 * G + 4 * h + q;
        const int off = (row * RC + (chunk ^ tr_swz<RC>(row))) * 16 + (pp & 1) * 8;
        v[h] = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4 *)((lds_char *)img + off));
    }
    return bf16x8{v[0][0], v[0][1], v[0][2], v[0][3], v[1][0], v[1][1], v[1][2], v[1][3]};
}

template <int BM, int BN, int WGM, int WGN>
__global__ __launch_bounds__(64 * WGM * WGN) void k_x6_tn(const u32x4 *__restrict__ A, const u32x4 *__restrict__ B,
                                                          int64_t Kd, int M, int N, int64_t sA, int64_t sB, int64_t kc,
                                                          int tiles_n, float *__restrict__ slab) {
    constexpr int NT = 64 * WGM * WGN;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int FM = WTM / 16, FN = WTN / 16;
    constexpr int RCA = BM / 8, RCB = BN / 8;                 // chunks per LDS row (one plane)
    constexpr int QA = BK * RCA * 3, QB = BK * RCB * 3;       // chunks per k step
    constexpr int CA = (QA + NT - 1) / NT, CB = (QB + NT - 1) / NT;
    static_assert(WTM % 16 == 0 && WTN % 16 == 0, "wave tile");
    // two LDS stages, one barrier per step (as k_x6_nt)
    // plane images of BK * RC chunks, padded to keep the staging writes conflict-free (rows of 16k + 8
    // chunks), planes major in the staging order
    constexpr int PSA = BK * RCA + (RCA % 16 ? 8 : 0), PSB = BK * RCB + (RCB % 16 ? 8 : 0);
    constexpr int STAGE = 3 * (PSA + PSB);
    __shared__ u32x4 lds[2 * STAGE];

    const int t = blockIdx.z, s = blockIdx.y;
    const int L = xcd_tile(blockIdx.x, gridDim.x);
    const int tm = L / tiles_n, tn = L - tm * tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int64_t k0 = (int64_t)s * kc, k1 = std::min<int64_t>(Kd, k0 + kc);
    const int64_t rowA = (int64_t)(M / 8) * 3, rowB = (int64_t)(N / 8) * 3;
    A += t * sA + (m0 / 8) * 3;
    B += t * sB + (n0 / 8) * 3;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WGN, wn = w - (w / WGN) * WGN;

    int ka[CA], oa[CA], la[CA];
#pragma unroll
    for (int i = 0; i < CA; i++) {
        const int q = tid + i * NT;
        const int k = std::min(q, QA - 1) / (RCA * 3), rem = std::min(q, QA - 1) - k * (RCA * 3);
        const int p = rem / RCA, g = rem - (rem / RCA) * RCA;
        ka[i] = k;
        oa[i] = g * 3 + p;
        la[i] = p * PSA + k * RCA + (g ^ tr_swz<RCA>(k));
    }
    int kb[CB], ob[CB], lb[CB];
#pragma unroll
    for (int i = 0; i < CB; i++) {
        const int q = tid + i * NT;
        const int k = std::min(q, QB - 1) / (RCB * 3), rem = std::min(q, QB - 1) - k * (RCB * 3);
        const int p = rem / RCB, g = rem - (rem / RCB) * RCB;
        kb[i] = k;
        ob[i] = g * 3 + p;
        lb[i] = 3 * PSA + p * PSB + k * RCB + (g ^ tr_swz<RCB>(k));
    }
    const u32x4 zero = u32x4{0u, 0u, 0u, 0u};
    u32x4 ra[CA], rb[CB];
    auto load = [&](int64_t kk) {
#pragma unroll
        for (int i = 0; i < CA; i++) {
            const int64_t k = kk + ka[i];
            const u32x4 v = A[std::min(k, k1 - 1) * rowA + oa[i]];
            ra[i] = k < k1 ? v : zero;
        }
#pragma unroll
        for (int i = 0; i < CB; i++) {
            const int64_t k = kk + kb[i];
            const u32x4 v = B[std::min(k, k1 - 1) * rowB + ob[i]];
            rb[i] = k < k1 ? v : zero;
        }
    };
    auto store = [&](int buf) {
        u32x4 *st = lds + buf * STAGE;
#pragma unroll
        for (int i = 0; i < CA; i++)
            if (QA % NT == 0 || i + 1 < CA || tid + i * NT < QA) st[la[i]] = ra[i];
#pragma unroll
        for (int i = 0; i < CB; i++)
            if (QB % NT == 0 || i + 1 < CB || tid + i * NT < QB) st[lb[i]] = rb[i];
    };

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

    if (k0 < k1) {
        load(k0);
        store(0);
        if (k0 + BK < k1) load(k0 + BK);
        __syncthreads();
    }
    int buf = 0;
    for (int64_t kk = k0; kk < k1; kk += BK, buf ^= 1) {
        if (kk + BK < k1) store(buf ^ 1);
        if (kk + 2 * BK < k1) load(kk + 2 * BK);
        const u32x4 *sAl = lds + buf * STAGE, *sBl = sAl + 3 * PSA;
        if constexpr (FM <= FN) {
            bf16x8 af[FM][3];
#pragma unroll
            for (int i = 0; i < FM; i++)
#pragma unroll
                for (int p = 0; p < 3; p++) af[i][p] = tr_frag<RCA>(sAl + p * PSA, wm * WTM + i * 16, lane);
#pragma unroll
            for (int j = 0; j < FN; j++) {
                bf16x8 bf[3];
#pragma unroll
                for (int p = 0; p < 3; p++) bf[p] = tr_frag<RCB>(sBl + p * PSB, wn * WTN + j * 16, lane);
#pragma unroll
                for (int i = 0; i < FM; i++) acc[i][j] = mma6(af[i], bf, acc[i][j]);
            }
        } else {
            bf16x8 bf[FN][3];
#pragma unroll
            for (int j = 0; j < FN; j++)
#pragma unroll
                for (int p = 0; p < 3; p++) bf[j][p] = tr_frag<RCB>(sBl + p * PSB, wn * WTN + j * 16, lane);
#pragma unroll
            for (int i = 0; i < FM; i++) {
                bf16x8 af[3];
#pragma unroll
                for (int p = 0; p < 3; p++) af[p] = tr_frag<RCA>(sAl + p * PSA, wm * WTM + i * 16, lane);
#pragma unroll
                for (int j = 0; j < FN; j++) acc[i][j] = mma6(af, bf[j], acc[i][j]);
            }
        }
        __syncthreads();
    }

    float *St = slab + ((int64_t)s * gridDim.z + t) * (int64_t)M * N;
    const int fr = lane & 15;
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = m0 + wm * WTM + i * 16 + 4 * (lane >> 4) + r;
                St[(int64_t)row * N + n0 + wn * WTN + j * 16 + fr] = acc[i][j][r];
            }
}

// out[e] = sum over s of slab[s][e] (e < total4 float4s), in split order
__global__ __launch_bounds__(256) void k_x6_fold(const float4 *__restrict__ slab, int S, int64_t total4,
                                                 float4 *__restrict__ out) {
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total4; e += (int64_t)gridDim.x * 256) {
        float4 a = slab[e];
        for (int s = 1; s < S; s++) {
            const float4 v = slab[(int64_t)s * total4 + e];
            a.x += v.x;
            a.y += v.y;
            a.z += v.z;
            a.w += v.w;
        }
        out[e] = a;
    }
}

// NT tile configurations (cfg): 0 = 128 x 128, 4 waves (forward, N = 512); 1 = 128 x 64, 4 waves
// (input gradient, N = 576); 2 = 256 x 128, 8 waves; 3 = 128 x 192, 8 waves; 4 = 128 x 96, 4 waves
template <int BM, int BN, int WGM, int WGN>
hipError_t nt_launch(const u32x4 *A, const u32x4 *B, int64_t M, int N, int K, int T, int64_t sA, int64_t sB,
                     const float *bias, float *C, int64_t sC, hipStream_t s) {
    if (N % BN) return hipErrorInvalidValue;
    const int64_t tiles_m = (M + BM - 1) / BM;
    const int tiles_n = N / BN;
    if (tiles_m * tiles_n > INT32_MAX) return hipErrorInvalidValue;
    const dim3 grid((unsigned)(tiles_m * tiles_n), T);
    if (bias)
        hipLaunchKernelGGL((k_x6_nt<BM, BN, WGM, WGN, 1>), grid, dim3(64 * WGM * WGN), 0, s, A, B, M, N, K, sA, sB, bias,
                           C, sC, tiles_n);
    else
        hipLaunchKernelGGL((k_x6_nt<BM, BN, WGM, WGN, 0>), grid, dim3(64 * WGM * WGN), 0, s, A, B, M, N, K, sA, sB,
                           nullptr, C, sC, tiles_n);
    return hipGetLastError();
}

int num_cus() {
    static int n = 0;
    if (!n) {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
            n = v;
        else
            n = 256;
    }
    return n;
}

template <int BM, int BN, int WGM, int WGN>
hipError_t ntp_launch(const u32x4 *A, const u32x4 *B, int64_t M, int N, int K, int T, int64_t sA, int64_t sB,
                      const float *bias, float *C, int64_t sC, hipStream_t s) {
    if (N % BN) return hipErrorInvalidValue;
    const int64_t tiles_m = (M + BM - 1) / BM;
    const int tiles_n = N / BN;
    const int64_t total = tiles_m * tiles_n * T;
    if (total > INT32_MAX / 2) return hipErrorInvalidValue;
    const int G = (int)std::min<int64_t>((total + 7) / 8 * 8, num_cus() / 8 * 8);
    if (bias)
        hipLaunchKernelGGL((k_x6_ntp<BM, BN, WGM, WGN, 1>), dim3(G), dim3(64 * WGM * WGN), 0, s, A, B, M, N, K, sA, sB,
                           bias, C, sC, (int)tiles_m, tiles_n, T);
    else
        hipLaunchKernelGGL((k_x6_ntp<BM, BN, WGM, WGN, 0>), dim3(G), dim3(64 * WGM * WGN), 0, s, A, B, M, N, K, sA, sB,
                           nullptr, C, sC, (int)tiles_m, tiles_n, T);
    return hipGetLastError();
}

template <int BM, int BN, int WGM, int WGN>
hipError_t tn_launch(const u32x4 *A, const u32x4 *B, int64_t Kd, int M, int N, int T, int64_t sA, int64_t sB,
                     int splits, float *slab, float *out, hipStream_t s) {
    if (M % BM || N % BN) return hipErrorInvalidValue;
    const int tiles_n = N / BN, tiles = (M / BM) * tiles_n;
    int S = std::max(1, splits);
    int64_t kc = (Kd + S - 1) / S;
    kc = (kc + BK - 1) / BK * BK;
    S = (int)std::max<int64_t>(1, (Kd + kc - 1) / kc);
    hipLaunchKernelGGL((k_x6_tn<BM, BN, WGM, WGN>), dim3(tiles, S, T), dim3(64 * WGM * WGN), 0, s, A, B, Kd, M, N, sA,
                       sB, kc, tiles_n, slab);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int64_t total4 = (int64_t)T * M * N / 4;
    const int grid = (int)std::min<int64_t>((total4 + 255) / 256, 256 * 8);
    hipLaunchKernelGGL(k_x6_fold, dim3(grid), dim3(256), 0, s, reinterpret_cast<const float4 *>(slab), S, total4,
                       reinterpret_cast<float4 *>(out));
    return hipGetLastError();
}

}  // namespace

hipError_t launch_x6_split(const float *x, int64_t n, void *planes, hipStream_t s) {
    if (n % 8) return hipErrorInvalidValue;
    const int64_t n4 = n / 4;
    if (n4 <= 0) return hipSuccess;
    const int grid = (int)std::min<int64_t>((n4 + 255) / 256, 256 * 16);
    hipLaunchKernelGGL(k_x6_split, dim3(grid), dim3(256), 0, s, reinterpret_cast<const float4 *>(x), n4,
                       reinterpret_cast<uint2 *>(planes));
    return hipGetLastError();
}

hipError_t launch_x6_join(const void *planes, int64_t n, float *x, hipStream_t s) {
    if (n % 8) return hipErrorInvalidValue;
    const int64_t n4 = n / 4;
    if (n4 <= 0) return hipSuccess;
    const int grid = (int)std::min<int64_t>((n4 + 255) / 256, 256 * 16);
    hipLaunchKernelGGL(k_x6_join, dim3(grid), dim3(256), 0, s, reinterpret_cast<const uint2 *>(planes), n4,
                       reinterpret_cast<float4 *>(x));
    return hipGetLastError();
}

hipError_t launch_x6_gemm_nt(const void *A, const void *B, int64_t M, int N, int K, int T, int64_t a_stride,
                             int64_t b_stride, const float *bias, float *C, int64_t c_stride, int cfg, hipStream_t s) {
    if (M <= 0) return hipSuccess;
    if (K % BK || N <= 0) return hipErrorInvalidValue;
    // strides are in elements; chunks of 8 bf16 x 3 planes = 8 logical elements per 3 chunks
    if (a_stride % 8 || b_stride % 8) return hipErrorInvalidValue;
    const u32x4 *a = static_cast<const u32x4 *>(A), *b = static_cast<const u32x4 *>(B);
    const int64_t sA = a_stride / 8 * 3, sB = b_stride / 8 * 3;
    switch (cfg) {
        case 0: return nt_launch<128, 128, 2, 2>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        case 1: return nt_launch<128, 64, 2, 2>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        case 2: return nt_launch<256, 128, 4, 2>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        case 3: return nt_launch<128, 192, 2, 4>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        case 4: return nt_launch<128, 96, 2, 2>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        case 5: return nt_launch<256, 64, 4, 2>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        case 6: return ntp_launch<256, 128, 4, 2>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        case 7: return ntp_launch<128, 192, 2, 4>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        case 8: return ntp_launch<256, 64, 4, 2>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        case 9: return ntp_launch<128, 128, 2, 2>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        default: return hipErrorInvalidValue;
    }
}

int x6_tn_max_splits() { return 64; }

hipError_t launch_x6_gemm_tn(const void *A, const void *B, int64_t Kd, int M, int N, int T, int64_t a_stride,
                             int64_t b_stride, int splits, float *slab, float *out, int cfg, hipStream_t s) {
    if (M <= 0 || N <= 0) return hipSuccess;
    if (M % 8 || N % 8 || a_stride % 8 || b_stride % 8) return hipErrorInvalidValue;
    if (Kd <= 0) return hipMemsetAsync(out, 0, sizeof(float) * (size_t)T * M * N, s);
    const u32x4 *a = static_cast<const u32x4 *>(A), *b = static_cast<const u32x4 *>(B);
    const int64_t sA = a_stride / 8 * 3, sB = b_stride / 8 * 3;
    switch (cfg) {
        case 0: return tn_launch<128, 64, 2, 2>(a, b, Kd, M, N, T, sA, sB, splits, slab, out, s);
        case 1: return tn_launch<128, 192, 2, 4>(a, b, Kd, M, N, T, sA, sB, splits, slab, out, s);
        case 2: return tn_launch<128, 192, 4, 2>(a, b, Kd, M, N, T, sA, sB, splits, slab, out, s);
        case 3: return tn_launch<64, 192, 2, 2>(a, b, Kd, M, N, T, sA, sB, splits, slab, out, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace merlin
