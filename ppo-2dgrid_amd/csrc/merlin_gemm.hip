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
// The activations (fc1's input rows a3 and output gradient dz, the big operands) are read as fp32
// and split in registers while they are staged into LDS (4 bytes per value from HBM / L2 instead of
// the planes' 6); the weights, small and re-read by every tile, are split once per call into
// "x6 planes" (merlin_x6.h: bf16 [R][C/8][3][8]).  LDS holds every operand as three plane images.
//
//   k_x6_nt  C[t][m][n] = epi(sum_k A[t][m][k] B[t][n][k]), A fp32 [M][K], B planes [N][K]
//            (forward with B = W4, input gradient with B = W4^T); block tile BM x BN, k steps of
//            32, two LDS stages (one barrier per step), the step after next in flight in
//            registers; plane images with rows of 64 B, the 16-B chunk index XORed by
//            (row >> 2) & 3, so the ds_read_b128 fragment reads and the staging writes are free of
//            bank conflicts.
//   k_x6_tn  slab[s][t][m][n] = sum_{k in split s} A[t][k][m] B[t][k][n], A and B fp32 row-major
//            over the long reduction dimension k = the minibatch's frames (weight gradient dz^T
//            a3); plane images [k][m] read with ds_read_b64_tr_b16 (the hardware transposed read)
//            so the MFMA fragments come out k-contiguous; k_x6_fold sums the slabs in split order.
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

// acc + the six plane products with i + j <= 2 of one k step.  CHUNK: the step's products are
// summed on their own (smallest first, into a fresh accumulator) and the step's total is added to
// acc with one rounding, so the five small products never round at the running sum's scale -- the
// error of a blocked fp32 sum (the matrix cores' own bf16 x bf16 products are exact); the weight
// gradient's long, cancelling sums need it.  Without CHUNK the six products accumulate straight into
// acc (smallest first): six roundings per 32-deep step at the running sum's scale, still fewer than
// an fp32 fma chain's 32, and no vector adds beside the matrix cores.
template <bool CHUNK, typename F>
__device__ __forceinline__ f32x4 mma6(const F a[3], const F b[3], f32x4 acc) {
    f32x4 c = mfma(a[2], b[0], CHUNK ? f32x4{0.0f, 0.0f, 0.0f, 0.0f} : acc);
    c = mfma(a[1], b[1], c);
    c = mfma(a[0], b[2], c);
    c = mfma(a[1], b[0], c);
    c = mfma(a[0], b[1], c);
    c = mfma(a[0], b[0], c);
    return CHUNK ? acc + c : c;
}

__device__ __forceinline__ float relu_nan(float v) { return v != v ? v : fmaxf(v, 0.0f); }

// block id -> tile id so that each XCD (blocks b % 8 share one) takes a contiguous run of tiles:
// the BN-column tiles of one BM-row panel run back to back on one L2 (bijective for any count)
__device__ __forceinline__ int xcd_tile(int b, int nb) {
    const int xcd = b & 7, q = nb >> 3, r = nb & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

// 8 fp32 values -> their three planes as 16-B fragments chunks
__device__ __forceinline__ void split8(const float4 a, const float4 b, u32x4 &p0, u32x4 &p1, u32x4 &p2) {
    uint2 x[3], y[3];
    x6_split4(a, x);
    x6_split4(b, y);
    p0 = u32x4{x[0].x, x[0].y, y[0].x, y[0].y};
    p1 = u32x4{x[1].x, x[1].y, y[1].x, y[1].y};
    p2 = u32x4{x[2].x, x[2].y, y[2].x, y[2].y};
}

// ---------------------------------------------------------------------------------------------
// NT: C[t][m][n] = epi(sum_k A[t][m][k] B[t][n][k]); A fp32 [M][K], B x6 planes [N][K/8][3][8]
// (K % 32 == 0, N % BN == 0); EPI 1: relu(. + bias[t][n]).  grid (tiles_m * tiles_n, T).
template <int BM, int BN, int WGM, int WGN, int EPI, bool CHUNK>
__global__ __launch_bounds__(64 * WGM * WGN) void k_x6_nt(const float4 *__restrict__ A, const u32x4 *__restrict__ B,
                                                          int64_t M, int N, int K, int64_t sA, int64_t sB,
                                                          const float *__restrict__ bias, float *__restrict__ C,
                                                          int64_t sC, int tiles_n) {
    constexpr int NT = 64 * WGM * WGN;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int FM = WTM / 16, FN = WTN / 16;
    constexpr int UA = (BM * 4 + NT - 1) / NT;        // A units (row, group of 8 values) per thread
    constexpr int CB = (BN * CPR + NT - 1) / NT;      // B 16-B plane chunks per thread
    static_assert(WTM % 16 == 0 && WTN % 16 == 0, "wave tile");
    // plane p of the A image at p * PSA chunks, of the B image at 3 * PSA + p * PSB; the B pad and
    // chunk order (planes major within a row) keep its staging writes conflict-free as well
    constexpr int PSA = BM * 4, PSB = BN * 4 + 12;
    constexpr int STAGE = 3 * (PSA + PSB);
    __shared__ u32x4 lds[2 * STAGE];

    const int t = blockIdx.y;
    const int L = xcd_tile(blockIdx.x, gridDim.x);
    const int tm = L / tiles_n, tn = L - tm * tiles_n;
    const int64_t m0 = (int64_t)tm * BM;
    const int n0 = tn * BN;
    const int64_t rowA = K / 4;                 // float4 per A row
    const int64_t rowB = (int64_t)(K / 8) * 3;  // chunks per B row
    A += t * sA;
    B += t * sB;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WGN, wn = w - (w / WGN) * WGN;

    const float4 *ga[UA];
    int la[UA];
#pragma unroll
    for (int i = 0; i < UA; i++) {
        const int q = tid + i * NT;
        const int row = std::min(q >> 2, BM - 1), g = q & 3;
        ga[i] = A + std::min<int64_t>(m0 + row, M - 1) * rowA + g * 2;
        la[i] = row * 4 + (g ^ ((row >> 2) & 3));
    }
    const u32x4 *gb[CB];
    int lb[CB];
#pragma unroll
    for (int i = 0; i < CB; i++) {
        const int q = tid + i * NT;
        const int row = q / CPR, rem = q - (q / CPR) * CPR, p = rem >> 2, g = rem & 3;
        gb[i] = B + (int64_t)(n0 + std::min(row, BN - 1)) * rowB + g * 3 + p;
        lb[i] = 3 * PSA + p * PSB + row * 4 + (g ^ ((row >> 2) & 3));
    }
    float4 ra[UA][2];
    u32x4 rb[CB];
    auto load = [&](int kt) {
#pragma unroll
        for (int i = 0; i < UA; i++) {
            ra[i][0] = ga[i][(int64_t)kt * 8];
            ra[i][1] = ga[i][(int64_t)kt * 8 + 1];
        }
#pragma unroll
        for (int i = 0; i < CB; i++) rb[i] = gb[i][(int64_t)kt * CPR];
    };
    auto store = [&](int buf) {
        u32x4 *st = lds + buf * STAGE;
#pragma unroll
        for (int i = 0; i < UA; i++)
            if ((BM * 4) % NT == 0 || i + 1 < UA || tid + i * NT < BM * 4) {
                u32x4 p0, p1, p2;
                split8(ra[i][0], ra[i][1], p0, p1, p2);
                st[la[i]] = p0;
                st[PSA + la[i]] = p1;
                st[2 * PSA + la[i]] = p2;
            }
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
                for (int i = 0; i < FM; i++) acc[i][j] = mma6<CHUNK>(af[i], bf, acc[i][j]);
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
                for (int j = 0; j < FN; j++) acc[i][j] = mma6<CHUNK>(af, bf[j], acc[i][j]);
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
// NT, interleaved: the same tiles, LDS images and numerics as k_x6_nt, but the staging of the next
// k step (the A split + plane stores, the B chunk stores) and the global loads of the step after are
// spread over the MFMA groups of the current step instead of running as one block before them: with
// one barrier per k step every wave of a SIMD otherwise reaches its split at the same time and the
// matrix pipe idles through it.  The loop body has no branches (the last steps stage/load clamped,
// never-read data), so the scheduler sees one block per k step.  SCHED 1: sched_group_barrier pins an
// MFMA / VALU / DS alternation; SCHED 2: additionally s_setprio 1 around the MFMA groups.
template <int BM, int BN, int WGM, int WGN, int EPI, int SCHED>
__global__ __launch_bounds__(64 * WGM * WGN) void k_x6_nt_il(const float4 *__restrict__ A, const u32x4 *__restrict__ B,
                                                             int64_t M, int N, int K, int64_t sA, int64_t sB,
                                                             const float *__restrict__ bias, float *__restrict__ C,
                                                             int64_t sC, int tiles_n) {
    constexpr int NT = 64 * WGM * WGN;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int FM = WTM / 16, FN = WTN / 16;
    constexpr int UA = (BM * 4 + NT - 1) / NT;
    constexpr int CB = (BN * CPR + NT - 1) / NT;
    static_assert(WTM % 16 == 0 && WTN % 16 == 0, "wave tile");
    constexpr int PSA = BM * 4, PSB = BN * 4 + 12;
    constexpr int STAGE = 3 * (PSA + PSB);
    constexpr int NO = FM <= FN ? FN : FM;  // outer fragment loop: staging pieces go between its groups
    static_assert(NO >= 2, "need two MFMA groups per k step");
    __shared__ u32x4 lds[2 * STAGE];

    const int t = blockIdx.y;
    const int L = xcd_tile(blockIdx.x, gridDim.x);
    const int tm = L / tiles_n, tn = L - tm * tiles_n;
    const int64_t m0 = (int64_t)tm * BM;
    const int n0 = tn * BN;
    const int64_t rowA = K / 4;
    const int64_t rowB = (int64_t)(K / 8) * 3;
    A += t * sA;
    B += t * sB;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WGN, wn = w - (w / WGN) * WGN;

    const float4 *ga[UA];
    int la[UA];
#pragma unroll
    for (int i = 0; i < UA; i++) {
        const int q = tid + i * NT;
        const int row = std::min(q >> 2, BM - 1), g = q & 3;
        ga[i] = A + std::min<int64_t>(m0 + row, M - 1) * rowA + g * 2;
        la[i] = row * 4 + (g ^ ((row >> 2) & 3));
    }
    const u32x4 *gb[CB];
    int lb[CB];
#pragma unroll
    for (int i = 0; i < CB; i++) {
        const int q = tid + i * NT;
        const int row = q / CPR, rem = q - (q / CPR) * CPR, p = rem >> 2, g = rem & 3;
        gb[i] = B + (int64_t)(n0 + std::min(row, BN - 1)) * rowB + g * 3 + p;
        lb[i] = 3 * PSA + p * PSB + row * 4 + (g ^ ((row >> 2) & 3));
    }
    float4 ra[UA][2];
    u32x4 rb[CB];
    const int nk = K / BK;
    auto load = [&](int kt) {
        kt = std::min(kt, nk - 1);  // past the end: reload the last step (never stored to a read stage)
#pragma unroll
        for (int i = 0; i < UA; i++) {
            ra[i][0] = ga[i][(int64_t)kt * 8];
            ra[i][1] = ga[i][(int64_t)kt * 8 + 1];
        }
#pragma unroll
        for (int i = 0; i < CB; i++) rb[i] = gb[i][(int64_t)kt * CPR];
    };
    auto store_a = [&](u32x4 *st, int i) {
        if ((BM * 4) % NT == 0 || i + 1 < UA || tid + i * NT < BM * 4) {
            u32x4 p0, p1, p2;
            split8(ra[i][0], ra[i][1], p0, p1, p2);
            st[la[i]] = p0;
            st[PSA + la[i]] = p1;
            st[2 * PSA + la[i]] = p2;
        }
    };
    auto store_b = [&](u32x4 *st, int i) {
        if ((BN * CPR) % NT == 0 || i + 1 < CB || tid + i * NT < BN * CPR) st[lb[i]] = rb[i];
    };
    // staging piece o (0 .. NO-2) of the next step: A units and groups of 3 B chunks, round robin
    constexpr int PIECES = UA + (CB + 2) / 3;
    auto stage = [&](u32x4 *st, int o) {
#pragma unroll
        for (int i = 0; i < UA; i++)
            if (i % (NO - 1) == o) store_a(st, i);
#pragma unroll
        for (int i = 0; i < CB; i++)
            if ((UA + i / 3) % (NO - 1) == o) store_b(st, i);
    };
    (void)PIECES;
    auto pin = [&]() {
        if constexpr (SCHED >= 1) {
            // per MFMA: one MFMA then two VALU; a DS write or read every few
#pragma unroll
            for (int q = 0; q < (FM <= FN ? FM : FN) * 6; q++) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
                if (q % 4 == 3) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
                if (q % 8 == 7) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
        }
    };

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

    const int fr = lane & 15, fc = (lane >> 4) ^ ((lane & 15) >> 2);
    load(0);
#pragma unroll
    for (int i = 0; i < UA; i++) store_a(lds, i);
#pragma unroll
    for (int i = 0; i < CB; i++) store_b(lds, i);
    load(1);
    __syncthreads();
    if constexpr (SCHED >= 2) __builtin_amdgcn_s_setprio(1);
    for (int kt = 0; kt < nk; kt++) {
        const int buf = kt & 1;
        const u32x4 *sAl = lds + buf * STAGE, *sBl = sAl + 3 * PSA;
        u32x4 *st = lds + (buf ^ 1) * STAGE;
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
                for (int i = 0; i < FM; i++) acc[i][j] = mma6<true>(af[i], bf, acc[i][j]);
                if (j < NO - 1)
                    stage(st, j);
                else
                    load(kt + 2);
                pin();
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
                for (int j = 0; j < FN; j++) acc[i][j] = mma6<true>(af, bf[j], acc[i][j]);
                if (i < NO - 1)
                    stage(st, i);
                else
                    load(kt + 2);
                pin();
            }
        }
        __syncthreads();
    }
    if constexpr (SCHED >= 2) __builtin_amdgcn_s_setprio(0);

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
// TN: slab[s][t][m][n] = sum_{k in [s*kc, min(Kd, (s+1)*kc))} A[t][k][m] B[t][k][n]; A fp32 [Kd][M],
// B fp32 [Kd][N]; M % BM == 0, N % BN == 0, kc % 32 == 0.  grid (tiles_m * tiles_n, splits, T).
// Plane image: [32 k rows][BM / 8 chunks], chunk index XOR tr_swz(row) so that a 32-lane half of
// a transposed read (rows r..r+3 and r+8..r+11, two adjacent chunks each) hits 16 distinct 16-B
// bank slots (rows of 16k chunks or of 16k + 8 chunks).
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
__global__ __launch_bounds__(64 * WGM * WGN) void k_x6_tn(const float4 *__restrict__ A, const float4 *__restrict__ B,
                                                          int64_t Kd, int M, int N, int64_t sA, int64_t sB, int64_t kc,
                                                          int tiles_n, int tiles, int S, float *__restrict__ slab) {
    constexpr int NT = 64 * WGM * WGN;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int FM = WTM / 16, FN = WTN / 16;
    constexpr int RCA = BM / 8, RCB = BN / 8;            // chunks (groups of 8 values) per image row
    constexpr int QA = BK * RCA, QB = BK * RCB;          // units per k step
    constexpr int UA = (QA + NT - 1) / NT, UB = (QB + NT - 1) / NT;
    static_assert(WTM % 16 == 0 && WTN % 16 == 0, "wave tile");
    constexpr int PSA = BK * RCA, PSB = BK * RCB;
    constexpr int STAGE = 3 * (PSA + PSB);
    __shared__ u32x4 lds[2 * STAGE];

    // 1-D grid over (tower, split, tile), tile fastest, XCD-contiguous (xcd_tile): the tiles of one
    // split read the same k rows of both operands, so they run together on one L2
    const int P = xcd_tile(blockIdx.x, gridDim.x);
    const int t = P / (S * tiles), s = (P / tiles) % S, L = P % tiles;
    const int tm = L / tiles_n, tn = L - tm * tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int64_t k0 = (int64_t)s * kc, k1 = std::min<int64_t>(Kd, k0 + kc);
    const int64_t rowA = M / 4, rowB = N / 4;  // float4 per row
    A += t * sA + m0 / 4;
    B += t * sB + n0 / 4;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WGN, wn = w - (w / WGN) * WGN;

    int ka[UA], oa[UA], la[UA];
#pragma unroll
    for (int i = 0; i < UA; i++) {
        const int q = std::min(tid + i * NT, QA - 1);
        const int k = q / RCA, g = q - (q / RCA) * RCA;
        ka[i] = k;
        oa[i] = g * 2;
        la[i] = k * RCA + (g ^ tr_swz<RCA>(k));
    }
    int kb[UB], ob[UB], lb[UB];
#pragma unroll
    for (int i = 0; i < UB; i++) {
        const int q = std::min(tid + i * NT, QB - 1);
        const int k = q / RCB, g = q - (q / RCB) * RCB;
        kb[i] = k;
        ob[i] = g * 2;
        lb[i] = 3 * PSA + k * RCB + (g ^ tr_swz<RCB>(k));
    }
    const float4 zero = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    float4 ra[UA][2], rb[UB][2];
    // each unit's row pointer at k0; a step whose rows are all below k1 (every step but a split's last) reads
    // pointer + a wave-uniform row offset, no per-lane 64-bit clamp arithmetic (whose temporaries made the
    // compiler park the loaded values in other registers: a wait right behind every load)
    const float4 *pa[UA], *pb[UB];
#pragma unroll
    for (int i = 0; i < UA; i++) pa[i] = A + (k0 + ka[i]) * rowA + oa[i];
#pragma unroll
    for (int i = 0; i < UB; i++) pb[i] = B + (k0 + kb[i]) * rowB + ob[i];
    auto load = [&](int64_t kk) {
        if (kk + BK <= k1) {
            const int64_t da = (kk - k0) * rowA, db = (kk - k0) * rowB;
#pragma unroll
            for (int i = 0; i < UA; i++) {
                ra[i][0] = pa[i][da];
                ra[i][1] = pa[i][da + 1];
            }
#pragma unroll
            for (int i = 0; i < UB; i++) {
                rb[i][0] = pb[i][db];
                rb[i][1] = pb[i][db + 1];
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < UA; i++) {
            const int64_t k = kk + ka[i];
            const float4 *src = A + std::min(k, k1 - 1) * rowA + oa[i];
            ra[i][0] = src[0];  // rows past k1 re-read row k1 - 1 and are zeroed when staged: a select
            ra[i][1] = src[1];  // here would make the wave wait for the loads right after issuing them
        }
#pragma unroll
        for (int i = 0; i < UB; i++) {
            const int64_t k = kk + kb[i];
            const float4 *src = B + std::min(k, k1 - 1) * rowB + ob[i];
            rb[i][0] = src[0];
            rb[i][1] = src[1];
        }
    };
    auto store = [&](int buf, int64_t kk) {  // the registers hold the rows of step kk; rows past k1 stage as zero
        u32x4 *st = lds + buf * STAGE;
#pragma unroll
        for (int i = 0; i < UA; i++)
            if (QA % NT == 0 || i + 1 < UA || tid + i * NT < QA) {
                const bool in = kk + ka[i] < k1;
                u32x4 p0, p1, p2;
                split8(in ? ra[i][0] : zero, in ? ra[i][1] : zero, p0, p1, p2);
                st[la[i]] = p0;
                st[PSA + la[i]] = p1;
                st[2 * PSA + la[i]] = p2;
            }
#pragma unroll
        for (int i = 0; i < UB; i++)
            if (QB % NT == 0 || i + 1 < UB || tid + i * NT < QB) {
                const bool in = kk + kb[i] < k1;
                u32x4 p0, p1, p2;
                split8(in ? rb[i][0] : zero, in ? rb[i][1] : zero, p0, p1, p2);
                st[lb[i]] = p0;
                st[PSB + lb[i]] = p1;
                st[2 * PSB + lb[i]] = p2;
            }
    };

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

    if (k0 < k1) {
        load(k0);
        store(0, k0);
        if (k0 + BK < k1) load(k0 + BK);
        __syncthreads();
    }
    int buf = 0;
    for (int64_t kk = k0; kk < k1; kk += BK, buf ^= 1) {
        if (kk + BK < k1) store(buf ^ 1, kk + BK);
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
                for (int i = 0; i < FM; i++) acc[i][j] = mma6<true>(af[i], bf, acc[i][j]);
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
                for (int j = 0; j < FN; j++) acc[i][j] = mma6<true>(af, bf[j], acc[i][j]);
            }
        }
        __syncthreads();
    }

    float *St = slab + ((int64_t)s * (gridDim.x / (S * tiles)) + t) * (int64_t)M * N;
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

template <int BM, int BN, int WGM, int WGN, bool CHUNK = true>
hipError_t nt_launch(const float4 *A, const u32x4 *B, int64_t M, int N, int K, int T, int64_t sA, int64_t sB,
                     const float *bias, float *C, int64_t sC, hipStream_t s) {
    if (N % BN) return hipErrorInvalidValue;
    const int64_t tiles_m = (M + BM - 1) / BM;
    const int tiles_n = N / BN;
    if (tiles_m * tiles_n > INT32_MAX) return hipErrorInvalidValue;
    const dim3 grid((unsigned)(tiles_m * tiles_n), T);
    if (bias)
        hipLaunchKernelGGL((k_x6_nt<BM, BN, WGM, WGN, 1, CHUNK>), grid, dim3(64 * WGM * WGN), 0, s, A, B, M, N, K, sA, sB, bias,
                           C, sC, tiles_n);
    else
        hipLaunchKernelGGL((k_x6_nt<BM, BN, WGM, WGN, 0, CHUNK>), grid, dim3(64 * WGM * WGN), 0, s, A, B, M, N, K, sA, sB,
                           nullptr, C, sC, tiles_n);
    return hipGetLastError();
}

template <int BM, int BN, int WGM, int WGN, int SCHED>
hipError_t nt_il_launch(const float4 *A, const u32x4 *B, int64_t M, int N, int K, int T, int64_t sA, int64_t sB,
                        const float *bias, float *C, int64_t sC, hipStream_t s) {
    if (N % BN) return hipErrorInvalidValue;
    const int64_t tiles_m = (M + BM - 1) / BM;
    const int tiles_n = N / BN;
    if (tiles_m * tiles_n > INT32_MAX) return hipErrorInvalidValue;
    const dim3 grid((unsigned)(tiles_m * tiles_n), T);
    if (bias)
        hipLaunchKernelGGL((k_x6_nt_il<BM, BN, WGM, WGN, 1, SCHED>), grid, dim3(64 * WGM * WGN), 0, s, A, B, M, N, K,
                           sA, sB, bias, C, sC, tiles_n);
    else
        hipLaunchKernelGGL((k_x6_nt_il<BM, BN, WGM, WGN, 0, SCHED>), grid, dim3(64 * WGM * WGN), 0, s, A, B, M, N, K,
                           sA, sB, nullptr, C, sC, tiles_n);
    return hipGetLastError();
}

template <int BM, int BN, int WGM, int WGN>
hipError_t tn_launch(const float4 *A, const float4 *B, int64_t Kd, int M, int N, int T, int64_t sA, int64_t sB,
                     int splits, float *slab, float *out, hipStream_t s) {
    if (M % BM || N % BN) return hipErrorInvalidValue;
    const int tiles_n = N / BN, tiles = (M / BM) * tiles_n;
    int S = std::max(1, splits);
    int64_t kc = (Kd + S - 1) / S;
    kc = (kc + BK - 1) / BK * BK;
    S = (int)std::max<int64_t>(1, (Kd + kc - 1) / kc);
    hipLaunchKernelGGL((k_x6_tn<BM, BN, WGM, WGN>), dim3(tiles * S * T), dim3(64 * WGM * WGN), 0, s, A, B, Kd, M, N,
                       sA, sB, kc, tiles_n, tiles, S, slab);
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

hipError_t launch_x6_gemm_nt(const float *A, const void *B, int64_t M, int N, int K, int T, int64_t a_stride,
                             int64_t b_stride, const float *bias, float *C, int64_t c_stride, int cfg, hipStream_t s) {
    if (M <= 0) return hipSuccess;
    if (K % BK || N <= 0) return hipErrorInvalidValue;
    // strides in values; B's planes: 3 chunks per 8 values
    if (a_stride % 4 || b_stride % 8) return hipErrorInvalidValue;
    if (cfg >= 20)  // the 32x32x16 MFMA kernels (merlin_gemm2.hip)
        return launch_x6_gemm_nt32(A, B, M, N, K, T, a_stride, b_stride, bias, C, c_stride, cfg, s);
    const float4 *a = reinterpret_cast<const float4 *>(A);
    const u32x4 *b = static_cast<const u32x4 *>(B);
    const int64_t sA = a_stride / 4, sB = b_stride / 8 * 3;
    switch (cfg) {
        case 0: return nt_launch<256, 128, 4, 2>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        case 1: return nt_launch<128, 192, 2, 4>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        case 2: return nt_launch<128, 128, 2, 2>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        case 3: return nt_launch<256, 64, 4, 2>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        // unchunked accumulation (all six products straight into the running sum): ~2-6 % faster,
        // error of the order of an fp32 fma chain (scripts/probe_x6.py); not used
        case 4: return nt_launch<256, 128, 4, 2, false>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        // interleaved staging (k_x6_nt_il): fwd / dgrad tiles, SCHED 0 / 1 / 2
        case 10: return nt_il_launch<256, 128, 4, 2, 0>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        case 11: return nt_il_launch<256, 128, 4, 2, 1>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        case 12: return nt_il_launch<256, 128, 4, 2, 2>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        case 13: return nt_il_launch<128, 192, 2, 4, 0>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        case 14: return nt_il_launch<128, 192, 2, 4, 1>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        case 15: return nt_il_launch<128, 192, 2, 4, 2>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        // one wave per SIMD: 256 x 128 over 4 waves (128 x 64 each)
        case 16: return nt_il_launch<256, 128, 2, 2, 0>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        case 17: return nt_il_launch<256, 128, 2, 2, 2>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        default: return hipErrorInvalidValue;
    }
}

int x6_tn_max_splits() { return 64; }

hipError_t launch_x6_fold(const float *slab, int S, int64_t total, float *out, hipStream_t s) {
    if (total % 4) return hipErrorInvalidValue;
    const int64_t total4 = total / 4;
    const int grid = (int)std::min<int64_t>((total4 + 255) / 256, 256 * 8);
    hipLaunchKernelGGL(k_x6_fold, dim3(grid), dim3(256), 0, s, reinterpret_cast<const float4 *>(slab), S, total4,
                       reinterpret_cast<float4 *>(out));
    return hipGetLastError();
}

hipError_t launch_x6_gemm_tn(const float *A, const float *B, int64_t Kd, int M, int N, int T, int64_t a_stride,
                             int64_t b_stride, int splits, float *slab, float *out, int cfg, hipStream_t s) {
    if (M <= 0 || N <= 0) return hipSuccess;
    if (M % 8 || N % 8 || a_stride % 4 || b_stride % 4) return hipErrorInvalidValue;
    if (Kd <= 0) return zero_async(out, sizeof(float) * (size_t)T * M * N, s);
    if (cfg >= 20) {  // the 32x32x16 MFMA kernels (merlin_gemm2.hip), then the same fold
        int S = 1;
        hipError_t e = launch_x6_gemm_tn32(A, B, Kd, M, N, T, a_stride, b_stride, splits, slab, cfg, s, &S);
        if (e != hipSuccess) return e;
        const int64_t total4 = (int64_t)T * M * N / 4;
        const int grid = (int)std::min<int64_t>((total4 + 255) / 256, 256 * 8);
        hipLaunchKernelGGL(k_x6_fold, dim3(grid), dim3(256), 0, s, reinterpret_cast<const float4 *>(slab), S, total4,
                           reinterpret_cast<float4 *>(out));
        return hipGetLastError();
    }
    const float4 *a = reinterpret_cast<const float4 *>(A), *b = reinterpret_cast<const float4 *>(B);
    const int64_t sA = a_stride / 4, sB = b_stride / 4;
    switch (cfg) {
        case 0: return tn_launch<128, 192, 2, 4>(a, b, Kd, M, N, T, sA, sB, splits, slab, out, s);
        case 1: return tn_launch<128, 64, 2, 2>(a, b, Kd, M, N, T, sA, sB, splits, slab, out, s);
        case 2: return tn_launch<128, 192, 4, 2>(a, b, Kd, M, N, T, sA, sB, splits, slab, out, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace merlin
