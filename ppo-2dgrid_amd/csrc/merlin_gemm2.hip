// merlin_gemm2.hip -- fc1's NT GEMMs (forward with the bias + ReLU epilogue, input gradient) on the
// 32x32x16 bf16 MFMA, same exact three-plane fp32 products as merlin_gemm.hip (merlin_x6.h).
//
// Why a second NT kernel: k_x6_nt issues one 16x16x32 MFMA per 16 matrix-pipe cycles, of which the
// MFMA itself holds the SIMD's issue port for 8; the k step's other instructions (the A split, LDS
// stores and fragment reads, the per-step accumulator adds, addressing) come to ~2.8 per MFMA, more
// than the ~2 issue slots each MFMA leaves free, so the matrix pipe idled half the time (profiles:
// MFMA busy 49 %).  v_mfma_f32_32x32x16_bf16 does twice the work per instruction for the same 8-cycle
// issue hold, which doubles the free issue slots per FLOP.  The per-step accumulator adds go too
// (ACC 1): the big products a0*b0 accumulate in one register set, the five small ones (a2 b0, a1 b1,
// a0 b2, a1 b0, a0 b1, smallest first) in a second, added once in the epilogue -- the small products
// never round at the running sum's scale, as with merlin_gemm.hip's per-step chunks (ACC 0 keeps that
// form: the k step's twelve products in a fresh accumulator, added to the running sum once).
//
// Tiles: block BM x BN, waves WGM x WGN, each wave (BM/WGM) x (BN/WGN) in 32 x 32 MFMA tiles; k steps of
// 32 (two MFMA k halves); LDS plane images exactly as k_x6_nt (64-B rows, 16-B chunk g XOR (row>>2)&3):
// a 32x32x16 fragment read (lane l: row l&31, chunk 2*kh + (l>>5)) hits 16 distinct 16-B bank slots per
// ds_read_b128 lane group.  Two LDS stages, one barrier per k step, the step after next in registers.
#include <algorithm>

#include "merlin_internal.h"
#include "merlin_x6.h"

namespace merlin {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 32;
constexpr int CPR = 12;  // 16-B chunks per row and k step (4 groups x 3 planes)

__device__ __forceinline__ f32x16 mfma32(const u32x4 a, const u32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                    0, 0, 0);
}

__device__ __forceinline__ float relu_nan(float v) { return v != v ? v : fmaxf(v, 0.0f); }

__device__ __forceinline__ int xcd_tile(int b, int nb) {
    const int xcd = b & 7, q = nb >> 3, r = nb & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

__device__ __forceinline__ void split8(const float4 a, const float4 b, u32x4 &p0, u32x4 &p1, u32x4 &p2) {
    uint2 x[3], y[3];
    x6_split4(a, x);
    x6_split4(b, y);
    p0 = u32x4{x[0].x, x[0].y, y[0].x, y[0].y};
    p1 = u32x4{x[1].x, x[1].y, y[1].x, y[1].y};
    p2 = u32x4{x[2].x, x[2].y, y[2].x, y[2].y};
}

// C[t][m][n] = epi(sum_k A[t][m][k] B[t][n][k]); A fp32 [M][K] (APL 0, split while staged) or x6
// planes [M][K/8][3][8] (APL 1, staged as copies like B), B x6 planes [N][K/8][3][8] (K % 32 == 0,
// N % BN == 0); EPI 1: relu(. + bias[t][n]).  grid (tiles_m * tiles_n, T).
template <int BM, int BN, int WGM, int WGN, int EPI, int ACC, int APL = 0>
__global__ __launch_bounds__(64 * WGM * WGN) void k_x6_nt32(const void *__restrict__ Av, const u32x4 *__restrict__ B,
                                                            int64_t M, int N, int K, int64_t sA, int64_t sB,
                                                            const float *__restrict__ bias, float *__restrict__ C,
                                                            int64_t sC, int tiles_n) {
    constexpr int NT = 64 * WGM * WGN;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int UA = APL ? (BM * CPR + NT - 1) / NT : (BM * 4 + NT - 1) / NT;  // A chunks / fp32 units
    constexpr int CB = (BN * CPR + NT - 1) / NT;
    static_assert(WTM % 32 == 0 && WTN % 32 == 0, "wave tile of 32 x 32 MFMA tiles");
    constexpr int PSA = BM * 4 + (APL ? 12 : 0), PSB = BN * 4 + 12;
    constexpr int STAGE = 3 * (PSA + PSB);
    __shared__ u32x4 lds[2 * STAGE];

    const int t = blockIdx.y;
    const int L = xcd_tile(blockIdx.x, gridDim.x);
    const int tm = L / tiles_n, tn = L - tm * tiles_n;
    const int64_t m0 = (int64_t)tm * BM;
    const int n0 = tn * BN;
    const int64_t rowA = APL ? (int64_t)(K / 8) * 3 : K / 4;  // A row in chunks (planes) / float4s
    const int64_t rowB = (int64_t)(K / 8) * 3;
    B += t * sB;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WGN, wn = w - (w / WGN) * WGN;

    const float4 *ga[APL ? 1 : UA];
    const u32x4 *Ap = static_cast<const u32x4 *>(Av) + t * sA;
    int gp[APL ? UA : 1];  // planes: chunk offsets from Ap (32-bit: fewer address registers)
    int la[UA];
#pragma unroll
    for (int i = 0; i < UA; i++) {
        const int q = tid + i * NT;
        if constexpr (APL) {
            const int row = std::min(q / CPR, BM - 1), rem = q - (q / CPR) * CPR, p = rem >> 2, g = rem & 3;
            gp[i] = (int)(std::min<int64_t>(m0 + row, M - 1) * rowA + g * 3 + p);
            la[i] = p * PSA + row * 4 + (g ^ ((row >> 2) & 3));
        } else {
            const int row = std::min(q >> 2, BM - 1), g = q & 3;
            ga[i] = static_cast<const float4 *>(Av) + t * sA + std::min<int64_t>(m0 + row, M - 1) * rowA + g * 2;
            la[i] = row * 4 + (g ^ ((row >> 2) & 3));
        }
    }
    int gb[CB];  // chunk offsets from B (the weights: N * K * 3 / 8 chunks, well inside 32 bits)
    int lb[CB];
#pragma unroll
    for (int i = 0; i < CB; i++) {
        const int q = tid + i * NT;
        const int row = q / CPR, rem = q - (q / CPR) * CPR, p = rem >> 2, g = rem & 3;
        gb[i] = (int)((int64_t)(n0 + std::min(row, BN - 1)) * rowB + g * 3 + p);
        lb[i] = 3 * PSA + p * PSB + row * 4 + (g ^ ((row >> 2) & 3));
    }
    float4 ra[APL ? 1 : UA][2];
    u32x4 rp[APL ? UA : 1];
    u32x4 rb[CB];
    auto load = [&](int kt) {
#pragma unroll
        for (int i = 0; i < UA; i++) {
            if constexpr (APL) {
                rp[i] = Ap[gp[i] + kt * CPR];
            } else {
                ra[i][0] = ga[i][(int64_t)kt * 8];
                ra[i][1] = ga[i][(int64_t)kt * 8 + 1];
            }
        }
#pragma unroll
        for (int i = 0; i < CB; i++) rb[i] = B[gb[i] + kt * CPR];
    };
    auto store = [&](int buf) {
        u32x4 *st = lds + buf * STAGE;
#pragma unroll
        for (int i = 0; i < UA; i++) {
            if constexpr (APL) {
                if ((BM * CPR) % NT == 0 || i + 1 < UA || tid + i * NT < BM * CPR) st[la[i]] = rp[i];
            } else if ((BM * 4) % NT == 0 || i + 1 < UA || tid + i * NT < BM * 4) {
                u32x4 p0, p1, p2;
                split8(ra[i][0], ra[i][1], p0, p1, p2);
                st[la[i]] = p0;
                st[PSA + la[i]] = p1;
                st[2 * PSA + la[i]] = p2;
            }
        }
#pragma unroll
        for (int i = 0; i < CB; i++)
            if ((BN * CPR) % NT == 0 || i + 1 < CB || tid + i * NT < BN * CPR) st[lb[i]] = rb[i];
    };

    f32x16 hi[TM][TN], lo[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++) {
            hi[i][j] = f32x16{};
            lo[i][j] = f32x16{};
        }

    // fragment reads: row (tile base + lane & 31), chunk (2 kh + (lane >> 5)) XOR ((lane & 31) >> 2) & 3
    const int fr = lane & 31, fh = lane >> 5, fs = (fr >> 2) & 3;
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
#pragma unroll
        for (int i = 0; i < TM; i++) {
            u32x4 af[2][3];
#pragma unroll
            for (int kh = 0; kh < 2; kh++)
#pragma unroll
                for (int p = 0; p < 3; p++)
                    af[kh][p] = sAl[p * PSA + (wm * WTM + i * 32 + fr) * 4 + ((2 * kh + fh) ^ fs)];
#pragma unroll
            for (int j = 0; j < TN; j++) {
                u32x4 bf[2][3];
#pragma unroll
                for (int kh = 0; kh < 2; kh++)
#pragma unroll
                    for (int p = 0; p < 3; p++)
                        bf[kh][p] = sBl[p * PSB + (wn * WTN + j * 32 + fr) * 4 + ((2 * kh + fh) ^ fs)];
                if constexpr (ACC == 1) {
                    f32x16 l = lo[i][j], h = hi[i][j];
#pragma unroll
                    for (int kh = 0; kh < 2; kh++) {
                        l = mfma32(af[kh][2], bf[kh][0], l);
                        l = mfma32(af[kh][1], bf[kh][1], l);
                        l = mfma32(af[kh][0], bf[kh][2], l);
                        l = mfma32(af[kh][1], bf[kh][0], l);
                        l = mfma32(af[kh][0], bf[kh][1], l);
                        h = mfma32(af[kh][0], bf[kh][0], h);
                    }
                    lo[i][j] = l;
                    hi[i][j] = h;
                } else {
                    f32x16 c = f32x16{};
#pragma unroll
                    for (int kh = 0; kh < 2; kh++) {
                        c = mfma32(af[kh][2], bf[kh][0], c);
                        c = mfma32(af[kh][1], bf[kh][1], c);
                        c = mfma32(af[kh][0], bf[kh][2], c);
                        c = mfma32(af[kh][1], bf[kh][0], c);
                        c = mfma32(af[kh][0], bf[kh][1], c);
                    }
#pragma unroll
                    for (int kh = 0; kh < 2; kh++) c = mfma32(af[kh][0], bf[kh][0], c);
                    hi[i][j] += c;
                }
            }
        }
        __syncthreads();
    }

    float *Ct = C + t * sC;
#pragma unroll
    for (int j = 0; j < TN; j++) {
        const int col = n0 + wn * WTN + j * 32 + fr;
        const float bv = EPI == 1 ? bias[(int64_t)t * N + col] : 0.0f;
#pragma unroll
        for (int i = 0; i < TM; i++) {
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int64_t row = m0 + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
                if (row < M) {
                    const float v = ACC == 1 ? hi[i][j][r] + lo[i][j][r] : hi[i][j][r];
                    Ct[row * N + col] = EPI == 1 ? relu_nan(v + bv) : v;
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// TN on the 32x32x16 MFMA: slab[s][t][m][n] = sum_{k in split s} A[t][k][m] B[t][k][n], A fp32 [Kd][M],
// B fp32 [Kd][N] (the weight gradient dz^T a3: both operands row-major over the minibatch's frames).
// Staging as merlin_gemm.hip's k_x6_tn (8 values of one k row per unit, split in registers) into
// plane images [32 k rows][RC chunks of 8 columns]; the operands come out k-contiguous through
// ds_read_b64_tr_b16: a 32x32x16 fragment (lane l: column l & 31, k = 8 (l >> 5) + j) is two
// transposed reads, 16-lane group g taking columns 16 (g & 1) .. + 15 and k rows 8 (g >> 1) + 4 h2 ..
// + 3.  A 32-lane half then reads 4 rows x 4 adjacent chunks; chunk c of row r sits at r * RC +
// (c ^ tr32_swz(r)), which puts those 16 chunks on 16 distinct 16-B bank slots for RC = 16 (XOR by
// 4 (r & 3)) and RC = 24 (row stride 24 = 8 mod 16 separates odd rows; XOR by 4 ((r >> 1) & 1)).
template <int RC>
__device__ __forceinline__ int tr32_swz(int row) {
    static_assert(RC % 16 == 0 || RC == 24, "row chunks");
    return RC % 16 == 0 ? (row & 3) << 2 : ((row >> 1) & 1) << 2;
}

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
typedef __attribute__((address_space(3))) char lds_char;

template <int RC>
__device__ __forceinline__ u32x4 tr32_frag(const u32x4 *img, int col0, int kh, int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int chunk = ((col0 + 16 * (g & 1)) >> 3) + (p >> 1);
    bf16x4 v[2];
#pragma unroll
    for (int h2 = 0; h2 < 2; h2++) {
        const int row = 16 * kh + 8 * (g >> 1) + 4 * h2 + q;
        const int off = (row * RC + (chunk ^ tr32_swz<RC>(row))) * 16 + (p & 1) * 8;
        v[h2] = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4 *)((lds_char *)img + off));
    }
    return __builtin_bit_cast(u32x4, bf16x8{v[0][0], v[0][1], v[0][2], v[0][3], v[1][0], v[1][1], v[1][2], v[1][3]});
}

// PL 1: both operands already in x6 planes ([Kd][M/8][3][8], [Kd][N/8][3][8]), staged as 16-B chunk
// copies (no split work in the loop).
template <int BM, int BN, int WGM, int WGN, int PL = 0>
__global__ __launch_bounds__(64 * WGM * WGN) void k_x6_tn32(const void *__restrict__ Av, const void *__restrict__ Bv,
                                                            int64_t Kd, int M, int N, int64_t sA, int64_t sB,
                                                            int64_t kc, int tiles_n, int tiles, int S,
                                                            float *__restrict__ slab) {
    constexpr int NT = 64 * WGM * WGN;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int RCA = BM / 8, RCB = BN / 8;
    constexpr int QA = BK * RCA * (PL ? 3 : 1), QB = BK * RCB * (PL ? 3 : 1);  // units (chunks) per k step
    constexpr int UA = (QA + NT - 1) / NT, UB = (QB + NT - 1) / NT;
    static_assert(WTM % 32 == 0 && WTN % 32 == 0, "wave tile of 32 x 32 MFMA tiles");
    constexpr int PSA = BK * RCA, PSB = BK * RCB;
    constexpr int STAGE = 3 * (PSA + PSB);
    __shared__ u32x4 lds[2 * STAGE];

    // 1-D grid over (tower, split, tile), tile fastest, XCD-contiguous: the tiles of one split read the
    // same k rows of both operands, so they run together on one L2
    const int P = xcd_tile(blockIdx.x, gridDim.x);
    const int t = P / (S * tiles), s = (P / tiles) % S, L = P % tiles;
    const int tm = L / tiles_n, tn = L - tm * tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int64_t k0 = (int64_t)s * kc, k1 = std::min<int64_t>(Kd, k0 + kc);
    // rows in float4s (fp32) or 16-B chunks (planes); the tile's first column in the same unit
    const int64_t rowA = PL ? M / 8 * 3 : M / 4, rowB = PL ? N / 8 * 3 : N / 4;
    const float4 *A = static_cast<const float4 *>(Av) + t * sA + (PL ? m0 / 8 * 3 : m0 / 4);
    const float4 *B = static_cast<const float4 *>(Bv) + t * sB + (PL ? n0 / 8 * 3 : n0 / 4);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WGN, wn = w - (w / WGN) * WGN;

    int ka[UA], oa[UA], la[UA];
#pragma unroll
    for (int i = 0; i < UA; i++) {
        const int q = std::min(tid + i * NT, QA - 1);
        if constexpr (PL) {  // chunk (k, g, p): memory order within a k row is [g][p]
            const int k = q / (RCA * 3), rem = q - k * (RCA * 3), g = rem / 3, p = rem - g * 3;
            ka[i] = k;
            oa[i] = rem;
            la[i] = p * PSA + k * RCA + (g ^ tr32_swz<RCA>(k));
        } else {
            const int k = q / RCA, g = q - (q / RCA) * RCA;
            ka[i] = k;
            oa[i] = g * 2;
            la[i] = k * RCA + (g ^ tr32_swz<RCA>(k));
        }
    }
    int kb[UB], ob[UB], lb[UB];
#pragma unroll
    for (int i = 0; i < UB; i++) {
        const int q = std::min(tid + i * NT, QB - 1);
        if constexpr (PL) {
            const int k = q / (RCB * 3), rem = q - k * (RCB * 3), g = rem / 3, p = rem - g * 3;
            kb[i] = k;
            ob[i] = rem;
            lb[i] = 3 * PSA + p * PSB + k * RCB + (g ^ tr32_swz<RCB>(k));
        } else {
            const int k = q / RCB, g = q - (q / RCB) * RCB;
            kb[i] = k;
            ob[i] = g * 2;
            lb[i] = 3 * PSA + k * RCB + (g ^ tr32_swz<RCB>(k));
        }
    }
    const float4 zero = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    constexpr int W = PL ? 1 : 2;  // float4s per unit
    float4 ra[UA][W], rb[UB][W];
    // full steps (every one but a split's last) read row pointers + a wave-uniform offset (no per-lane clamp)
    const float4 *pa[UA], *pb[UB];
#pragma unroll
    for (int i = 0; i < UA; i++) pa[i] = A + (k0 + ka[i]) * rowA + oa[i];
#pragma unroll
    for (int i = 0; i < UB; i++) pb[i] = B + (k0 + kb[i]) * rowB + ob[i];
    auto load = [&](int64_t kk) {
        if (kk + BK <= k1) {
            const int64_t da = (kk - k0) * rowA, db = (kk - k0) * rowB;
#pragma unroll
            for (int i = 0; i < UA; i++)
#pragma unroll
                for (int v = 0; v < W; v++) ra[i][v] = pa[i][da + v];
#pragma unroll
            for (int i = 0; i < UB; i++)
#pragma unroll
                for (int v = 0; v < W; v++) rb[i][v] = pb[i][db + v];
            return;
        }
#pragma unroll
        for (int i = 0; i < UA; i++) {
            const int64_t k = kk + ka[i];
            const float4 *src = A + std::min(k, k1 - 1) * rowA + oa[i];
#pragma unroll
            for (int v = 0; v < W; v++) ra[i][v] = src[v];  // zeroed when staged (no select next to the load)
        }
#pragma unroll
        for (int i = 0; i < UB; i++) {
            const int64_t k = kk + kb[i];
            const float4 *src = B + std::min(k, k1 - 1) * rowB + ob[i];
#pragma unroll
            for (int v = 0; v < W; v++) rb[i][v] = src[v];
        }
    };
    auto store = [&](int buf, int64_t kk) {  // the registers hold the rows of step kk; rows past k1 stage as zero
        u32x4 *st = lds + buf * STAGE;
#pragma unroll
        for (int i = 0; i < UA; i++)
            if (QA % NT == 0 || i + 1 < UA || tid + i * NT < QA) {
                const bool in = kk + ka[i] < k1;
                if constexpr (PL) {
                    st[la[i]] = __builtin_bit_cast(u32x4, in ? ra[i][0] : zero);
                } else {
                    u32x4 p0, p1, p2;
                    split8(in ? ra[i][0] : zero, in ? ra[i][W - 1] : zero, p0, p1, p2);
                    st[la[i]] = p0;
                    st[PSA + la[i]] = p1;
                    st[2 * PSA + la[i]] = p2;
                }
            }
#pragma unroll
        for (int i = 0; i < UB; i++)
            if (QB % NT == 0 || i + 1 < UB || tid + i * NT < QB) {
                const bool in = kk + kb[i] < k1;
                if constexpr (PL) {
                    st[lb[i]] = __builtin_bit_cast(u32x4, in ? rb[i][0] : zero);
                } else {
                    u32x4 p0, p1, p2;
                    split8(in ? rb[i][0] : zero, in ? rb[i][W - 1] : zero, p0, p1, p2);
                    st[lb[i]] = p0;
                    st[PSB + lb[i]] = p1;
                    st[2 * PSB + lb[i]] = p2;
                }
            }
    };

    // the big products a0 b0 in hi, the five small ones (smallest first) in lo, added once at the end
    f32x16 hi[TM][TN], lo[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++) {
            hi[i][j] = f32x16{};
            lo[i][j] = f32x16{};
        }

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
#pragma unroll
        for (int i = 0; i < TM; i++) {
            u32x4 af[2][3];
#pragma unroll
            for (int kh = 0; kh < 2; kh++)
#pragma unroll
                for (int p = 0; p < 3; p++) af[kh][p] = tr32_frag<RCA>(sAl + p * PSA, wm * WTM + i * 32, kh, lane);
#pragma unroll
            for (int j = 0; j < TN; j++) {
                u32x4 bf[2][3];
#pragma unroll
                for (int kh = 0; kh < 2; kh++)
#pragma unroll
                    for (int p = 0; p < 3; p++)
                        bf[kh][p] = tr32_frag<RCB>(sBl + p * PSB, wn * WTN + j * 32, kh, lane);
                f32x16 l = lo[i][j], h = hi[i][j];
#pragma unroll
                for (int kh = 0; kh < 2; kh++) {
                    l = mfma32(af[kh][2], bf[kh][0], l);
                    l = mfma32(af[kh][1], bf[kh][1], l);
                    l = mfma32(af[kh][0], bf[kh][2], l);
                    l = mfma32(af[kh][1], bf[kh][0], l);
                    l = mfma32(af[kh][0], bf[kh][1], l);
                    h = mfma32(af[kh][0], bf[kh][0], h);
                }
                lo[i][j] = l;
                hi[i][j] = h;
            }
        }
        __syncthreads();
    }

    float *St = slab + ((int64_t)s * (gridDim.x / (S * tiles)) + t) * (int64_t)M * N;
    const int fr = lane & 31, fh = lane >> 5;
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int row = m0 + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
                St[(int64_t)row * N + n0 + wn * WTN + j * 32 + fr] = hi[i][j][r] + lo[i][j][r];
            }
}

// TN with 16-deep k steps and a bigger block tile: 256 x 192 (both of fc1's weight-gradient dimensions in 2 x 3
// tiles) over 8 waves of 64 x 96.  Per MFMA it stages, splits and reads from LDS 35-65 % less than the 128 x 192 /
// 32-deep form (the split and the staging are per element of the tile's edges, the MFMAs per element of its
// area); two 43-KB LDS stages.  The accumulators are chunked per k step (the step's six plane products of a
// 32 x 32 tile in a fresh register set, added to the running sum once): 96 + 16 registers instead of the
// 192 of split hi / lo sums.
template <int BM, int BN, int WGM, int WGN>
__global__ __launch_bounds__(64 * WGM * WGN) void k_x6_tn32k16(const float4 *__restrict__ A,
                                                               const float4 *__restrict__ B, int64_t Kd, int M, int N,
                                                               int64_t sA, int64_t sB, int64_t kc, int tiles_n,
                                                               int tiles, int S, float *__restrict__ slab) {
    constexpr int K16 = 16;
    constexpr int NT = 64 * WGM * WGN;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int RCA = BM / 8, RCB = BN / 8;
    constexpr int QA = K16 * RCA, QB = K16 * RCB;
    constexpr int UA = (QA + NT - 1) / NT, UB = (QB + NT - 1) / NT;
    static_assert(WTM % 32 == 0 && WTN % 32 == 0, "wave tile of 32 x 32 MFMA tiles");
    constexpr int PSA = K16 * RCA, PSB = K16 * RCB;
    constexpr int STAGE = 3 * (PSA + PSB);
    __shared__ u32x4 lds[2 * STAGE];

    const int P = xcd_tile(blockIdx.x, gridDim.x);
    const int t = P / (S * tiles), s = (P / tiles) % S, L = P % tiles;
    const int tm = L / tiles_n, tn = L - tm * tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int64_t k0 = (int64_t)s * kc, k1 = std::min<int64_t>(Kd, k0 + kc);
    const int64_t rowA = M / 4, rowB = N / 4;
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
        la[i] = k * RCA + (g ^ tr32_swz<RCA>(k));
    }
    int kb[UB], ob[UB], lb[UB];
#pragma unroll
    for (int i = 0; i < UB; i++) {
        const int q = std::min(tid + i * NT, QB - 1);
        const int k = q / RCB, g = q - (q / RCB) * RCB;
        kb[i] = k;
        ob[i] = g * 2;
        lb[i] = 3 * PSA + k * RCB + (g ^ tr32_swz<RCB>(k));
    }
    const float4 zero = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    float4 ra[UA][2], rb[UB][2];
    const float4 *pa[UA], *pb[UB];
#pragma unroll
    for (int i = 0; i < UA; i++) pa[i] = A + (k0 + ka[i]) * rowA + oa[i];
#pragma unroll
    for (int i = 0; i < UB; i++) pb[i] = B + (k0 + kb[i]) * rowB + ob[i];
    auto load = [&](int64_t kk) {
        if (kk + K16 <= k1) {  // full step: row pointers + a wave-uniform offset
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

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++) acc[i][j] = f32x16{};

    if (k0 < k1) {
        load(k0);
        store(0, k0);
        if (k0 + K16 < k1) load(k0 + K16);
        __syncthreads();
    }
    int buf = 0;
    for (int64_t kk = k0; kk < k1; kk += K16, buf ^= 1) {
        if (kk + K16 < k1) store(buf ^ 1, kk + K16);
        if (kk + 2 * K16 < k1) load(kk + 2 * K16);
        const u32x4 *sAl = lds + buf * STAGE, *sBl = sAl + 3 * PSA;
        u32x4 af[TM][3];
#pragma unroll
        for (int i = 0; i < TM; i++)
#pragma unroll
            for (int p = 0; p < 3; p++) af[i][p] = tr32_frag<RCA>(sAl + p * PSA, wm * WTM + i * 32, 0, lane);
#pragma unroll
        for (int j = 0; j < TN; j++) {
            u32x4 bf[3];
#pragma unroll
            for (int p = 0; p < 3; p++) bf[p] = tr32_frag<RCB>(sBl + p * PSB, wn * WTN + j * 32, 0, lane);
#pragma unroll
            for (int i = 0; i < TM; i++) {
                f32x16 c = mfma32(af[i][2], bf[0], f32x16{});
                c = mfma32(af[i][1], bf[1], c);
                c = mfma32(af[i][0], bf[2], c);
                c = mfma32(af[i][1], bf[0], c);
                c = mfma32(af[i][0], bf[1], c);
                c = mfma32(af[i][0], bf[0], c);
                acc[i][j] += c;
            }
        }
        __syncthreads();
    }

    float *St = slab + ((int64_t)s * (gridDim.x / (S * tiles)) + t) * (int64_t)M * N;
    const int fr = lane & 31, fh = lane >> 5;
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int row = m0 + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
                St[(int64_t)row * N + n0 + wn * WTN + j * 32 + fr] = acc[i][j][r];
            }
}

template <int BM, int BN, int WGM, int WGN>
hipError_t tn32k16_launch(const void *A, const void *B, int64_t Kd, int M, int N, int T, int64_t sA, int64_t sB,
                          int splits, float *slab, hipStream_t s, int *S_out) {
    if (M % BM || N % BN) return hipErrorInvalidValue;
    const int tiles_n = N / BN, tiles = (M / BM) * tiles_n;
    int S = std::max(1, splits);
    int64_t kc = (Kd + S - 1) / S;
    kc = (kc + 15) / 16 * 16;
    S = (int)std::max<int64_t>(1, (Kd + kc - 1) / kc);
    *S_out = S;
    hipLaunchKernelGGL((k_x6_tn32k16<BM, BN, WGM, WGN>), dim3(tiles * S * T), dim3(64 * WGM * WGN), 0, s,
                       static_cast<const float4 *>(A), static_cast<const float4 *>(B), Kd, M, N, sA, sB, kc, tiles_n,
                       tiles, S, slab);
    return hipGetLastError();
}

// NT with 16-deep k steps, four waves and two blocks per CU.  The 8-wave kernels above hold a whole CU (one block:
// 122-147 KB of LDS), and one barrier per k step keeps both waves of each SIMD in the same phase, so the matrix
// pipe idles while they split, stage and wait for fragments together.  Here a block is one wave per SIMD with a
// 61-74 KB two-stage LDS ring, two blocks share a CU, and the two waves of a SIMD come from different blocks:
// one's staging runs beside the other's MFMAs.  Per MFMA the split, the staging and the fragment reads are
// smaller too (wave tiles of 128 x 64 / 64 x 96).  Accumulators chunked per k step (the step's six plane
// products of a 32 x 32 tile in a fresh set, added to the running sum once).  LDS plane images: rows of two
// 16-B chunks, chunk index XOR (row >> 3) & 1 (the ds_read_b128 fragment reads of each lane group hit 16
// distinct 16-B bank slots).
template <int BM, int BN, int WGM, int WGN, int EPI>
__global__ __launch_bounds__(64 * WGM * WGN, 2) void k_x6_nt32b(const float4 *__restrict__ A, const u32x4 *__restrict__ B,
                                                                int64_t M, int N, int K, int64_t sA, int64_t sB,
                                                                const float *__restrict__ bias, float *__restrict__ C,
                                                                int64_t sC, int tiles_n) {
    constexpr int K16 = 16;
    constexpr int NT = 64 * WGM * WGN;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int QA = BM * 2;           // A units (row, group of 8 values) per k step
    constexpr int QB = BN * 6;           // B 16-B chunks (row, group, plane) per k step
    constexpr int UA = (QA + NT - 1) / NT, CB = (QB + NT - 1) / NT;
    static_assert(WTM % 32 == 0 && WTN % 32 == 0, "wave tile of 32 x 32 MFMA tiles");
    constexpr int PSA = BM * 2, PSB = BN * 2;  // chunks per plane image
    constexpr int STAGE = 3 * (PSA + PSB);
    __shared__ u32x4 lds[2 * STAGE];

    const int t = blockIdx.y;
    const int L = xcd_tile(blockIdx.x, gridDim.x);
    const int tm = L / tiles_n, tn = L - tm * tiles_n;
    const int64_t m0 = (int64_t)tm * BM;
    const int n0 = tn * BN;
    const int64_t rowA = K / 4;                 // float4s per A row
    const int64_t rowB = (int64_t)(K / 8) * 3;  // chunks per B row
    A += t * sA;
    B += t * sB;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WGN, wn = w - (w / WGN) * WGN;

    int oa[UA], la[UA];  // A: float4 offset of the unit's first value at k step 0; LDS chunk of plane 0
#pragma unroll
    for (int i = 0; i < UA; i++) {
        const int q = std::min(tid + i * NT, QA - 1);
        const int row = q >> 1, g = q & 1;
        oa[i] = (int)(std::min<int64_t>(m0 + row, M - 1) * rowA) + g * 2;
        la[i] = row * 2 + (g ^ ((row >> 3) & 1));
    }
    int ob[CB], lb[CB];
#pragma unroll
    for (int i = 0; i < CB; i++) {
        const int q = std::min(tid + i * NT, QB - 1);
        const int row = q / 6, rem = q - row * 6, g = rem / 3, p = rem - g * 3;
        ob[i] = (int)((int64_t)(n0 + row) * rowB) + g * 3 + p;
        lb[i] = 3 * PSA + p * PSB + row * 2 + (g ^ ((row >> 3) & 1));
    }
    float4 ra[UA][2];
    u32x4 rb[CB];
    auto load = [&](int kt) {
#pragma unroll
        for (int i = 0; i < UA; i++) {
            ra[i][0] = A[(int64_t)oa[i] + kt * 4];
            ra[i][1] = A[(int64_t)oa[i] + kt * 4 + 1];
        }
#pragma unroll
        for (int i = 0; i < CB; i++) rb[i] = B[ob[i] + kt * 6];
    };
    auto store = [&](int buf) {
        u32x4 *st = lds + buf * STAGE;
#pragma unroll
        for (int i = 0; i < UA; i++)
            if (QA % NT == 0 || i + 1 < UA || tid + i * NT < QA) {
                u32x4 p0, p1, p2;
                split8(ra[i][0], ra[i][1], p0, p1, p2);
                st[la[i]] = p0;
                st[PSA + la[i]] = p1;
                st[2 * PSA + la[i]] = p2;
            }
#pragma unroll
        for (int i = 0; i < CB; i++)
            if (QB % NT == 0 || i + 1 < CB || tid + i * NT < QB) st[lb[i]] = rb[i];
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++) acc[i][j] = f32x16{};

    // fragment reads: row (tile base + lane & 31), chunk (lane >> 5) XOR (row >> 3) & 1
    const int fr = lane & 31, fh = lane >> 5;
    const int nk = K / K16;
    load(0);
    store(0);
    if (nk > 1) load(1);
    __syncthreads();
    for (int kt = 0; kt < nk; kt++) {
        const int buf = kt & 1;
        if (kt + 1 < nk) store(buf ^ 1);
        if (kt + 2 < nk) load(kt + 2);
        const u32x4 *sAl = lds + buf * STAGE, *sBl = sAl + 3 * PSA;
        u32x4 bf[TN][3];
#pragma unroll
        for (int j = 0; j < TN; j++) {
            const int row = wn * WTN + j * 32 + fr;
#pragma unroll
            for (int p = 0; p < 3; p++) bf[j][p] = sBl[p * PSB + row * 2 + (fh ^ ((row >> 3) & 1))];
        }
#pragma unroll
        for (int i = 0; i < TM; i++) {
            const int row = wm * WTM + i * 32 + fr;
            u32x4 af[3];
#pragma unroll
            for (int p = 0; p < 3; p++) af[p] = sAl[p * PSA + row * 2 + (fh ^ ((row >> 3) & 1))];
#pragma unroll
            for (int j = 0; j < TN; j++) {
                f32x16 c = mfma32(af[2], bf[j][0], f32x16{});
                c = mfma32(af[1], bf[j][1], c);
                c = mfma32(af[0], bf[j][2], c);
                c = mfma32(af[1], bf[j][0], c);
                c = mfma32(af[0], bf[j][1], c);
                c = mfma32(af[0], bf[j][0], c);
                acc[i][j] += c;
            }
        }
        __syncthreads();
    }

    float *Ct = C + t * sC;
#pragma unroll
    for (int j = 0; j < TN; j++) {
        const int col = n0 + wn * WTN + j * 32 + fr;
        const float bv = EPI == 1 ? bias[(int64_t)t * N + col] : 0.0f;
#pragma unroll
        for (int i = 0; i < TM; i++) {
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int64_t row = m0 + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
                if (row < M) {
                    const float v = acc[i][j][r];
                    Ct[row * N + col] = EPI == 1 ? relu_nan(v + bv) : v;
                }
            }
        }
    }
}

template <int BM, int BN, int WGM, int WGN>
hipError_t nt32b_launch(const float *A, const u32x4 *B, int64_t M, int N, int K, int T, int64_t sA, int64_t sB,
                        const float *bias, float *C, int64_t sC, hipStream_t s) {
    if (N % BN || K % 16) return hipErrorInvalidValue;
    if ((M + BM) * (int64_t)(K / 4) > INT32_MAX) return hipErrorInvalidValue;  // 32-bit A offsets
    const int64_t tiles_m = (M + BM - 1) / BM;
    const int tiles_n = N / BN;
    const dim3 grid((unsigned)(tiles_m * tiles_n), T);
    const float4 *a = reinterpret_cast<const float4 *>(A);
    if (bias)
        hipLaunchKernelGGL((k_x6_nt32b<BM, BN, WGM, WGN, 1>), grid, dim3(64 * WGM * WGN), 0, s, a, B, M, N, K, sA, sB, bias,
                           C, sC, tiles_n);
    else
        hipLaunchKernelGGL((k_x6_nt32b<BM, BN, WGM, WGN, 0>), grid, dim3(64 * WGM * WGN), 0, s, a, B, M, N, K, sA, sB,
                           nullptr, C, sC, tiles_n);
    return hipGetLastError();
}

template <int BM, int BN, int WGM, int WGN, int ACC, int APL = 0>
hipError_t nt32_launch(const void *A, const u32x4 *B, int64_t M, int N, int K, int T, int64_t sA, int64_t sB,
                       const float *bias, float *C, int64_t sC, hipStream_t s) {
    if (N % BN) return hipErrorInvalidValue;
    // planes-A form: the kernel keeps A chunk offsets (and B's, N * K * 3 / 8) in 32 bits
    if (APL && (M + BM) * ((int64_t)(K / 8) * 3) > INT32_MAX) return hipErrorInvalidValue;
    if ((int64_t)N * (K / 8) * 3 > INT32_MAX) return hipErrorInvalidValue;
    const int64_t tiles_m = (M + BM - 1) / BM;
    const int tiles_n = N / BN;
    if (tiles_m * tiles_n > INT32_MAX) return hipErrorInvalidValue;
    const dim3 grid((unsigned)(tiles_m * tiles_n), T);
    if (bias)
        hipLaunchKernelGGL((k_x6_nt32<BM, BN, WGM, WGN, 1, ACC, APL>), grid, dim3(64 * WGM * WGN), 0, s, A, B, M, N, K,
                           sA, sB, bias, C, sC, tiles_n);
    else
        hipLaunchKernelGGL((k_x6_nt32<BM, BN, WGM, WGN, 0, ACC, APL>), grid, dim3(64 * WGM * WGN), 0, s, A, B, M, N, K,
                           sA, sB, nullptr, C, sC, tiles_n);
    return hipGetLastError();
}

template <int BM, int BN, int WGM, int WGN, int PL = 0>
hipError_t tn32_launch(const void *A, const void *B, int64_t Kd, int M, int N, int T, int64_t sA, int64_t sB,
                       int splits, float *slab, hipStream_t s, int *S_out) {
    if (M % BM || N % BN) return hipErrorInvalidValue;
    const int tiles_n = N / BN, tiles = (M / BM) * tiles_n;
    int S = std::max(1, splits);
    int64_t kc = (Kd + S - 1) / S;
    kc = (kc + BK - 1) / BK * BK;
    S = (int)std::max<int64_t>(1, (Kd + kc - 1) / kc);
    *S_out = S;
    hipLaunchKernelGGL((k_x6_tn32<BM, BN, WGM, WGN, PL>), dim3(tiles * S * T), dim3(64 * WGM * WGN), 0, s, A, B, Kd, M, N,
                       sA, sB, kc, tiles_n, tiles, S, slab);
    return hipGetLastError();
}

}  // namespace

// the 32x32x16 weight-gradient kernels (launch_x6_gemm_tn forwards cfg >= 20 here); the slab count
// actually used comes back in *S_out for the fold
hipError_t launch_x6_gemm_tn32(const float *A, const float *B, int64_t Kd, int M, int N, int T, int64_t a_stride,
                               int64_t b_stride, int splits, float *slab, int cfg, hipStream_t s, int *S_out) {
    if (cfg >= 30) {  // both operands as x6 planes (strides in values: 3 chunks per 8)
        const int64_t sA = a_stride / 8 * 3, sB = b_stride / 8 * 3;
        switch (cfg) {
            case 30: return tn32_launch<128, 192, 4, 2, 1>(A, B, Kd, M, N, T, sA, sB, splits, slab, s, S_out);
            default: return hipErrorInvalidValue;
        }
    }
    const int64_t sA = a_stride / 4, sB = b_stride / 4;
    const float *a = A, *b = B;
    switch (cfg) {
        // 128 x 192 blocks: 8 waves of 32 x 96, or 4 waves (one per SIMD) of 64 x 96
        case 20: return tn32_launch<128, 192, 4, 2>(a, b, Kd, M, N, T, sA, sB, splits, slab, s, S_out);
        case 21: return tn32_launch<128, 192, 2, 2>(a, b, Kd, M, N, T, sA, sB, splits, slab, s, S_out);
        // 256 x 192 blocks, 16-deep k steps, 8 waves of 64 x 96 (k_x6_tn32k16)
        case 24: return tn32k16_launch<256, 192, 4, 2>(a, b, Kd, M, N, T, sA, sB, splits, slab, s, S_out);
        case 25: return tn32k16_launch<256, 192, 8, 1>(a, b, Kd, M, N, T, sA, sB, splits, slab, s, S_out);
        default: return hipErrorInvalidValue;
    }
}

// cfg numbers continue merlin_gemm.hip's (launch_x6_gemm_nt forwards cfg >= 20 here)
hipError_t launch_x6_gemm_nt32(const float *A, const void *B, int64_t M, int N, int K, int T, int64_t a_stride,
                               int64_t b_stride, const float *bias, float *C, int64_t c_stride, int cfg,
                               hipStream_t s) {
    const u32x4 *b = static_cast<const u32x4 *>(B);
    const int64_t sB = b_stride / 8 * 3;
    if (cfg >= 30) {  // A as x6 planes too (a_stride in values: 3 chunks per 8)
        const int64_t sA = a_stride / 8 * 3;
        switch (cfg) {
            case 30: return nt32_launch<256, 128, 4, 2, 1, 1>(A, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
            case 32: return nt32_launch<128, 192, 4, 2, 1, 1>(A, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
            default: return hipErrorInvalidValue;
        }
    }
    const float *a = A;
    const int64_t sA = a_stride / 4;
    switch (cfg) {
        // k_x6_nt32b: 16-deep k steps, 4 waves, two blocks per CU (forward 256 x 128, input gradient 128 x 192)
        case 26: return nt32b_launch<256, 128, 2, 2>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        case 27: return nt32b_launch<128, 192, 2, 2>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        case 28: return nt32b_launch<128, 128, 2, 2>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        // small row counts (the rollout's fc1: 4,096 rows): 64 x 128 tiles, twice the blocks
        case 29: return nt32b_launch<64, 128, 2, 2>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        // forward shape (N = 512): 256 x 128 blocks, 8 waves of 64 x 64
        case 20: return nt32_launch<256, 128, 4, 2, 1>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        case 21: return nt32_launch<256, 128, 4, 2, 0>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        // input-gradient shape (N = 576): 128 x 192 blocks, 8 waves of 32 x 96
        case 22: return nt32_launch<128, 192, 4, 2, 1>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        case 23: return nt32_launch<128, 192, 4, 2, 0>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        // 256 x 128 over 4 waves (1 per SIMD) of 128 x 64
        case 24: return nt32_launch<256, 128, 2, 2, 1>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        // 128 x 128, 4 waves of 64 x 64 (2 blocks per CU)
        case 25: return nt32_launch<128, 128, 2, 2, 1>(a, b, M, N, K, T, sA, sB, bias, C, c_stride, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace merlin
