// merlin_h3.hip -- fc1's fp32 GEMMs on the f16 matrix cores in two-plane form ("h3": three f16 products per fp32
// product; src/actor_critic.py:31-41, the Linear(576, 512) of both towers in PPO.update, src/ppo.py:136-155).
//
// Every fp32 operand x of a GEMM is used as x' = x * 2^e (e: one power of two per tensor and tower, from its max
// |x|, so that max |x'| lies in [2^14, 2^15): inside the f16 range with room to round) and two f16 planes
//     h = f16(x'),   l = f16((x' - h) * 2^11)          (round to nearest even)
// x' - h is exact in fp32 and |x' - h| <= 2^-11 |h|, so l lies inside the f16 range too and carries the next 11
// bits: |x' - (h + l 2^-11)| <= 2^-23 |x'| for every |x'| >= 2^-12 (values within 2^26 of the tensor's max; below
// that the error is 2^-36 absolute, i.e. 2^-50 of the max).  A product a b is then
//     a' b' = h_a h_b + 2^-11 (h_a l_b + l_a h_b) + 2^-22 l_a l_b
// and the GEMM sums the first three on the f16 MFMA (v_mfma_f32_32x32x16_f16: every f16 x f16 product is exact in
// the fp32 accumulator) into two accumulators -- hi = sum h_a h_b, lo = sum (h_a l_b + l_a h_b) -- combined once in
// the epilogue, C = (hi + 2^-11 lo) * 2^-(e_A + e_B) (exact power-of-two scalings).  Per product the error is
// <= ~2^-21 |a b| (the dropped 2^-22 l_a l_b and the planes' rounding), of random sign; per output it stays below
// the error of the fp32 GEMM on the f32 MFMA (hipBLASLt) on the same operands (tests/test_gpu_h3.py holds it to
// that against float64).  That is Ootomo & Yokota's fp16 split (IJHPCA 2022) with a per-tensor exponent.
//
// Half the matrix-core work of the exact three-plane bf16 form (merlin_gemm.hip, six products) for an error still
// below the fp32 GEMM's; 4 B of LDS per staged value (two f16 planes) instead of 6.
//
// Scales: merlin_h3_amax writes max |x| per tower as float bits (uint32, atomicMax of non-negative floats); the
// GEMMs read it and derive e in-kernel, so no host round trip.
#include <algorithm>

#include "merlin_internal.h"

namespace merlin {
namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
typedef __attribute__((address_space(3))) char lds_char;

constexpr int BK = 32;           // k per step
constexpr float LO_INV = 1.0f / 2048.0f;

__device__ __forceinline__ f32x16 mfma16(const u32x4 a, const u32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                   0);
}

__device__ __forceinline__ float relu_nan(float v) { return v != v ? v : fmaxf(v, 0.0f); }

__device__ __forceinline__ int xcd_tile(int b, int nb) {
    const int xcd = b & 7, q = nb >> 3, r = nb & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

// h3_exp / pow2f / h3_pair: merlin_internal.h (shared with the producers that write planes)

// an operand scale written by another kernel's atomics: read with a vector load at agent scope (L2-coherent), not
// through the scalar data cache a wave-uniform load would take
__device__ __forceinline__ uint32_t load_amax(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// 8 consecutive values (two float4) scaled by sc (sc2 = 2^11 sc) -> hi chunk p0, lo chunk p1
__device__ __forceinline__ void h3_split8(const float4 a, const float4 b, float sc, float sc2, u32x4 &p0, u32x4 &p1) {
    uint32_t h0, h1, h2, h3, l0, l1, l2, l3;
    h3_pair(a.x, a.y, sc, sc2, h0, l0);
    h3_pair(a.z, a.w, sc, sc2, h1, l1);
    h3_pair(b.x, b.y, sc, sc2, h2, l2);
    h3_pair(b.z, b.w, sc, sc2, h3, l3);
    p0 = u32x4{h0, h1, h2, h3};
    p1 = u32x4{l0, l1, l2, l3};
}

// ---------------------------------------------------------------------------------------------------------------
// amax[t] = max over the tower's rows x cols of |x| (float bits; the caller zeroes amax)
__global__ __launch_bounds__(256) void k_h3_amax(const float4 *__restrict__ x, int64_t n4, int64_t s4,
                                                 uint32_t *__restrict__ amax) {
    const int t = blockIdx.y;
    x += t * s4;
    uint32_t m = 0u;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n4; e += (int64_t)gridDim.x * 256) {
        const float4 v = x[e];
        m = std::max(m, std::max(std::max(__float_as_uint(v.x) & 0x7fffffffu, __float_as_uint(v.y) & 0x7fffffffu),
                                 std::max(__float_as_uint(v.z) & 0x7fffffffu, __float_as_uint(v.w) & 0x7fffffffu)));
    }
    for (int o = 32; o > 0; o >>= 1) m = std::max(m, (uint32_t)__shfl_xor((int)m, o));
    __shared__ uint32_t red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        m = std::max(std::max(red[0], red[1]), std::max(red[2], red[3]));
        if (m) atomicMax(amax + t, m);
    }
}

__global__ void k_h3_zero(uint32_t *__restrict__ amax, int T) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i < T) amax[i] = 0u;
}

// planes of a row-major [T][R][C] fp32 tensor: [T][R][C/8][2][8] f16 (per group of 8 values a hi chunk and a lo
// chunk), each tower scaled by its own 2^e
__global__ __launch_bounds__(256) void k_h3_split(const float4 *__restrict__ x, int64_t g8, const uint32_t *amax,
                                                  u32x4 *__restrict__ planes) {
    const int t = blockIdx.y;
    const int e = h3_exp(load_amax(amax + t));
    const float sc = pow2f(e), sc2 = pow2f(e + 11);
    x += t * g8 * 2;
    planes += t * g8 * 2;
    for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < g8; q += (int64_t)gridDim.x * 256) {
        u32x4 p0, p1;
        h3_split8(x[2 * q], x[2 * q + 1], sc, sc2, p0, p1);
        planes[2 * q] = p0;
        planes[2 * q + 1] = p1;
    }
}

// ---------------------------------------------------------------------------------------------------------------
// NT: C[t][m][n] = epi(sum_k A[t][m][k] B[t][n][k]); A fp32 [M][K] (split while staged), B h3 planes [N][K/8][2][8]
// (K % 32 == 0, N % BN == 0); EPI 1: relu(. + bias[t][n]).  grid (tiles_m * tiles_n, T).
// Block BM x BN, waves WGM x WGN, each wave (BM/WGM) x (BN/WGN) in 32 x 32 MFMA tiles.  LDS plane images: 64-B rows
// (a k step's 4 chunks of 8 values), chunk g stored at g XOR (row >> 2) & 3 -- a 32x32x16 fragment read (lane l:
// row l & 31, chunk 2 kh + (l >> 5)) hits 16 distinct 16-B bank slots per ds_read_b128 lane group; B's images padded
// by 12 chunks so a lane group's 8 staging writes (4 chunks of each plane) land on 8 distinct slots.  Two LDS
// stages, one barrier per k step, the step after next in registers.
template <int BM, int BN, int WGM, int WGN, int EPI>
__global__ __launch_bounds__(64 * WGM * WGN) void k_h3_nt(const float *__restrict__ A, const u32x4 *__restrict__ B,
                                                          const uint32_t *__restrict__ amaxA,
                                                          const uint32_t *__restrict__ amaxB, int64_t M, int N, int K,
                                                          int64_t sA, int64_t sB, const float *__restrict__ bias,
                                                          float *__restrict__ C, int64_t sC, int tiles_n,
    u32x4 *__restrict__ Pout) {
    constexpr int NT = 64 * WGM * WGN;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int QA = BM * 4, QB = BN * 8;  // A units (row, group of 8 values), B chunks (row, group, plane)
    constexpr int UA = (QA + NT - 1) / NT, CB = (QB + NT - 1) / NT;
    static_assert(WTM % 32 == 0 && WTN % 32 == 0, "wave tile of 32 x 32 MFMA tiles");
    constexpr int PSA = BM * 4, PSB = BN * 4 + 12;
    constexpr int STAGE = 2 * (PSA + PSB);
    __shared__ u32x4 lds[2 * STAGE];

    const int t = blockIdx.y;
    const int L = xcd_tile(blockIdx.x, gridDim.x);
    const int tm = L / tiles_n, tn = L - tm * tiles_n;
    const int64_t m0 = (int64_t)tm * BM;
    const int n0 = tn * BN;
    const int eA = h3_exp(load_amax(amaxA + t)), eB = h3_exp(load_amax(amaxB + t));
    const float scA = pow2f(eA), scA2 = pow2f(eA + 11);
    const int64_t rowB = (int64_t)(K / 8) * 2;  // chunks per B row
    B += t * sB;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WGN, wn = w - (w / WGN) * WGN;

    const float4 *ga[UA];
    int la[UA];
    u32x4 *pa[UA];  // plane output of this unit (the first column tile's blocks write A's planes; else null)
#pragma unroll
    for (int i = 0; i < UA; i++) {
        const int q = tid + i * NT;
        const int row = std::min(q >> 2, BM - 1), g = q & 3;
        ga[i] = reinterpret_cast<const float4 *>(A + t * sA + std::min<int64_t>(m0 + row, M - 1) * K) + g * 2;
        la[i] = row * 4 + (g ^ ((row >> 2) & 3));
        pa[i] = Pout && tn == 0 && m0 + row < M ? Pout + (t * sA + (m0 + row) * K) / 4 + g * 2 : nullptr;
    }
    int gb[CB], lb[CB];
#pragma unroll
    for (int i = 0; i < CB; i++) {
        const int q = tid + i * NT;
        const int row = std::min(q >> 3, BN - 1), g = (q >> 1) & 3, p = q & 1;
        gb[i] = (int)((int64_t)(n0 + row) * rowB + g * 2 + p);
        lb[i] = 2 * PSA + p * PSB + row * 4 + (g ^ ((row >> 2) & 3));
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
        for (int i = 0; i < CB; i++) rb[i] = B[gb[i] + kt * 8];
    };
    auto store = [&](int buf, int kt) {
        u32x4 *st = lds + buf * STAGE;
#pragma unroll
        for (int i = 0; i < UA; i++)
            if (QA % NT == 0 || i + 1 < UA || tid + i * NT < QA) {
                u32x4 p0, p1;
                h3_split8(ra[i][0], ra[i][1], scA, scA2, p0, p1);
                st[la[i]] = p0;
                st[PSA + la[i]] = p1;
                if (pa[i]) {
                    pa[i][kt * 8] = p0;
                    pa[i][kt * 8 + 1] = p1;
                }
            }
#pragma unroll
        for (int i = 0; i < CB; i++)
            if (QB % NT == 0 || i + 1 < CB || tid + i * NT < QB) st[lb[i]] = rb[i];
    };

    f32x16 hi[TM][TN], lo[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++) {
            hi[i][j] = f32x16{};
            lo[i][j] = f32x16{};
        }

    const int fr = lane & 31, fh = lane >> 5, fs = (fr >> 2) & 3;
    const int nk = K / BK;
    load(0);
    store(0, 0);
    if (nk > 1) load(1);
    __syncthreads();
    for (int kt = 0; kt < nk; kt++) {
        const int buf = kt & 1;
        if (kt + 1 < nk) store(buf ^ 1, kt + 1);
        if (kt + 2 < nk) load(kt + 2);
        const u32x4 *sAl = lds + buf * STAGE, *sBl = sAl + 2 * PSA;
        u32x4 bf[TN][2][2];
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int kh = 0; kh < 2; kh++)
#pragma unroll
                for (int p = 0; p < 2; p++)
                    bf[j][kh][p] = sBl[p * PSB + (wn * WTN + j * 32 + fr) * 4 + ((2 * kh + fh) ^ fs)];
#pragma unroll
        for (int i = 0; i < TM; i++) {
            u32x4 af[2][2];
#pragma unroll
            for (int kh = 0; kh < 2; kh++)
#pragma unroll
                for (int p = 0; p < 2; p++) af[kh][p] = sAl[p * PSA + (wm * WTM + i * 32 + fr) * 4 + ((2 * kh + fh) ^ fs)];
#pragma unroll
            for (int j = 0; j < TN; j++) {
                f32x16 l = lo[i][j], h = hi[i][j];
#pragma unroll
                for (int kh = 0; kh < 2; kh++) {
                    l = mfma16(af[kh][1], bf[j][kh][0], l);
                    l = mfma16(af[kh][0], bf[j][kh][1], l);
                    h = mfma16(af[kh][0], bf[j][kh][0], h);
                }
                lo[i][j] = l;
                hi[i][j] = h;
            }
        }
        __syncthreads();
    }

    const float inv = pow2f(-eA), invB = pow2f(-eB);
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
                    const float v = (hi[i][j][r] + lo[i][j][r] * LO_INV) * inv * invB;
                    Ct[row * N + col] = EPI == 1 ? relu_nan(v + bv) : v;
                }
            }
        }
    }
}

// The same NT product with the k step's split and staging interleaved into its MFMAs.  In k_h3_nt every k step is
// [split + stage the next step, VALU] -> [fragment reads -> MFMAs] -> barrier, and the two waves of a SIMD, held in
// step by the barrier, run their VALU blocks side by side and then their MFMA blocks: the matrix pipe idles through
// the first (PMC: MFMA busy 38 %, 3.3 VALU per MFMA).  Here the main loop has no conditional parts (the last two
// steps are peeled), the body reads all its fragments first, and sched_group_barrier hints lay the next step's
// split (VALU), its LDS stores and the global loads of the step after it between the MFMAs (guide T19).
// GA: A's rows gathered by 64-value chunks -- row m's chunk j (values 64 j .. 64 j + 63) is row amap[m * K / 64 + j]
// of A seen as [*][64] (K <= 64 * GA_CHUNKS; the launcher checks): the minibatch's conv3 rows through their patch
// representatives (merlin_tower_window_conv3_reuse), so the non-representative rows are never written.  The
// thread's chunk rows are read once into registers; a k step picks its chunk's with a uniform select.
constexpr int GA_CHUNKS = 9;
// EPI 2 (the update's fc1 forward): bias + ReLU as EPI 1, and the policy / value heads' dot products of the rows
// (src/actor_critic.py:41-46, Linear(512, A) on the actor tower's h, Linear(512, 1) on the critic's) folded into the
// epilogue, so h is not read again for them: every wave leaves, per row, the dot products of its WTN columns with
// the head weights (w0 [na][N] for tower 0, w1 [N] for tower 1) as partial [t][tn * WGN + wn][row][o], o < 4, and
// merlin_heads_combine adds a row's tiles_n * WGN partials in order.
struct HeadsArg {
    const float *w0, *w1;
    int na;
    float *part;
};
// AP (round 5): A arrives as h3 plane images (the same 4 B per value and addressing; conv3's representatives written
// as planes, merlin_tower_window_conv3_planes): staged as copies, no split
template <int BM, int BN, int WGM, int WGN, int EPI, bool GA, bool AP = false>
__device__ __forceinline__ void h3_ntp_body(const float *__restrict__ A, const u32x4 *__restrict__ B,
                                            const uint32_t *__restrict__ amaxA, const uint32_t *__restrict__ amaxB,
                                            int64_t M, int N, int K, int64_t sA, int64_t sB,
                                            const float *__restrict__ bias, float *__restrict__ C, int64_t sC,
                                            int tiles_n, u32x4 *__restrict__ Pout, const int32_t *__restrict__ amap,
                                            HeadsArg hd) {
    constexpr int NT = 64 * WGM * WGN;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int QA = BM * 4, QB = BN * 8;
    constexpr int UA = (QA + NT - 1) / NT, CB = (QB + NT - 1) / NT;
    static_assert(WTM % 32 == 0 && WTN % 32 == 0, "wave tile of 32 x 32 MFMA tiles");
    static_assert(QA % NT == 0 && QB % NT == 0, "whole staging units per thread");
    constexpr int PSA = BM * 4, PSB = BN * 4 + 12;
    constexpr int STAGE = 2 * (PSA + PSB);
    constexpr int NMFMA = TM * TN * 6;  // per k step and wave
    __shared__ u32x4 lds[2 * STAGE];

    const int t = blockIdx.y;
    const int L = xcd_tile(blockIdx.x, gridDim.x);
    const int tm = L / tiles_n, tn = L - tm * tiles_n;
    const int64_t m0 = (int64_t)tm * BM;
    const int n0 = tn * BN;
    const int eA = h3_exp(load_amax(amaxA + t)), eB = h3_exp(load_amax(amaxB + t));
    const float scA = pow2f(eA), scA2 = pow2f(eA + 11);
    const int64_t rowB = (int64_t)(K / 8) * 2;
    B += t * sB;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WGN, wn = w - (w / WGN) * WGN;

    const float4 *ga[UA];
    int la[UA];
    u32x4 *pa[UA];
    int32_t gx[GA ? UA : 1][GA ? GA_CHUNKS : 1];  // GA: the row's chunk rows
#pragma unroll
    for (int i = 0; i < UA; i++) {
        const int q = tid + i * NT;
        const int row = q >> 2, g = q & 3;
        const int64_t ar = std::min<int64_t>(m0 + row, M - 1);
        if constexpr (GA) {
            ga[i] = reinterpret_cast<const float4 *>(A + t * sA) + g * 2;
            const int kc = K / 64;
#pragma unroll
            for (int j = 0; j < GA_CHUNKS; j++) gx[i][j] = j < kc ? amap[ar * kc + j] : 0;
        } else {
            ga[i] = reinterpret_cast<const float4 *>(A + t * sA + ar * K) + g * 2;
        }
        la[i] = row * 4 + (g ^ ((row >> 2) & 3));
        pa[i] = !GA && Pout && tn == 0 && m0 + row < M ? Pout + (t * sA + (m0 + row) * K) / 4 + g * 2 : nullptr;
    }
    int gb[CB], lb[CB];
#pragma unroll
    for (int i = 0; i < CB; i++) {
        const int q = tid + i * NT;
        const int row = q >> 3, g = (q >> 1) & 3, p = q & 1;
        gb[i] = (int)((int64_t)(n0 + row) * rowB + g * 2 + p);
        lb[i] = 2 * PSA + p * PSB + row * 4 + (g ^ ((row >> 2) & 3));
    }
    float4 ra[UA][2];
    u32x4 rb[CB];
    auto load = [&](int kt) {
#pragma unroll
        for (int i = 0; i < UA; i++) {
            if constexpr (GA) {
                const int kj = kt >> 1;
                int32_t r = gx[i][0];
#pragma unroll
                for (int j = 1; j < GA_CHUNKS; j++) r = kj == j ? gx[i][j] : r;
                const float4 *src = ga[i] + (int64_t)r * 16 + (kt & 1) * 8;
                ra[i][0] = src[0];
                ra[i][1] = src[1];
            } else {
                ra[i][0] = ga[i][(int64_t)kt * 8];
                ra[i][1] = ga[i][(int64_t)kt * 8 + 1];
            }
        }
#pragma unroll
        for (int i = 0; i < CB; i++) rb[i] = B[gb[i] + kt * 8];
    };
    auto store = [&](int buf, int kt) {
        u32x4 *st = lds + buf * STAGE;
#pragma unroll
        for (int i = 0; i < UA; i++) {
            u32x4 p0, p1;
            if constexpr (AP) {
                p0 = __builtin_bit_cast(u32x4, ra[i][0]);
                p1 = __builtin_bit_cast(u32x4, ra[i][1]);
            } else {
                h3_split8(ra[i][0], ra[i][1], scA, scA2, p0, p1);
            }
            st[la[i]] = p0;
            st[PSA + la[i]] = p1;
            if (pa[i]) {
                pa[i][kt * 8] = p0;
                pa[i][kt * 8 + 1] = p1;
            }
        }
#pragma unroll
        for (int i = 0; i < CB; i++) st[lb[i]] = rb[i];
    };

    f32x16 hi[TM][TN], lo[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++) {
            hi[i][j] = f32x16{};
            lo[i][j] = f32x16{};
        }
    const int fr = lane & 31, fh = lane >> 5, fs = (fr >> 2) & 3;
    auto compute = [&](int buf) {
        const u32x4 *sAl = lds + buf * STAGE, *sBl = sAl + 2 * PSA;
        u32x4 af[TM][2][2], bf[TN][2][2];
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int kh = 0; kh < 2; kh++)
#pragma unroll
                for (int p = 0; p < 2; p++)
                    bf[j][kh][p] = sBl[p * PSB + (wn * WTN + j * 32 + fr) * 4 + ((2 * kh + fh) ^ fs)];
#pragma unroll
        for (int i = 0; i < TM; i++)
#pragma unroll
            for (int kh = 0; kh < 2; kh++)
#pragma unroll
                for (int p = 0; p < 2; p++)
                    af[i][kh][p] = sAl[p * PSA + (wm * WTM + i * 32 + fr) * 4 + ((2 * kh + fh) ^ fs)];
#pragma unroll
        for (int i = 0; i < TM; i++)
#pragma unroll
            for (int j = 0; j < TN; j++) {
                f32x16 l = lo[i][j], h = hi[i][j];
#pragma unroll
                for (int kh = 0; kh < 2; kh++) {
                    l = mfma16(af[i][kh][1], bf[j][kh][0], l);
                    l = mfma16(af[i][kh][0], bf[j][kh][1], l);
                    h = mfma16(af[i][kh][0], bf[j][kh][0], h);
                }
                lo[i][j] = l;
                hi[i][j] = h;
            }
    };

    const int nk = K / BK;  // >= 2 (K % 32 == 0, K >= 64: the launcher checks)
    load(0);
    store(0, 0);
    load(1);
    __syncthreads();
    int kt = 0;
    for (; kt + 2 < nk; kt++) {
        const int buf = kt & 1;
        compute(buf);
        store(buf ^ 1, kt + 1);
        load(kt + 2);
        // the fragment reads first, then each MFMA followed by a share of the split, the stores and the loads
        __builtin_amdgcn_sched_group_barrier(0x100, TM * 4 + TN * 4, 0);
#pragma unroll
        for (int m = 0; m < NMFMA; m++) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
            if (m % 4 == 3) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
            if (m >= NMFMA / 2 && m % 2 == 0) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
        __syncthreads();
    }
    compute(kt & 1);  // kt = nk - 2: stage the last step
    store((kt & 1) ^ 1, kt + 1);
    __syncthreads();
    compute((kt + 1) & 1);

    const float inv = pow2f(-eA), invB = pow2f(-eB);
    float *Ct = C + t * sC;
    if constexpr (EPI >= 2) {  // EPI 3: the heads only (the acting path: h itself is not needed)
        // per i: the 16 rows x 4 head outputs of this lane's two columns, then a reduce-scatter over the 32 column
        // lanes of the half-wave (xor 16 .. 1, each step keeping the half of the values its lane bit selects): lane fr
        // ends with output o = fr >> 3 of rows r = 2 (fr & 7) + k, k < 2, summed over the wave's WTN columns
        static_assert(TN == 2 && WTN == 64, "heads epilogue: a wave tile 64 columns wide");
        const float *hw = t == 0 ? hd.w0 : hd.w1;
        const int nh = t == 0 ? hd.na : 1;
        float wv[4][TN], bv[TN];
#pragma unroll
        for (int j = 0; j < TN; j++) {
            const int col = n0 + wn * WTN + j * 32 + fr;
            bv[j] = bias[(int64_t)t * N + col];
#pragma unroll
            for (int o = 0; o < 4; o++) {  // loaded unconditionally (row clamped into [0, nh)): no load behind a branch
                const float x = hw[(int64_t)(o < nh ? o : 0) * N + col];
                wv[o][j] = o < nh ? x : 0.0f;
            }
        }
        float *part = hd.part + ((int64_t)(t * tiles_n + tn) * WGN + wn) * M * 4;
#pragma unroll
        for (int i = 0; i < TM; i++) {
            float pv[64];  // [o][r]
#pragma unroll
            for (int q = 0; q < 64; q++) pv[q] = 0.0f;
#pragma unroll
            for (int j = 0; j < TN; j++) {
                const int col = n0 + wn * WTN + j * 32 + fr;
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const int64_t row = m0 + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
                    const float v = relu_nan((hi[i][j][r] + lo[i][j][r] * LO_INV) * inv * invB + bv[j]);
                    if (EPI == 2 && row < M) Ct[row * N + col] = v;
#pragma unroll
                    for (int o = 0; o < 4; o++) pv[o * 16 + r] += v * wv[o][j];
                }
            }
#pragma unroll
            for (int c = 64, off = 16; off >= 1; c >>= 1, off >>= 1) {
                const bool up = (fr & off) != 0;
#pragma unroll
                for (int k = 0; k < c / 2; k++) {
                    const float send = up ? pv[k] : pv[k + c / 2], keep = up ? pv[k + c / 2] : pv[k];
                    pv[k] = keep + __shfl_xor(send, off);
                }
            }
            const int o = fr >> 3;
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const int r = 2 * (fr & 7) + k;
                const int64_t row = m0 + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
                if (row < M) part[row * 4 + o] = pv[k];
            }
        }
        return;
    }
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
                    const float v = (hi[i][j][r] + lo[i][j][r] * LO_INV) * inv * invB;
                    Ct[row * N + col] = EPI == 1 ? relu_nan(v + bv) : v;
                }
            }
        }
    }
}

template <int BM, int BN, int WGM, int WGN, int EPI>
__global__ __launch_bounds__(64 * WGM * WGN) void k_h3_ntp(const float *__restrict__ A, const u32x4 *__restrict__ B,
                                                           const uint32_t *__restrict__ amaxA,
                                                           const uint32_t *__restrict__ amaxB, int64_t M, int N,
                                                           int K, int64_t sA, int64_t sB,
                                                           const float *__restrict__ bias, float *__restrict__ C,
                                                           int64_t sC, int tiles_n, u32x4 *__restrict__ Pout,
                                                           HeadsArg hd) {
    h3_ntp_body<BM, BN, WGM, WGN, EPI, false>(A, B, amaxA, amaxB, M, N, K, sA, sB, bias, C, sC, tiles_n, Pout, nullptr,
                                              hd);
}
template <int BM, int BN, int WGM, int WGN, int EPI, bool AP = false>
__global__ __launch_bounds__(64 * WGM * WGN) void k_h3_ntpg(const float *__restrict__ A, const u32x4 *__restrict__ B,
                                                            const uint32_t *__restrict__ amaxA,
                                                            const uint32_t *__restrict__ amaxB, int64_t M, int N,
                                                            int K, int64_t sA, int64_t sB,
                                                            const float *__restrict__ bias, float *__restrict__ C,
                                                            int64_t sC, int tiles_n, const int32_t *__restrict__ amap,
                                                            HeadsArg hd) {
    h3_ntp_body<BM, BN, WGM, WGN, EPI, true, AP>(A, B, amaxA, amaxB, M, N, K, sA, sB, bias, C, sC, tiles_n, nullptr,
                                                 amap, hd);
}

// ---------------------------------------------------------------------------------------------------------------
// The NT product with both operands staged by LDS-DMA (global_load_lds_dwordx4) three k steps deep: k_h3_nt's one
// step of register prefetch left every k step waiting on the global loads issued one step before (PMC: a third of
// the wave cycles in s_waitcnt, LDS waits 4 %, MFMA busy 38 %).  Here a k step's A (fp32, 128 B per row) and B
// (planes, 128 B per row) go straight into LDS two steps ahead, with no staging registers and no ds_write pass;
// each wave splits its own A fragments after reading them (the A values a wave reads are split by the WGN waves of
// its row band).  LDS images: rows of 8 16-B chunks, chunk c of row r at c ^ ((r >> 1) & 7) -- a DMA writes 1 KB
// lane-linear, so the permutation is applied to the global source address; a fragment read (16 lanes of a
// ds_read_b128 group, 16 different rows, one chunk) then hits 16 distinct 16-B bank slots.  Raw s_barrier with
// counted vmcnt: the DMA of step kt + 2 stays in flight across the barrier that publishes step kt + 1.
__device__ __forceinline__ int g_swz(int r) { return (r >> 1) & 7; }

// AP: A arrives as plane images too ([M][K/8][2][8] f16, h3_split's layout: 4 B per value like fp32, so the DMA
// addressing is the same) -- no split at all, A's fragments read like B's.
// ABL (probe ablations, round 5): 1 = no DMA in the main loop (compute on whatever the stages hold), 2 = no MFMAs
// (fragment reads kept live), 3 = neither fragment reads nor MFMAs (the DMA stream alone)
// ORD (round 5): in the first half step the MFMAs are issued before the reads of the second half -- with the reads
// first, hipcc waits lgkmcnt(0) for them before the first MFMA (the MFMAs' operands come from the reads issued after
// the previous barrier, and it does not count the newer ones out), so every other half step's MFMAs waited for a
// full LDS read round trip (the .s of cfg 42)
template <int BM, int BN, int WGM, int WGN, int EPI, bool KP, bool AP = false, bool PR = false, int ABL = 0,
          bool ORD = false>
__global__ __launch_bounds__(64 * WGM * WGN) void k_h3_ntg(const float *__restrict__ A, const u32x4 *__restrict__ B,
                                                           const uint32_t *__restrict__ amaxA,
                                                           const uint32_t *__restrict__ amaxB, int64_t M, int N,
                                                           int K, int64_t sA, int64_t sB,
                                                           const float *__restrict__ bias, float *__restrict__ C,
                                                           int64_t sC, int tiles_n) {
    constexpr int NT = 64 * WGM * WGN;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int GA = BM * 8 / NT, GB = BN * 8 / NT;  // DMA instructions per thread and k step
    constexpr int G = GA + GB;
    constexpr int STG = (BM + BN) * 8;  // chunks per stage
    static_assert(WTM % 32 == 0 && WTN % 32 == 0, "wave tile of 32 x 32 MFMA tiles");
    static_assert((BM * 8) % NT == 0 && (BN * 8) % NT == 0, "whole DMA instructions per thread");
    __shared__ u32x4 lds[3 * STG];

    const int t = blockIdx.y;
    const int L = xcd_tile(blockIdx.x, gridDim.x);
    const int tm = L / tiles_n, tn = L - tm * tiles_n;
    const int64_t m0 = (int64_t)tm * BM;
    const int n0 = tn * BN;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WGN, wn = w - (w / WGN) * WGN;
    const int64_t rowB = (int64_t)(K / 8) * 2;  // chunks per B row

    // DMA sources: the chunk lane q of instruction i lands on is LDS chunk i NT + q (row q >> 3 of the image)
    const float *srcA[GA];
    const u32x4 *srcB[GB];
#pragma unroll
    for (int i = 0; i < GA; i++) {
        const int q = i * NT + tid, r = q >> 3, c = (q & 7) ^ g_swz(r);
        srcA[i] = A + t * sA + std::min<int64_t>(m0 + r, M - 1) * K + c * 4;
    }
#pragma unroll
    for (int i = 0; i < GB; i++) {
        const int q = i * NT + tid, r = q >> 3, c = (q & 7) ^ g_swz(r);
        srcB[i] = B + t * sB + (int64_t)(n0 + r) * rowB + c;
    }
    // the scales first: an ordinary load consumed after a DMA is issued makes the compiler wait for the DMA too
    const int eA = h3_exp(load_amax(amaxA + t)), eB = h3_exp(load_amax(amaxB + t));
    const float scA = pow2f(eA), scA2 = pow2f(eA + 11);
    typedef __attribute__((address_space(3))) void lds_void;
    typedef __attribute__((address_space(1))) void gbl_void;
    auto issue = [&](int kt, int st) {
        if constexpr (ABL == 1) {
            if (kt >= 2) return;
        }
        u32x4 *base = lds + st * STG + w * 64;
#pragma unroll
        for (int i = 0; i < GA; i++)
            __builtin_amdgcn_global_load_lds((gbl_void *)(srcA[i] + kt * 32), (lds_void *)(base + i * NT), 16, 0, 0);
#pragma unroll
        for (int i = 0; i < GB; i++)
            __builtin_amdgcn_global_load_lds((gbl_void *)(srcB[i] + kt * 8), (lds_void *)(base + BM * 8 + i * NT),
                                             16, 0, 0);
    };

    f32x16 hi[TM][TN], lo[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++) {
            hi[i][j] = f32x16{};
            lo[i][j] = f32x16{};
        }
    const int fr = lane & 31, fh = lane >> 5;

    const int nk = K / BK;
    issue(0, 0);
    if (nk > 1) {
        issue(1, 1);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    // a 16-deep half step's fragments: A as fp32 (two chunks per 32-row tile, split after the read), B as planes
    struct Frag {
        u32x4 a[TM][2], b[TN][2];
    };
    auto read = [&](int st, int kh, Frag &f) {
        if constexpr (ABL == 3) return;
        const u32x4 *sAl = lds + st * STG, *sBl = sAl + BM * 8;
#pragma unroll
        for (int j = 0; j < TN; j++) {
            const int r = wn * WTN + j * 32 + fr, g = 2 * kh + fh;
#pragma unroll
            for (int p = 0; p < 2; p++) f.b[j][p] = sBl[r * 8 + ((2 * g + p) ^ g_swz(r))];
        }
#pragma unroll
        for (int i = 0; i < TM; i++) {
            const int r = wm * WTM + i * 32 + fr, c = 4 * kh + 2 * fh;
            f.a[i][0] = sAl[r * 8 + (c ^ g_swz(r))];
            f.a[i][1] = sAl[r * 8 + ((c + 1) ^ g_swz(r))];
        }
    };  // AP: chunk c = 2 g + p is plane p of k chunk g -- the same reads give (h, l)
    // A's fragments split into planes (in place: a[i][0] = hi plane, a[i][1] = lo plane), then the MFMAs
    auto split = [&](Frag &f) {
        if constexpr (AP) return;
#pragma unroll
        for (int i = 0; i < TM; i++) {
            u32x4 ah, al;
            h3_split8(__builtin_bit_cast(float4, f.a[i][0]), __builtin_bit_cast(float4, f.a[i][1]), scA, scA2, ah, al);
            f.a[i][0] = ah;
            f.a[i][1] = al;
        }
    };
    auto mfmas = [&](const Frag &f) {
        if constexpr (ABL >= 2) {
#pragma unroll
            for (int i = 0; i < TM; i++) asm volatile("" ::"v"(f.a[i][0]), "v"(f.a[i][1]));
#pragma unroll
            for (int j = 0; j < TN; j++) asm volatile("" ::"v"(f.b[j][0]), "v"(f.b[j][1]));
            return;
        }
        if constexpr (PR) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < TM; i++)
#pragma unroll
            for (int j = 0; j < TN; j++) {
                lo[i][j] = mfma16(f.a[i][1], f.b[j][0], lo[i][j]);
                lo[i][j] = mfma16(f.a[i][0], f.b[j][1], lo[i][j]);
                hi[i][j] = mfma16(f.a[i][0], f.b[j][0], hi[i][j]);
            }
        if constexpr (PR) __builtin_amdgcn_s_setprio(0);
    };
    auto mma = [&](Frag &f) {
        split(f);
        mfmas(f);
    };
    auto touch = [&](const Frag &f) {
#pragma unroll
        for (int i = 0; i < TM; i++) asm volatile("" ::"v"(f.a[i][0]), "v"(f.a[i][1]));
#pragma unroll
        for (int j = 0; j < TN; j++) asm volatile("" ::"v"(f.b[j][0]), "v"(f.b[j][1]));
    };
    int st = 0;
    if constexpr (KP) {
        // each half step's MFMAs run while the next half step's fragments are read: split kh 0, [read kh 1 | MFMA
        // kh 0], barrier (publishes step kt + 1), split kh 1, [read kh 0 of step kt + 1 | MFMA kh 1].  The split
        // goes before the reads so its wait covers only its own fragments; the last two steps are peeled, so the
        // loop has no conditional part (a join makes the compiler wait for every read in flight); scheduling
        // barriers keep the reads ahead of the MFMAs they are to run under and the barrier behind them.
        auto next = [](int s) { return s == 2 ? 0 : s + 1; };
        Frag f0, f1;
        read(0, 0, f0);
        int kt = 0;
        for (; kt + 2 < nk; kt++) {
            const int sn = next(st);
            issue(kt + 2, next(sn));  // the stage read in step kt - 1
            split(f0);
            if constexpr (ORD) {
                mfmas(f0);
                __builtin_amdgcn_sched_barrier(0);
                read(st, 1, f1);
            } else {
                read(st, 1, f1);
                __builtin_amdgcn_sched_barrier(0);
                mfmas(f0);
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (ORD) {
                // the compiler's own wait for f1 here (a use of its registers), so it does not add one after the
                // barrier, where it would also cover the reads of the next half
                touch(f1);
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(G) : "memory");
            }
            __builtin_amdgcn_s_barrier();
            split(f1);
            read(sn, 0, f0);
            __builtin_amdgcn_sched_barrier(0);
            mfmas(f1);
            __builtin_amdgcn_sched_barrier(0);
            st = sn;
        }
        if (kt + 1 < nk) {  // step nk - 2: no DMA left to issue
            const int sn = next(st);
            split(f0);
            if constexpr (ORD) {
                mfmas(f0);
                __builtin_amdgcn_sched_barrier(0);
                read(st, 1, f1);
            } else {
                read(st, 1, f1);
                __builtin_amdgcn_sched_barrier(0);
                mfmas(f0);
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (ORD) touch(f1);
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            split(f1);
            read(sn, 0, f0);
            __builtin_amdgcn_sched_barrier(0);
            mfmas(f1);
            st = sn;
        }
        split(f0);  // step nk - 1
        read(st, 1, f1);
        __builtin_amdgcn_sched_barrier(0);
        mfmas(f0);
        mma(f1);
    } else {
        for (int kt = 0; kt < nk; kt++) {
            if (kt + 2 < nk) issue(kt + 2, st == 0 ? 2 : st - 1);  // the stage read in step kt - 1
#pragma unroll
            for (int kh = 0; kh < 2; kh++) {
                Frag f;
                read(st, kh, f);
                mma(f);
            }
            // publish step kt + 1 (this wave's DMA of it done; step kt + 2's may stay in flight), and every wave is
            // past its reads of stage st before step kt + 3's DMA overwrites it
            if (kt + 2 < nk)
                asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(G) : "memory");
            else
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            st = st == 2 ? 0 : st + 1;
        }
    }

    const float inv = pow2f(-eA), invB = pow2f(-eB);
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
                    const float v = (hi[i][j][r] + lo[i][j][r] * LO_INV) * inv * invB;
                    Ct[row * N + col] = EPI == 1 ? relu_nan(v + bv) : v;
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------------------------
// TN: slab[s][t][m][n] = sum_{k in split s} A[t][k][m] B[t][k][n], A fp32 [Kd][M], B fp32 [Kd][N] (the weight
// gradient dz^T a3: both operands row-major over the minibatch's frames), both split while staged into plane
// images [32 k rows][RC chunks of 8 columns]; fragments k-contiguous through ds_read_b64_tr_b16 (a 32x32x16
// fragment, lane l: column l & 31, k = 8 (l >> 5) + j, is two transposed reads: 16-lane group g takes columns
// 16 (g & 1) .. + 15 and k rows 8 (g >> 1) + 4 h2 .. + 3).  Chunk c of row r sits at r RC + (c ^ swz(r)): the 16
// chunks a 32-lane half reads (4 rows x 4 adjacent chunks) land on 16 distinct 16-B bank slots for RC = 16 (XOR
// 4 (r & 3)) and RC = 24 (XOR 4 ((r >> 1) & 1)).  Slabs are written already unscaled (x 2^-(eA + eB), exact).
template <int RC>
__device__ __forceinline__ int tr_swz(int row) {
    // RC = 8 (128-B rows) as RC = 24: two rows per 256-B bank row, rows r and r + 2 on the same slots
    static_assert(RC % 16 == 0 || RC == 24 || RC == 8, "row chunks");
    return RC % 16 == 0 ? (row & 3) << 2 : ((row >> 1) & 1) << 2;
}

template <int RC>
__device__ __forceinline__ u32x4 tr_frag(const u32x4 *img, int col0, int kh, int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int chunk = ((col0 + 16 * (g & 1)) >> 3) + (p >> 1);
    bf16x4 v[2];  // 16-bit lanes moved as bits (the planes are f16)
#pragma unroll
    for (int h2 = 0; h2 < 2; h2++) {
        const int row = 16 * kh + 8 * (g >> 1) + 4 * h2 + q;
        const int off = (row * RC + (chunk ^ tr_swz<RC>(row))) * 16 + (p & 1) * 8;
        v[h2] = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4 *)((lds_char *)img + off));
    }
    return __builtin_bit_cast(u32x4, bf16x8{v[0][0], v[0][1], v[0][2], v[0][3], v[1][0], v[1][1], v[1][2], v[1][3]});
}

// GB: B's rows gathered by 64-column chunks -- row k's chunk j is row bmap[k * N / 64 + j] of B seen as [*][64] (the
// minibatch's conv3 rows through their patch representatives, as k_h3_ntp's GA).  A unit's chunk is fixed, its row
// changes every k step: each load issues the next step's chunk-row reads behind its data reads (ready by then).
// AQ: A arrives as plane images ([Kd][M/8][2][8] f16, 4 B per value like fp32, so the addressing is the same): its
// staging copies the hi / lo chunks instead of splitting (k_head_bwd's dz planes, merlin_tower_head_bwd_planes)
// BQ: B (gathered) arrives as plane images too (conv3's representatives as planes)
template <int BM, int BN, int WGM, int WGN, bool GB, bool AQ = false, bool BQ = false>
__device__ __forceinline__ void h3_tn_body(const float4 *__restrict__ A, const float4 *__restrict__ B,
                                           const uint32_t *__restrict__ amaxA, const uint32_t *__restrict__ amaxB,
                                           int64_t Kd, int M, int N, int64_t sA, int64_t sB, int64_t kc, int tiles_n,
                                           int tiles, int S, float *__restrict__ slab,
                                           const int32_t *__restrict__ bmap) {
    constexpr int NT = 64 * WGM * WGN;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int RCA = BM / 8, RCB = BN / 8;
    constexpr int QA = BK * RCA, QB = BK * RCB;  // units (k row, group of 8 columns) per k step
    constexpr int UA = (QA + NT - 1) / NT, UB = (QB + NT - 1) / NT;
    static_assert(WTM % 32 == 0 && WTN % 32 == 0, "wave tile of 32 x 32 MFMA tiles");
    constexpr int PSA = BK * RCA, PSB = BK * RCB;
    constexpr int STAGE = 2 * (PSA + PSB);
    __shared__ u32x4 lds[2 * STAGE];

    // 1-D grid over (tower, split, tile), tile fastest, XCD-contiguous: the tiles of one split read the same k rows
    const int P = xcd_tile(blockIdx.x, gridDim.x);
    const int t = P / (S * tiles), s = (P / tiles) % S, Lt = P % tiles;
    const int tm = Lt / tiles_n, tn = Lt - tm * tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int64_t k0 = (int64_t)s * kc, k1 = std::min<int64_t>(Kd, k0 + kc);
    const int eA = h3_exp(load_amax(amaxA + t)), eB = h3_exp(load_amax(amaxB + t));
    const float scA = pow2f(eA), scB = pow2f(eB), scA2 = pow2f(eA + 11), scB2 = pow2f(eB + 11);
    const int64_t rowA = M / 4, rowB = N / 4;
    A += t * sA + m0 / 4;
    B += t * sB + (GB ? 0 : n0 / 4);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WGN, wn = w - (w / WGN) * WGN;

    int ka[UA], la[UA], kb[UB], lb[UB];
    const float4 *pa[UA], *pb[UB];
    constexpr bool PAIR = GB && 8 % UB == 0 && RCB % UB == 0;
    const int32_t *mb[UB];  // GB: the unit's chunk column of bmap (stride N / 64 per k row)
    int32_t xb[UB];         // GB: the chunk rows of the next load
    const int nc = N / 64;
#pragma unroll
    for (int i = 0; i < UA; i++) {
        const int q = std::min(tid + i * NT, QA - 1);
        const int k = q / RCA, g = q - (q / RCA) * RCA;
        ka[i] = k;
        la[i] = k * RCA + (g ^ tr_swz<RCA>(k));
        pa[i] = A + (k0 + k) * rowA + g * 2;
    }
#pragma unroll
    for (int i = 0; i < UB; i++) {
        // GB with PAIR: a thread's UB units are adjacent column groups of one row and one 64-column chunk, so they
        // share one chunk row (one index read per thread and step)
        const int q = std::min(PAIR ? UB * tid + i : tid + i * NT, QB - 1);
        const int k = q / RCB, g = q - (q / RCB) * RCB;
        kb[i] = k;
        lb[i] = 2 * PSA + k * RCB + (g ^ tr_swz<RCB>(k));
        if constexpr (GB) {
            const int col = n0 + 8 * g;
            pb[i] = B + (col & 63) / 4;
            mb[i] = bmap + (k0 + k) * nc + (col >> 6);
        } else {
            pb[i] = B + (k0 + k) * rowB + g * 2;
        }
    }
    auto fetch_rows = [&](int64_t kk) {  // GB: chunk rows of step kk (rows past k1 clamped, zeroed when staged)
        if constexpr (GB) {
            constexpr int NX = PAIR ? 1 : UB;
            if (kk + BK <= k1) {  // full step: a wave-uniform offset
                const int64_t dm = (kk - k0) * nc;
#pragma unroll
                for (int i = 0; i < NX; i++) xb[i] = mb[i][dm];
            } else {
#pragma unroll
                for (int i = 0; i < NX; i++) xb[i] = mb[i][(std::min(kk + kb[i], k1 - 1) - k0 - kb[i]) * nc];
            }
#pragma unroll
            for (int i = NX; i < UB; i++) xb[i] = xb[0];
        }
    };
    const float4 zero = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    float4 ra[UA][2], rb[UB][2];
    auto load = [&](int64_t kk) {
        if constexpr (GB) {
            if (kk + BK <= k1) {
                const int64_t da = (kk - k0) * rowA;
#pragma unroll
                for (int i = 0; i < UA; i++) {
                    ra[i][0] = pa[i][da];
                    ra[i][1] = pa[i][da + 1];
                }
            } else {
#pragma unroll
                for (int i = 0; i < UA; i++) {
                    const float4 *src = pa[i] + (std::min(kk + ka[i], k1 - 1) - k0 - ka[i]) * rowA;
                    ra[i][0] = src[0];
                    ra[i][1] = src[1];
                }
            }
#pragma unroll
            for (int i = 0; i < UB; i++) {
                const float4 *src = pb[i] + (int64_t)xb[i] * 16;
                rb[i][0] = src[0];
                rb[i][1] = src[1];
            }
            fetch_rows(kk + BK);
            return;
        }
        if (kk + BK <= k1) {  // full step: row pointers + a wave-uniform offset
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
        for (int i = 0; i < UA; i++) {  // a split's last step: rows past k1 re-read row k1 - 1, zeroed when staged
            const float4 *src = pa[i] + (std::min(kk + ka[i], k1 - 1) - k0 - ka[i]) * rowA;
            ra[i][0] = src[0];
            ra[i][1] = src[1];
        }
#pragma unroll
        for (int i = 0; i < UB; i++) {
            const float4 *src = pb[i] + (std::min(kk + kb[i], k1 - 1) - k0 - kb[i]) * rowB;
            rb[i][0] = src[0];
            rb[i][1] = src[1];
        }
    };
    auto store = [&](int buf, int64_t kk) {
        u32x4 *st = lds + buf * STAGE;
#pragma unroll
        for (int i = 0; i < UA; i++)
            if (QA % NT == 0 || i + 1 < UA || tid + i * NT < QA) {
                const bool in = kk + ka[i] < k1;
                u32x4 p0, p1;
                if constexpr (AQ) {
                    p0 = __builtin_bit_cast(u32x4, in ? ra[i][0] : zero);
                    p1 = __builtin_bit_cast(u32x4, in ? ra[i][1] : zero);
                } else {
                    h3_split8(in ? ra[i][0] : zero, in ? ra[i][1] : zero, scA, scA2, p0, p1);
                }
                st[la[i]] = p0;
                st[PSA + la[i]] = p1;
            }
#pragma unroll
        for (int i = 0; i < UB; i++)
            if (PAIR ? UB * tid + i < QB : (QB % NT == 0 || i + 1 < UB || tid + i * NT < QB)) {
                const bool in = kk + kb[i] < k1;
                u32x4 p0, p1;
                if constexpr (BQ) {
                    p0 = __builtin_bit_cast(u32x4, in ? rb[i][0] : zero);
                    p1 = __builtin_bit_cast(u32x4, in ? rb[i][1] : zero);
                } else {
                    h3_split8(in ? rb[i][0] : zero, in ? rb[i][1] : zero, scB, scB2, p0, p1);
                }
                st[lb[i]] = p0;
                st[PSB + lb[i]] = p1;
            }
    };

    f32x16 hi[TM][TN], lo[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++) {
            hi[i][j] = f32x16{};
            lo[i][j] = f32x16{};
        }

    if (k0 < k1) {
        fetch_rows(k0);
        load(k0);
        store(0, k0);
        if (k0 + BK < k1) load(k0 + BK);
        __syncthreads();
    }
    int buf = 0;
    for (int64_t kk = k0; kk < k1; kk += BK, buf ^= 1) {
        if (kk + BK < k1) store(buf ^ 1, kk + BK);
        if (kk + 2 * BK < k1) load(kk + 2 * BK);
        const u32x4 *sAl = lds + buf * STAGE, *sBl = sAl + 2 * PSA;
        u32x4 af[TM][2][2];
#pragma unroll
        for (int i = 0; i < TM; i++)
#pragma unroll
            for (int kh = 0; kh < 2; kh++)
#pragma unroll
                for (int p = 0; p < 2; p++) af[i][kh][p] = tr_frag<RCA>(sAl + p * PSA, wm * WTM + i * 32, kh, lane);
#pragma unroll
        for (int j = 0; j < TN; j++) {
            u32x4 bf[2][2];
#pragma unroll
            for (int kh = 0; kh < 2; kh++)
#pragma unroll
                for (int p = 0; p < 2; p++) bf[kh][p] = tr_frag<RCB>(sBl + p * PSB, wn * WTN + j * 32, kh, lane);
#pragma unroll
            for (int i = 0; i < TM; i++) {
                f32x16 l = lo[i][j], h = hi[i][j];
#pragma unroll
                for (int kh = 0; kh < 2; kh++) {
                    l = mfma16(af[i][kh][1], bf[kh][0], l);
                    l = mfma16(af[i][kh][0], bf[kh][1], l);
                    h = mfma16(af[i][kh][0], bf[kh][0], h);
                }
                lo[i][j] = l;
                hi[i][j] = h;
            }
        }
        __syncthreads();
    }

    const float inv = pow2f(-eA), invB = pow2f(-eB);
    float *St = slab + ((int64_t)s * (gridDim.x / (S * tiles)) + t) * (int64_t)M * N;
    const int fr = lane & 31, fh = lane >> 5;
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int row = m0 + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
                St[(int64_t)row * N + n0 + wn * WTN + j * 32 + fr] =
                    (hi[i][j][r] + lo[i][j][r] * LO_INV) * inv * invB;
            }
}

template <int BM, int BN, int WGM, int WGN>
__global__ __launch_bounds__(64 * WGM * WGN) void k_h3_tn(const float4 *__restrict__ A, const float4 *__restrict__ B,
                                                          const uint32_t *__restrict__ amaxA,
                                                          const uint32_t *__restrict__ amaxB, int64_t Kd, int M, int N,
                                                          int64_t sA, int64_t sB, int64_t kc, int tiles_n, int tiles,
                                                          int S, float *__restrict__ slab) {
    h3_tn_body<BM, BN, WGM, WGN, false>(A, B, amaxA, amaxB, Kd, M, N, sA, sB, kc, tiles_n, tiles, S, slab, nullptr);
}
template <int BM, int BN, int WGM, int WGN, bool AQ = false, bool BQ = false>
__global__ __launch_bounds__(64 * WGM * WGN) void k_h3_tng(const float4 *__restrict__ A, const float4 *__restrict__ B,
                                                           const uint32_t *__restrict__ amaxA,
                                                           const uint32_t *__restrict__ amaxB, int64_t Kd, int M,
                                                           int N, int64_t sA, int64_t sB, int64_t kc, int tiles_n,
                                                           int tiles, int S, float *__restrict__ slab,
                                                           const int32_t *__restrict__ bmap) {
    h3_tn_body<BM, BN, WGM, WGN, true, AQ, BQ>(A, B, amaxA, amaxB, Kd, M, N, sA, sB, kc, tiles_n, tiles, S, slab,
                                               bmap);
}

// The TN product with the k step's split and staging interleaved into its MFMAs, as k_h3_ntp does for NT: the
// steps whose loads are whole (all but a split's last one or two) run in a loop with no conditional part, each
// reading its fragments first, then sched_group_barrier hints lay the next step's split (VALU), its LDS stores and
// the global loads of the step after it between the MFMAs; the remaining steps run as in k_h3_tn.  Same
// instructions per output as k_h3_tn, the same order of products and sums: the same bits.
template <int BM, int BN, int WGM, int WGN>
__global__ __launch_bounds__(64 * WGM * WGN) void k_h3_tnp(const float4 *__restrict__ A, const float4 *__restrict__ B,
                                                           const uint32_t *__restrict__ amaxA,
                                                           const uint32_t *__restrict__ amaxB, int64_t Kd, int M,
                                                           int N, int64_t sA, int64_t sB, int64_t kc, int tiles_n,
                                                           int tiles, int S, float *__restrict__ slab) {
    constexpr int NT = 64 * WGM * WGN;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int RCA = BM / 8, RCB = BN / 8;
    constexpr int QA = BK * RCA, QB = BK * RCB;
    constexpr int UA = (QA + NT - 1) / NT, UB = (QB + NT - 1) / NT;
    static_assert(WTM % 32 == 0 && WTN % 32 == 0, "wave tile of 32 x 32 MFMA tiles");
    constexpr int PSA = BK * RCA, PSB = BK * RCB;
    constexpr int STAGE = 2 * (PSA + PSB);
    constexpr int NMFMA = TM * TN * 6;
    __shared__ u32x4 lds[2 * STAGE];

    const int P = xcd_tile(blockIdx.x, gridDim.x);
    const int t = P / (S * tiles), s = (P / tiles) % S, Lt = P % tiles;
    const int tm = Lt / tiles_n, tn = Lt - tm * tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int64_t k0 = (int64_t)s * kc, k1 = std::min<int64_t>(Kd, k0 + kc);
    const int eA = h3_exp(load_amax(amaxA + t)), eB = h3_exp(load_amax(amaxB + t));
    const float scA = pow2f(eA), scB = pow2f(eB), scA2 = pow2f(eA + 11), scB2 = pow2f(eB + 11);
    const int64_t rowA = M / 4, rowB = N / 4;
    A += t * sA + m0 / 4;
    B += t * sB + n0 / 4;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WGN, wn = w - (w / WGN) * WGN;

    int ka[UA], la[UA], kb[UB], lb[UB];
    const float4 *pa[UA], *pb[UB];
#pragma unroll
    for (int i = 0; i < UA; i++) {
        const int q = std::min(tid + i * NT, QA - 1);
        const int k = q / RCA, g = q - (q / RCA) * RCA;
        ka[i] = k;
        la[i] = k * RCA + (g ^ tr_swz<RCA>(k));
        pa[i] = A + (k0 + k) * rowA + g * 2;
    }
#pragma unroll
    for (int i = 0; i < UB; i++) {
        const int q = std::min(tid + i * NT, QB - 1);
        const int k = q / RCB, g = q - (q / RCB) * RCB;
        kb[i] = k;
        lb[i] = 2 * PSA + k * RCB + (g ^ tr_swz<RCB>(k));
        pb[i] = B + (k0 + k) * rowB + g * 2;
    }
    const float4 zero = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    float4 ra[UA][2], rb[UB][2];
    auto load_full = [&](int64_t kk) {
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
    };
    auto load = [&](int64_t kk) {
        if (kk + BK <= k1) {
            load_full(kk);
            return;
        }
#pragma unroll
        for (int i = 0; i < UA; i++) {
            const float4 *src = pa[i] + (std::min(kk + ka[i], k1 - 1) - k0 - ka[i]) * rowA;
            ra[i][0] = src[0];
            ra[i][1] = src[1];
        }
#pragma unroll
        for (int i = 0; i < UB; i++) {
            const float4 *src = pb[i] + (std::min(kk + kb[i], k1 - 1) - k0 - kb[i]) * rowB;
            rb[i][0] = src[0];
            rb[i][1] = src[1];
        }
    };
    auto store = [&](int buf, int64_t kk) {
        u32x4 *st = lds + buf * STAGE;
#pragma unroll
        for (int i = 0; i < UA; i++)
            if (QA % NT == 0 || i + 1 < UA || tid + i * NT < QA) {
                const bool in = kk + ka[i] < k1;
                u32x4 p0, p1;
                h3_split8(in ? ra[i][0] : zero, in ? ra[i][1] : zero, scA, scA2, p0, p1);
                st[la[i]] = p0;
                st[PSA + la[i]] = p1;
            }
#pragma unroll
        for (int i = 0; i < UB; i++)
            if (QB % NT == 0 || i + 1 < UB || tid + i * NT < QB) {
                const bool in = kk + kb[i] < k1;
                u32x4 p0, p1;
                h3_split8(in ? rb[i][0] : zero, in ? rb[i][1] : zero, scB, scB2, p0, p1);
                st[lb[i]] = p0;
                st[PSB + lb[i]] = p1;
            }
    };

    f32x16 hi[TM][TN], lo[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++) {
            hi[i][j] = f32x16{};
            lo[i][j] = f32x16{};
        }
    auto compute = [&](int buf) {
        const u32x4 *sAl = lds + buf * STAGE, *sBl = sAl + 2 * PSA;
        u32x4 af[TM][2][2], bf[TN][2][2];
#pragma unroll
        for (int i = 0; i < TM; i++)
#pragma unroll
            for (int kh = 0; kh < 2; kh++)
#pragma unroll
                for (int p = 0; p < 2; p++) af[i][kh][p] = tr_frag<RCA>(sAl + p * PSA, wm * WTM + i * 32, kh, lane);
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int kh = 0; kh < 2; kh++)
#pragma unroll
                for (int p = 0; p < 2; p++) bf[j][kh][p] = tr_frag<RCB>(sBl + p * PSB, wn * WTN + j * 32, kh, lane);
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int i = 0; i < TM; i++) {
                f32x16 l = lo[i][j], h = hi[i][j];
#pragma unroll
                for (int kh = 0; kh < 2; kh++) {
                    l = mfma16(af[i][kh][1], bf[j][kh][0], l);
                    l = mfma16(af[i][kh][0], bf[j][kh][1], l);
                    h = mfma16(af[i][kh][0], bf[j][kh][0], h);
                }
                lo[i][j] = l;
                hi[i][j] = h;
            }
    };

    const int64_t nsteps = k0 < k1 ? (k1 - k0 + BK - 1) / BK : 0, nfull = k0 < k1 ? (k1 - k0) / BK : 0;
    if (nsteps > 0) {
        load(k0);
        store(0, k0);
        if (nsteps > 1) load(k0 + BK);
        __syncthreads();
    }
    int buf = 0;
    int64_t st = 0, kk = k0;
    for (; st + 2 < nfull; st++, kk += BK, buf ^= 1) {  // the load of step st + 2 is whole
        compute(buf);
        store(buf ^ 1, kk + BK);
        load_full(kk + 2 * BK);
        __builtin_amdgcn_sched_group_barrier(0x100, (TM + TN) * 8, 0);
#pragma unroll
        for (int m = 0; m < NMFMA; m++) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
            if (m % 3 == 2) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
            if (m >= NMFMA / 2 && m % 2 == 1) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
        __syncthreads();
    }
    for (; st < nsteps; st++, kk += BK, buf ^= 1) {
        if (st + 1 < nsteps) store(buf ^ 1, kk + BK);
        if (st + 2 < nsteps) load(kk + 2 * BK);
        compute(buf);
        __syncthreads();
    }

    const float inv = pow2f(-eA), invB = pow2f(-eB);
    float *Sl = slab + ((int64_t)s * (gridDim.x / (S * tiles)) + t) * (int64_t)M * N;
    const int fr = lane & 31, fh = lane >> 5;
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int row = m0 + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
                Sl[(int64_t)row * N + n0 + wn * WTN + j * 32 + fr] =
                    (hi[i][j][r] + lo[i][j][r] * LO_INV) * inv * invB;
            }
}

// TN over operands already in plane form ([T][Kd][cols/8][2][8] f16 -- the a_planes output of the NT kernels, so
// the fast step's weight gradient reads the planes its forward and input-gradient GEMMs made): k_h3_tn without the
// split, staging a copy of 16-B chunks.  Thread q of a k row takes plane q / RC, chunk q % RC: the 8 lanes of a
// ds_write_b128 group write 8 chunks of one plane image (8 distinct bank slots).
template <int BM, int BN, int WGM, int WGN>
__global__ __launch_bounds__(64 * WGM * WGN) void k_h3_tnq(const u32x4 *__restrict__ A, const u32x4 *__restrict__ B,
                                                           const uint32_t *__restrict__ amaxA,
                                                           const uint32_t *__restrict__ amaxB, int64_t Kd, int M,
                                                           int N, int64_t sA, int64_t sB, int64_t kc, int tiles_n,
                                                           int tiles, int S, float *__restrict__ slab) {
    constexpr int NT = 64 * WGM * WGN;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int RCA = BM / 8, RCB = BN / 8;
    constexpr int QA = BK * RCA * 2, QB = BK * RCB * 2;  // chunks per k step
    constexpr int UA = QA / NT, UB = QB / NT;
    static_assert(WTM % 32 == 0 && WTN % 32 == 0, "wave tile of 32 x 32 MFMA tiles");
    static_assert(QA % NT == 0 && QB % NT == 0 && RCA % 8 == 0 && RCB % 8 == 0, "whole staging chunks per thread");
    constexpr int PSA = BK * RCA, PSB = BK * RCB;
    constexpr int STAGE = 2 * (PSA + PSB);
    __shared__ u32x4 lds[2 * STAGE];

    const int P = xcd_tile(blockIdx.x, gridDim.x);
    const int t = P / (S * tiles), s = (P / tiles) % S, Lt = P % tiles;
    const int tm = Lt / tiles_n, tn = Lt - tm * tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int64_t k0 = (int64_t)s * kc, k1 = std::min<int64_t>(Kd, k0 + kc);
    const int eA = h3_exp(load_amax(amaxA + t)), eB = h3_exp(load_amax(amaxB + t));
    const int64_t rowA = M / 4, rowB = N / 4;  // chunks per k row
    A += t * sA + m0 / 4;
    B += t * sB + n0 / 4;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WGN, wn = w - (w / WGN) * WGN;

    int ka[UA], la[UA], kb[UB], lb[UB];
    const u32x4 *pa[UA], *pb[UB];
#pragma unroll
    for (int i = 0; i < UA; i++) {
        const int q = tid + i * NT;
        const int k = q / (2 * RCA), c = q - k * (2 * RCA), p = c / RCA, g = c - p * RCA;
        ka[i] = k;
        la[i] = p * PSA + k * RCA + (g ^ tr_swz<RCA>(k));
        pa[i] = A + (k0 + k) * rowA + g * 2 + p;
    }
#pragma unroll
    for (int i = 0; i < UB; i++) {
        const int q = tid + i * NT;
        const int k = q / (2 * RCB), c = q - k * (2 * RCB), p = c / RCB, g = c - p * RCB;
        kb[i] = k;
        lb[i] = 2 * PSA + p * PSB + k * RCB + (g ^ tr_swz<RCB>(k));
        pb[i] = B + (k0 + k) * rowB + g * 2 + p;
    }
    u32x4 ra[UA], rb[UB];
    auto load = [&](int64_t kk) {
        if (kk + BK <= k1) {
            const int64_t da = (kk - k0) * rowA, db = (kk - k0) * rowB;
#pragma unroll
            for (int i = 0; i < UA; i++) ra[i] = pa[i][da];
#pragma unroll
            for (int i = 0; i < UB; i++) rb[i] = pb[i][db];
            return;
        }
#pragma unroll
        for (int i = 0; i < UA; i++) ra[i] = pa[i][(std::min(kk + ka[i], k1 - 1) - k0 - ka[i]) * rowA];
#pragma unroll
        for (int i = 0; i < UB; i++) rb[i] = pb[i][(std::min(kk + kb[i], k1 - 1) - k0 - kb[i]) * rowB];
    };
    auto store = [&](int buf, int64_t kk) {
        u32x4 *st = lds + buf * STAGE;
        const u32x4 zero = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
        for (int i = 0; i < UA; i++) st[la[i]] = kk + ka[i] < k1 ? ra[i] : zero;
#pragma unroll
        for (int i = 0; i < UB; i++) st[lb[i]] = kk + kb[i] < k1 ? rb[i] : zero;
    };

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
        const u32x4 *sAl = lds + buf * STAGE, *sBl = sAl + 2 * PSA;
        u32x4 af[TM][2][2];
#pragma unroll
        for (int i = 0; i < TM; i++)
#pragma unroll
            for (int kh = 0; kh < 2; kh++)
#pragma unroll
                for (int p = 0; p < 2; p++) af[i][kh][p] = tr_frag<RCA>(sAl + p * PSA, wm * WTM + i * 32, kh, lane);
#pragma unroll
        for (int j = 0; j < TN; j++) {
            u32x4 bf[2][2];
#pragma unroll
            for (int kh = 0; kh < 2; kh++)
#pragma unroll
                for (int p = 0; p < 2; p++) bf[kh][p] = tr_frag<RCB>(sBl + p * PSB, wn * WTN + j * 32, kh, lane);
#pragma unroll
            for (int i = 0; i < TM; i++) {
                f32x16 l = lo[i][j], h = hi[i][j];
#pragma unroll
                for (int kh = 0; kh < 2; kh++) {
                    l = mfma16(af[i][kh][1], bf[kh][0], l);
                    l = mfma16(af[i][kh][0], bf[kh][1], l);
                    h = mfma16(af[i][kh][0], bf[kh][0], h);
                }
                lo[i][j] = l;
                hi[i][j] = h;
            }
        }
        __syncthreads();
    }

    const float inv = pow2f(-eA), invB = pow2f(-eB);
    float *St = slab + ((int64_t)s * (gridDim.x / (S * tiles)) + t) * (int64_t)M * N;
    const int fr = lane & 31, fh = lane >> 5;
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int row = m0 + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
                St[(int64_t)row * N + n0 + wn * WTN + j * 32 + fr] =
                    (hi[i][j][r] + lo[i][j][r] * LO_INV) * inv * invB;
            }
}

template <int BM, int BN, int WGM, int WGN, bool PIPE>
hipError_t nt_launch(const float *A, const u32x4 *B, const uint32_t *amaxA, const uint32_t *amaxB, int64_t M, int N,
                     int K, int T, int64_t sA, int64_t sB, const float *bias, float *C, int64_t sC, u32x4 *Pout,
                     const int32_t *amap, const HeadsArg &hd, hipStream_t s, bool ap = false) {
    if (N % BN || (PIPE && K < 2 * BK)) return hipErrorInvalidValue;
    if (ap) {  // A as planes: the gathered pipelined kernel (the update's forward), with or without the heads
        if constexpr (!PIPE || BN / WGN != 64) {
            return hipErrorInvalidValue;
        } else {
            if (!amap || !C || !bias || Pout || K % 64 || K > 64 * GA_CHUNKS) return hipErrorInvalidValue;
            const int64_t tiles_m = (M + BM - 1) / BM;
            const dim3 grid((unsigned)(tiles_m * (N / BN)), T), block(64 * WGM * WGN);
            if (hd.part) {
                if (T != 2 || hd.na < 1 || hd.na > 4 || !hd.w0 || !hd.w1) return hipErrorInvalidValue;
                hipLaunchKernelGGL((k_h3_ntpg<BM, BN, WGM, WGN, 2, true>), grid, block, 0, s, A, B, amaxA, amaxB, M, N,
                                   K, sA, sB, bias, C, sC, N / BN, amap, hd);
            } else {
                hipLaunchKernelGGL((k_h3_ntpg<BM, BN, WGM, WGN, 1, true>), grid, block, 0, s, A, B, amaxA, amaxB, M, N,
                                   K, sA, sB, bias, C, sC, N / BN, amap, hd);
            }
            return hipGetLastError();
        }
    }
    if ((int64_t)N * (K / 8) * 2 > INT32_MAX) return hipErrorInvalidValue;  // 32-bit B chunk offsets
    const int64_t tiles_m = (M + BM - 1) / BM;
    const int tiles_n = N / BN;
    if (tiles_m * tiles_n > INT32_MAX) return hipErrorInvalidValue;
    const dim3 grid((unsigned)(tiles_m * tiles_n), T), block(64 * WGM * WGN);
    if (hd.part) {  // heads in the epilogue: the pipelined kernel with bias + ReLU, both towers, 64-column wave tiles
        if constexpr (!PIPE || BN / WGN != 64) {
            return hipErrorInvalidValue;
        } else {
            if (!bias || T != 2 || Pout || hd.na < 1 || hd.na > 4 || !hd.w0 || !hd.w1) return hipErrorInvalidValue;
            if (amap) {
                if (K % 64 || K > 64 * GA_CHUNKS || !C) return hipErrorInvalidValue;
                hipLaunchKernelGGL((k_h3_ntpg<BM, BN, WGM, WGN, 2>), grid, block, 0, s, A, B, amaxA, amaxB, M, N, K,
                                   sA, sB, bias, C, sC, tiles_n, amap, hd);
            } else if (C) {
                hipLaunchKernelGGL((k_h3_ntp<BM, BN, WGM, WGN, 2>), grid, block, 0, s, A, B, amaxA, amaxB, M, N, K, sA,
                                   sB, bias, C, sC, tiles_n, nullptr, hd);
            } else {  // heads only
                hipLaunchKernelGGL((k_h3_ntp<BM, BN, WGM, WGN, 3>), grid, block, 0, s, A, B, amaxA, amaxB, M, N, K, sA,
                                   sB, bias, nullptr, sC, tiles_n, nullptr, hd);
            }
            return hipGetLastError();
        }
    }
    if (amap) {  // gathered A rows: the pipelined kernel only, no plane output
        if (!PIPE || Pout || K % 64 || K > 64 * GA_CHUNKS) return hipErrorInvalidValue;
        if (bias)
            hipLaunchKernelGGL((k_h3_ntpg<BM, BN, WGM, WGN, 1>), grid, block, 0, s, A, B, amaxA, amaxB, M, N, K, sA,
                               sB, bias, C, sC, tiles_n, amap, hd);
        else
            hipLaunchKernelGGL((k_h3_ntpg<BM, BN, WGM, WGN, 0>), grid, block, 0, s, A, B, amaxA, amaxB, M, N, K, sA,
                               sB, nullptr, C, sC, tiles_n, amap, hd);
        return hipGetLastError();
    }
    if (PIPE) {
        if (bias)
            hipLaunchKernelGGL((k_h3_ntp<BM, BN, WGM, WGN, 1>), grid, block, 0, s, A, B, amaxA, amaxB, M, N, K, sA, sB,
                               bias, C, sC, tiles_n, Pout, hd);
        else
            hipLaunchKernelGGL((k_h3_ntp<BM, BN, WGM, WGN, 0>), grid, block, 0, s, A, B, amaxA, amaxB, M, N, K, sA, sB,
                               nullptr, C, sC, tiles_n, Pout, hd);
    } else {
        if (bias)
            hipLaunchKernelGGL((k_h3_nt<BM, BN, WGM, WGN, 1>), grid, block, 0, s, A, B, amaxA, amaxB, M, N, K, sA, sB,
                               bias, C, sC, tiles_n, Pout);
        else
            hipLaunchKernelGGL((k_h3_nt<BM, BN, WGM, WGN, 0>), grid, block, 0, s, A, B, amaxA, amaxB, M, N, K, sA, sB,
                               nullptr, C, sC, tiles_n, Pout);
    }
    return hipGetLastError();
}

template <int BM, int BN, int WGM, int WGN, bool KP, bool AP = false, bool PR = false, int ABL = 0, bool ORD = false>
hipError_t ntg_launch(const float *A, const u32x4 *B, const uint32_t *amaxA, const uint32_t *amaxB, int64_t M, int N,
                      int K, int T, int64_t sA, int64_t sB, const float *bias, float *C, int64_t sC, u32x4 *Pout,
                      hipStream_t s) {
    if (N % BN || Pout) return hipErrorInvalidValue;  // no plane output from the DMA-staged kernel
    if ((int64_t)N * (K / 8) * 2 > INT32_MAX) return hipErrorInvalidValue;
    const int64_t tiles_m = (M + BM - 1) / BM;
    const int tiles_n = N / BN;
    if (tiles_m * tiles_n > INT32_MAX) return hipErrorInvalidValue;
    const dim3 grid((unsigned)(tiles_m * tiles_n), T), block(64 * WGM * WGN);
    if (bias)
        hipLaunchKernelGGL((k_h3_ntg<BM, BN, WGM, WGN, 1, KP, AP, PR, ABL, ORD>), grid, block, 0, s, A, B, amaxA, amaxB,
                           M, N, K, sA, sB, bias, C, sC, tiles_n);
    else
        hipLaunchKernelGGL((k_h3_ntg<BM, BN, WGM, WGN, 0, KP, AP, PR, ABL, ORD>), grid, block, 0, s, A, B, amaxA, amaxB,
                           M, N, K, sA, sB, nullptr, C, sC, tiles_n);
    return hipGetLastError();
}

// Q: the operands are plane images (k_h3_tnq), strides in values as for fp32 operands (4 B per value either way)
template <int BM, int BN, int WGM, int WGN, int Q>
hipError_t tn_launch(const void *A, const void *B, const uint32_t *amaxA, const uint32_t *amaxB, int64_t Kd, int M,
                     int N, int T, int64_t sA, int64_t sB, int splits, float *slab, int *S_out, const int32_t *bmap,
                     hipStream_t s) {
    if (M % BM || N % BN) return hipErrorInvalidValue;
    if (bmap && ((Q != 0 && Q != 3 && Q != 4) || N % 64)) return hipErrorInvalidValue;  // gathered B: k_h3_tng only
    if (Q >= 3 && !bmap) return hipErrorInvalidValue;
    const int tiles_n = N / BN, tiles = (M / BM) * tiles_n;
    int S = std::max(1, splits);
    int64_t kc = (Kd + S - 1) / S;
    kc = (kc + BK - 1) / BK * BK;
    S = (int)std::max<int64_t>(1, (Kd + kc - 1) / kc);
    *S_out = S;
    if (Q == 1)
        hipLaunchKernelGGL((k_h3_tnq<BM, BN, WGM, WGN>), dim3(tiles * S * T), dim3(64 * WGM * WGN), 0, s,
                           static_cast<const u32x4 *>(A), static_cast<const u32x4 *>(B), amaxA, amaxB, Kd, M, N,
                           sA / 4, sB / 4, kc, tiles_n, tiles, S, slab);
    else if (Q == 2)
        hipLaunchKernelGGL((k_h3_tnp<BM, BN, WGM, WGN>), dim3(tiles * S * T), dim3(64 * WGM * WGN), 0, s,
                           static_cast<const float4 *>(A), static_cast<const float4 *>(B), amaxA, amaxB, Kd, M, N,
                           sA / 4, sB / 4, kc, tiles_n, tiles, S, slab);
    else if (Q == 4)  // both as planes, B gathered
        hipLaunchKernelGGL((k_h3_tng<BM, BN, WGM, WGN, true, true>), dim3(tiles * S * T), dim3(64 * WGM * WGN), 0, s,
                           static_cast<const float4 *>(A), static_cast<const float4 *>(B), amaxA, amaxB, Kd, M, N,
                           sA / 4, sB / 4, kc, tiles_n, tiles, S, slab, bmap);
    else if (Q == 3)  // A as planes (AQ), B fp32 gathered
        hipLaunchKernelGGL((k_h3_tng<BM, BN, WGM, WGN, true>), dim3(tiles * S * T), dim3(64 * WGM * WGN), 0, s,
                           static_cast<const float4 *>(A), static_cast<const float4 *>(B), amaxA, amaxB, Kd, M, N,
                           sA / 4, sB / 4, kc, tiles_n, tiles, S, slab, bmap);
    else if (bmap)
        hipLaunchKernelGGL((k_h3_tng<BM, BN, WGM, WGN>), dim3(tiles * S * T), dim3(64 * WGM * WGN), 0, s,
                           static_cast<const float4 *>(A), static_cast<const float4 *>(B), amaxA, amaxB, Kd, M, N,
                           sA / 4, sB / 4, kc, tiles_n, tiles, S, slab, bmap);
    else
        hipLaunchKernelGGL((k_h3_tn<BM, BN, WGM, WGN>), dim3(tiles * S * T), dim3(64 * WGM * WGN), 0, s,
                           static_cast<const float4 *>(A), static_cast<const float4 *>(B), amaxA, amaxB, Kd, M, N,
                           sA / 4, sB / 4, kc, tiles_n, tiles, S, slab);
    return hipGetLastError();
}

__global__ void k_h3_fill0(float4 *__restrict__ out, int64_t n4) {
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n4; e += (int64_t)gridDim.x * 256)
        out[e] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}

}  // namespace

hipError_t launch_h3_amax(const float *x, int64_t n, int T, int64_t stride, uint32_t *amax, hipStream_t s) {
    // zeroed by a kernel, not hipMemsetAsync: this runs inside the fast step's captured forward graph, and a
    // captured memset node replays with a wrong fill value on ROCm 7 (scripts/probe_graph_then.py: 0x80808080)
    hipLaunchKernelGGL(k_h3_zero, dim3((T + 63) / 64), dim3(64), 0, s, amax, T);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || n <= 0) return e;
    if (n % 4 || stride % 4) return hipErrorInvalidValue;
    const int64_t n4 = n / 4;
    const int grid = (int)std::min<int64_t>((n4 + 255) / 256, 1024);
    hipLaunchKernelGGL(k_h3_amax, dim3(grid, T), dim3(256), 0, s, reinterpret_cast<const float4 *>(x), n4, stride / 4,
                       amax);
    return hipGetLastError();
}

hipError_t launch_h3_split(const float *x, int64_t n, int T, const uint32_t *amax, void *planes, hipStream_t s) {
    if (n % 8) return hipErrorInvalidValue;
    if (n <= 0) return hipSuccess;
    const int64_t g8 = n / 8;
    const int grid = (int)std::min<int64_t>((g8 + 255) / 256, 2048);
    hipLaunchKernelGGL(k_h3_split, dim3(grid, T), dim3(256), 0, s, reinterpret_cast<const float4 *>(x), g8, amax,
                       static_cast<u32x4 *>(planes));
    return hipGetLastError();
}

hipError_t launch_h3_gemm_nt(const float *A, const uint32_t *amaxA, const void *B, const uint32_t *amaxB, int64_t M,
                             int N, int K, int T, int64_t a_stride, int64_t b_stride, const float *bias, float *C,
                             int64_t c_stride, void *a_planes, int cfg, hipStream_t s, const int32_t *a_rows,
                             const float *head_w0, int n_actions, const float *head_w1, float *head_part,
                             bool a_is_planes) {
    const HeadsArg hd{head_w0, head_w1, n_actions, head_part};
    if (M <= 0) return hipSuccess;
    if (K % BK || N <= 0 || a_stride % 4 || b_stride % 8) return hipErrorInvalidValue;
    const u32x4 *b = static_cast<const u32x4 *>(B);
    u32x4 *P = static_cast<u32x4 *>(a_planes);
    const int64_t sB = b_stride / 8 * 2;  // chunks
#define H3_NT(BM, BN, WM, WN, PIPE) \
    nt_launch<BM, BN, WM, WN, PIPE>(A, b, amaxA, amaxB, M, N, K, T, a_stride, sB, bias, C, c_stride, P, a_rows, hd, s, \
                                    a_is_planes)
    if (a_is_planes && (cfg < 10 || cfg > 14) && cfg != 60) return hipErrorInvalidValue;
#ifdef MERLIN_PROBES
    constexpr int PLANE_CFG_END = 80;  // + the probe ablations 70..74
#else
    constexpr int PLANE_CFG_END = 70;
#endif
    if (cfg >= 60 && cfg < PLANE_CFG_END) {  // both operands as plane images (merlin_h3p.hip)
        if (P || ((a_rows || head_part) && !a_is_planes)) return hipErrorInvalidValue;
        return launch_h3p_gemm_nt(A, amaxA, B, amaxB, M, N, K, T, a_stride, b_stride, bias, C, c_stride, cfg, s, a_rows,
                                  head_w0, n_actions, head_w1, head_part);
    }
    switch (cfg) {
        case 0: return H3_NT(256, 128, 4, 2, false);
        case 1: return H3_NT(128, 192, 4, 2, false);
        case 2: return H3_NT(128, 128, 2, 2, false);
        case 3: return H3_NT(128, 256, 2, 4, false);
        case 5: return H3_NT(128, 64, 4, 1, false);  // N = 64 (the window GEMM's input gradient)
        // k_h3_ntp: the k step's split / staging interleaved into the MFMAs
        case 10: return H3_NT(256, 128, 4, 2, true);
        case 11: return H3_NT(128, 192, 4, 2, true);
        case 12: return H3_NT(128, 128, 2, 2, true);
        case 13: return H3_NT(128, 256, 2, 4, true);
        case 14: return H3_NT(64, 128, 2, 2, true);  // twice cfg 12's blocks (the rollout's 4096-row fc1)
#undef H3_NT
        // k_h3_ntg: both operands staged by LDS-DMA, three k steps deep
#define H3_NTG(BM, BN, WM, WN, KP) \
    ((a_rows || head_part) ? hipErrorInvalidValue                                                  \
            : ntg_launch<BM, BN, WM, WN, KP>(A, b, amaxA, amaxB, M, N, K, T, a_stride, sB, bias, C, c_stride, P, s))
        case 20: return H3_NTG(256, 128, 4, 2, false);
        case 21: return H3_NTG(128, 192, 4, 2, false);
        // the same with each half step's fragment reads under the previous half step's MFMAs
        case 30: return H3_NTG(256, 128, 4, 2, true);
        case 31: return H3_NTG(128, 192, 4, 2, true);
#undef H3_NTG
        // probe (round 5): A as plane images (h3_split of A with amaxA, passed as A), both operands by LDS-DMA
#define H3_NTGP(BM, BN, WM, WN, KP) \
    ((a_rows || head_part) ? hipErrorInvalidValue                                                  \
            : ntg_launch<BM, BN, WM, WN, KP, true>(A, b, amaxA, amaxB, M, N, K, T, a_stride, sB, bias, C, c_stride, P, s))
        case 40: return H3_NTGP(256, 128, 4, 2, true);
        case 41: return H3_NTGP(128, 192, 4, 2, true);
        case 42: return H3_NTGP(128, 256, 2, 4, true);
        case 43: return H3_NTGP(256, 128, 4, 2, false);
#undef H3_NTGP
#define H3_NTGQ(BM, BN, WM, WN, KP) \
    ((a_rows || head_part) ? hipErrorInvalidValue                                                  \
            : ntg_launch<BM, BN, WM, WN, KP, true, true>(A, b, amaxA, amaxB, M, N, K, T, a_stride, sB, bias, C, c_stride, P, s))
        case 44: return H3_NTGQ(128, 256, 2, 4, true);
        case 45: return H3_NTGQ(256, 128, 4, 2, true);
        case 46: return H3_NTGQ(256, 128, 4, 2, false);
#undef H3_NTGQ
#ifdef MERLIN_PROBES  // ablations (round 5): results are wrong on purpose (no DMA / no MFMA in the k loop)
#define H3_NTGA(BM, BN, WM, WN, ABL) \
    ((a_rows || head_part) ? hipErrorInvalidValue                                                  \
            : ntg_launch<BM, BN, WM, WN, true, true, false, ABL>(A, b, amaxA, amaxB, M, N, K, T, a_stride, sB, bias, C, c_stride, P, s))
        case 47: return H3_NTGA(128, 256, 2, 4, 1);
        case 48: return H3_NTGA(128, 256, 2, 4, 2);
        case 49: return H3_NTGA(128, 256, 2, 4, 3);
#undef H3_NTGA
#endif
#define H3_NTGO(BM, BN, WM, WN, AP, ABL) \
    ((a_rows || head_part) ? hipErrorInvalidValue                                                  \
            : ntg_launch<BM, BN, WM, WN, true, AP, false, ABL, true>(A, b, amaxA, amaxB, M, N, K, T, a_stride, sB, bias, C, c_stride, P, s))
        case 50: return H3_NTGO(128, 256, 2, 4, true, 0);
        case 51: return H3_NTGO(256, 128, 4, 2, true, 0);
        case 52: return H3_NTGO(128, 192, 4, 2, true, 0);
#ifdef MERLIN_PROBES
        case 53: return H3_NTGO(128, 256, 2, 4, true, 1);  // ablation: no DMA in the main loop
#endif
        case 54: return H3_NTGO(128, 256, 2, 4, false, 0);  // fp32 A split at the fragment reads
#undef H3_NTGO
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_h3_gemm_tn(const void *A, const uint32_t *amaxA, const void *B, const uint32_t *amaxB, int64_t Kd,
                             int M, int N, int T, int64_t a_stride, int64_t b_stride, int splits, float *slab,
                             float *out, bool planes, int cfg, hipStream_t s, const int32_t *b_rows, bool a_planes,
                             bool b_planes) {
    if (b_planes && !a_planes) return hipErrorInvalidValue;
    if (M <= 0 || N <= 0) return hipSuccess;
    if (M % 8 || N % 8 || a_stride % 4 || b_stride % 4) return hipErrorInvalidValue;
    const int64_t total = (int64_t)T * M * N;
    if (Kd <= 0) {  // a kernel, not a memset (capture-safe, see launch_h3_amax)
        hipLaunchKernelGGL(k_h3_fill0, dim3((unsigned)std::min<int64_t>((total / 4 + 255) / 256, 2048)), dim3(256),
                           0, s, reinterpret_cast<float4 *>(out), total / 4);
        return hipGetLastError();
    }
    int S = 1;
    hipError_t e;
    if (cfg == 20 || cfg == 21) {  // both operands as planes, B gathered, LDS-DMA staged (merlin_h3p.hip k_h3_tq)
        if (!(a_planes && b_planes)) return hipErrorInvalidValue;
        e = launch_h3p_gemm_tn_gather(A, amaxA, B, amaxB, Kd, M, N, T, a_stride, b_stride, splits, slab, b_rows, cfg,
                                      &S, s);
        if (e != hipSuccess) return e;
        return launch_x6_fold(slab, S, total, out, s);
    }
#define H3_TN(BM, BN, WM, WN, PIPE)                                                                              \
    (planes ? tn_launch<BM, BN, WM, WN, 1>(A, B, amaxA, amaxB, Kd, M, N, T, a_stride, b_stride, splits, slab, &S,   \
                                           b_rows, s)                                                              \
     : a_planes ? (b_planes ? tn_launch<BM, BN, WM, WN, 4>(A, B, amaxA, amaxB, Kd, M, N, T, a_stride, b_stride,    \
                                                           splits, slab, &S, b_rows, s)                            \
                           : tn_launch<BM, BN, WM, WN, 3>(A, B, amaxA, amaxB, Kd, M, N, T, a_stride, b_stride,    \
                                                          splits, slab, &S, b_rows, s))                            \
            : tn_launch<BM, BN, WM, WN, PIPE>(A, B, amaxA, amaxB, Kd, M, N, T, a_stride, b_stride, splits, slab, &S, \
                                              b_rows, s))
    switch (cfg) {
        case 0: e = H3_TN(128, 192, 4, 2, 0); break;
        case 1: e = H3_TN(128, 192, 2, 2, 0); break;
        case 2: e = H3_TN(64, 192, 2, 2, 0); break;  // M = 64 (the window GEMM's weight gradient)
        // k_h3_tnp: the split / staging interleaved into the MFMAs
        case 10: e = H3_TN(128, 192, 4, 2, 2); break;
        case 11: e = H3_TN(128, 192, 2, 2, 2); break;
        default: return hipErrorInvalidValue;
    }
#undef H3_TN
    if (e != hipSuccess) return e;
    return launch_x6_fold(slab, S, total, out, s);
}

namespace {
// logits[r][a] = sum over p < P of part[0][p][r][a] (a < na), value[r] = sum over p of part[1][p][r][0]: the heads'
// partials of the forward GEMM's epilogue (EPI 2) added in partial order (no biases: the loss adds them)
__global__ __launch_bounds__(256) void k_heads_combine(const float4 *__restrict__ part, int P, int64_t M, int na,
                                                       float *__restrict__ logits, float *__restrict__ value) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= M) return;
    float4 a = part[r], v = part[(int64_t)P * M + r];
    for (int p = 1; p < P; p++) {
        const float4 x = part[(int64_t)p * M + r], y = part[(int64_t)(P + p) * M + r];
        a.x += x.x;
        a.y += x.y;
        a.z += x.z;
        a.w += x.w;
        v.x += y.x;
    }
    const float av[4] = {a.x, a.y, a.z, a.w};
    for (int o = 0; o < na; o++) logits[r * na + o] = av[o];
    value[r] = v.x;
}
}  // namespace

// partials per row of the heads epilogue: tiles_n * WGN of the configuration (0 if it has none)
int h3_heads_parts(int N, int cfg) {
    switch (cfg) {
        case 10: return N % 128 ? 0 : N / 128 * 2;
        // cfg 11: 96-column wave tiles, no heads epilogue
        case 12: return N % 128 ? 0 : N / 128 * 2;
        case 13: return N % 256 ? 0 : N / 256 * 4;
        case 14: return N % 128 ? 0 : N / 128 * 2;
        case 60: return N % 256 ? 0 : N / 256 * 4;  // k_h3_pqg (planes, gathered rows): cfg 13's tiles
        default: return 0;
    }
}

hipError_t launch_heads_combine(const float *part, int P, int64_t M, int na, float *logits, float *value,
                                hipStream_t s) {
    if (M <= 0) return hipSuccess;
    if (P < 1 || na < 1 || na > 4) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_heads_combine, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<const float4 *>(part), P, M, na, logits, value);
    return hipGetLastError();
}

}  // namespace merlin
