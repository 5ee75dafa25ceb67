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

// C[t][m][n] = epi(sum_k A[t][m][k] B[t][n][k]); A fp32 [M][K], B x6 planes [N][K/8][3][8]
// (K % 32 == 0, N % BN == 0); EPI 1: relu(. + bias[t][n]).  grid (tiles_m * tiles_n, T).
template <int BM, int BN, int WGM, int WGN, int EPI, int ACC>
__global__ __launch_bounds__(64 * WGM * WGN) void k_x6_nt32(const float4 *__restrict__ A, const u32x4 *__restrict__ B,
                                                            int64_t M, int N, int K, int64_t sA, int64_t sB,
                                                            const float *__restrict__ bias, float *__restrict__ C,
                                                            int64_t sC, int tiles_n) {
    constexpr int NT = 64 * WGM * WGN;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int UA = (BM * 4 + NT - 1) / NT;
    constexpr int CB = (BN * CPR + NT - 1) / NT;
    static_assert(WTM % 32 == 0 && WTN % 32 == 0, "wave tile of 32 x 32 MFMA tiles");
    constexpr int PSA = BM * 4, PSB = BN * 4 + 12;
    constexpr int STAGE = 3 * (PSA + PSB);
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

template <int BM, int BN, int WGM, int WGN, int ACC>
hipError_t nt32_launch(const float4 *A, const u32x4 *B, int64_t M, int N, int K, int T, int64_t sA, int64_t sB,
                       const float *bias, float *C, int64_t sC, hipStream_t s) {
    if (N % BN) return hipErrorInvalidValue;
    const int64_t tiles_m = (M + BM - 1) / BM;
    const int tiles_n = N / BN;
    if (tiles_m * tiles_n > INT32_MAX) return hipErrorInvalidValue;
    const dim3 grid((unsigned)(tiles_m * tiles_n), T);
    if (bias)
        hipLaunchKernelGGL((k_x6_nt32<BM, BN, WGM, WGN, 1, ACC>), grid, dim3(64 * WGM * WGN), 0, s, A, B, M, N, K, sA,
                           sB, bias, C, sC, tiles_n);
    else
        hipLaunchKernelGGL((k_x6_nt32<BM, BN, WGM, WGN, 0, ACC>), grid, dim3(64 * WGM * WGN), 0, s, A, B, M, N, K, sA,
                           sB, nullptr, C, sC, tiles_n);
    return hipGetLastError();
}

}  // namespace

// cfg numbers continue merlin_gemm.hip's (launch_x6_gemm_nt forwards cfg >= 20 here)
hipError_t launch_x6_gemm_nt32(const float *A, const void *B, int64_t M, int N, int K, int T, int64_t a_stride,
                               int64_t b_stride, const float *bias, float *C, int64_t c_stride, int cfg,
                               hipStream_t s) {
    const float4 *a = reinterpret_cast<const float4 *>(A);
    const u32x4 *b = static_cast<const u32x4 *>(B);
    const int64_t sA = a_stride / 4, sB = b_stride / 8 * 3;
    switch (cfg) {
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
