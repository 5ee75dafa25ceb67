// merlin_h3p.hip -- fc1's NT GEMM with BOTH operands already in h3 plane form (round 5): no split in the kernel,
// both operands staged by LDS-DMA three k steps deep, the LDS fragment reads interleaved with the MFMAs.
//
// Why hand-placed waits (profiles/r05a_probe_h3_planes.log, the .s of k_h3_ntg): with the fragment reads as plain
// loads, hipcc waited lgkmcnt(0) before the first MFMA of every other half step -- the MFMAs' operands came from
// reads issued after the previous barrier, and the wait also covered the reads issued for the next half -- so the
// matrix pipe drained for an LDS round trip twice per k step.  Ablations of that kernel at the update's shape: 505
// us with everything, 400 us with no DMA in the loop, 384 us for the DMA stream alone.
//
// Here every half step is 3 TM TN MFMAs (TM x TN tiles of 32x32x16 x {hi, lo, lo}) with the 2 (TM + TN) fragment
// reads of the next half interleaved one per MFMA (sched_group_barrier), and the k loop is unrolled (one
// instantiation per K), so the compiler's lgkmcnt waits are exact counts: the reads of a half are waited for once,
// by the first MFMA that needs them (the MFMAs still in the pipe cover it).
//
// Layouts as merlin_h3.hip's k_h3_ntg: operand rows of K/8 groups x (hi, lo) x 8 f16 (h3_split), a k step (32
// values) = 8 16-B chunks per row; LDS image rows of 8 chunks, chunk c of row r at slot c ^ ((r >> 1) & 7), the
// permutation applied to the DMA's global source address (a DMA writes lane-linear).
#include <algorithm>
#include <type_traits>

#include "merlin_internal.h"

namespace merlin {
namespace {

typedef _Float16 p_f16x8 __attribute__((ext_vector_type(8)));
typedef float p_f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t p_u32x4 __attribute__((ext_vector_type(4)));

constexpr float P_LO_INV = 1.0f / 2048.0f;

__device__ __forceinline__ p_f32x16 p_mfma(const p_u32x4 a, const p_u32x4 b, p_f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(p_f16x8, a), __builtin_bit_cast(p_f16x8, b), c, 0,
                                                   0, 0);
}
__device__ __forceinline__ float p_relu(float v) { return v != v ? v : fmaxf(v, 0.0f); }
__device__ __forceinline__ int p_xcd_tile(int b, int nb) {
    const int xcd = b & 7, q = nb >> 3, r = nb & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}
__device__ __forceinline__ int p_exp(uint32_t amax) {  // merlin_h3.hip h3_exp
    if (amax == 0u) return 0;
    const int e = (int)((amax >> 23) & 0xffu) - 127;
    return std::min(std::max(14 - e, -120), 115);
}
__device__ __forceinline__ float p_pow2(int e) { return __uint_as_float((uint32_t)(e + 127) << 23); }
__device__ __forceinline__ uint32_t p_amax(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int p_swz(int r) { return (r >> 1) & 7; }
// a lo plane fragment (8 f16 at 2^11 x their value) back at scale: v_pk_mul_f16 x 4, exact unless the result is
// subnormal (then rounded to the f16 subnormal grid, 2^-24)
__device__ __forceinline__ p_u32x4 p_unscale(const p_u32x4 x) {
    return __builtin_bit_cast(p_u32x4, __builtin_bit_cast(p_f16x8, x) * (_Float16)(1.0f / 2048.0f));
}

template <int V>
using IC = std::integral_constant<int, V>;
template <int N, int I = 0, class F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (I < N) {
        f(IC<I>{});
        static_for<N, I + 1>(f);
    }
}

typedef __attribute__((address_space(3))) p_u32x4 lds_u32x4;
// one 16-B LDS fragment read (a plain load: the k loop is unrolled, so the compiler's waits are exact counts)
__device__ __forceinline__ void lds_rd(p_u32x4 &d, uint32_t addr) { d = *(const lds_u32x4 *)(uintptr_t)addr; }

// NS: LDS stages of the DMA ring (NS - 1 k steps in flight).  3: 120 KB at 128 x 192; 4 (round 6): 160 KB, the whole
// LDS of a CU -- a step's DMA is latency-bound (~2.5 us under load against ~1.2 us of MFMA work per step), so the
// feed rate per CU is the bytes in flight over that latency
// ONE (round 6): one accumulator per tile -- the lo planes (stored 2^11 up) brought back to scale in registers
// (v_pk_mul_f16 by 2^-11: exact while the result stays normal, f16 subnormals kept) so all three products of a k
// step add into the same fp32 accumulator: half the accumulator registers, hence twice the tile area per byte staged.
// Not the same bits as the two-accumulator kernels (a different summation); its error is held to float64 by
// tests/test_gpu_h3.py like theirs.
template <int BM, int BN, int WGM, int WGN, int EPI, int NK, int NS = 3, bool ONE = false, int ABL = 0, int ORD = 0>
__global__ __launch_bounds__(64 * WGM * WGN) void k_h3_pq(const p_u32x4 *__restrict__ A, const p_u32x4 *__restrict__ B,
                                                          const uint32_t *__restrict__ amaxA,
                                                          const uint32_t *__restrict__ amaxB, int64_t M, int N, int K,
                                                          int64_t sA, int64_t sB, const float *__restrict__ bias,
                                                          float *__restrict__ C, int64_t sC, int tiles_n) {
    constexpr int NT = 64 * WGM * WGN;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int NR = 2 * (TM + TN), NM = 3 * TM * TN;  // fragment reads / MFMAs per half step
    static_assert(NM >= NR, "a read behind every MFMA");
    constexpr int G = (BM + BN) * 8 / NT;  // DMA instructions per thread and k step
    static_assert((BM * 8) % NT == 0 && (BN * 8) % NT == 0, "whole DMA instructions per thread");
    constexpr int STG = (BM + BN) * 8;  // chunks per stage
    constexpr uint32_t STG_B = STG * 16;
    static_assert(NS >= 2 && NS <= 4, "ring depth");
    __shared__ p_u32x4 lds[NS * STG];

    const int t = blockIdx.y;
    const int L = p_xcd_tile(blockIdx.x, gridDim.x);
    const int tm = L / tiles_n, tn = L - tm * tiles_n;
    const int64_t m0 = (int64_t)tm * BM;
    const int n0 = tn * BN;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WGN, wn = w - (w / WGN) * WGN;
    const int64_t row_ch = K / 4;  // chunks per operand row (4 B per value, planes)

    // the scales first: an ordinary load consumed after a DMA is issued makes the compiler wait for the DMA too
    const int eA = p_exp(p_amax(amaxA + t)), eB = p_exp(p_amax(amaxB + t));
    // DMA sources as 32-bit chunk offsets from the uniform row-block bases (6 VGPRs, not 6 64-bit pointers): A's
    // block rows m0.. and B's n0.. (the last A rows clamped to M - 1: read, never stored)
    const p_u32x4 *baseA = A + t * sA + m0 * row_ch, *baseB = B + t * sB + (int64_t)n0 * row_ch;
    uint32_t off[G];
#pragma unroll
    for (int i = 0; i < G; i++) {
        const int q = i * NT + tid, r = q >> 3, c = (q & 7) ^ p_swz(r);
        off[i] = r < BM ? (uint32_t)(std::min<int64_t>(r, M - 1 - m0) * row_ch + c) : (uint32_t)((r - BM) * row_ch + c);
    }
    typedef __attribute__((address_space(3))) void lds_void;
    typedef __attribute__((address_space(1))) void gbl_void;
    auto issue = [&](int kt, int st) __attribute__((always_inline)) {
        p_u32x4 *base = lds + st * STG + w * 64;
#pragma unroll
        for (int i = 0; i < G; i++) {
            const int q0 = i * NT;  // instruction-uniform: which operand
            const p_u32x4 *b = (q0 >> 3) < BM ? baseA : baseB;
            __builtin_amdgcn_global_load_lds((gbl_void *)(b + off[i] + kt * 8), (lds_void *)(base + i * NT), 16, 0, 0);
        }
    };

    // fragment addresses (bytes, stage 0): A tile i / B tile j at half kh, plane p -> row r, chunk 2 (2 kh + fh) + p
    const int fr = lane & 31, fh = lane >> 5;
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) p_u32x4 *)lds;
    uint32_t adA[2][2], adB[2][2];  // [kh][p], tile 0; tile i is +32 i rows (same swizzle)
    {
        const int ra = wm * WTM + fr, rb = BM + wn * WTN + fr;
#pragma unroll
        for (int kh = 0; kh < 2; kh++)
#pragma unroll
            for (int p = 0; p < 2; p++) {
                const int c = 2 * (2 * kh + fh) + p;
                adA[kh][p] = lds0 + (uint32_t)(ra * 8 + (c ^ p_swz(ra))) * 16u;
                adB[kh][p] = lds0 + (uint32_t)(rb * 8 + (c ^ p_swz(rb))) * 16u;
            }
    }
    struct Frag {
        p_u32x4 a[TM][2], b[TN][2];  // [tile][plane]
    };
    // the 8 reads of half kh of stage st, interleaved behind the 12 MFMAs on f (fenced one by one)
    p_f32x16 hi[TM][TN], lo[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++) {
            hi[i][j] = p_f32x16{};
            lo[i][j] = p_f32x16{};
        }
    // the k-th of the NR fragment reads of half KH into g (k, KH compile-time: no runtime-indexed fragment arrays)
    auto rd = [&](Frag &g, auto K_, uint32_t so, auto KH) __attribute__((always_inline)) {
        constexpr int k = decltype(K_)::value, kh = decltype(KH)::value;
        if constexpr (k < 2 * TM)
            lds_rd(g.a[k >> 1][k & 1], adA[kh][k & 1] + so + (k >> 1) * 32 * 128);
        else
            lds_rd(g.b[(k - 2 * TM) >> 1][k & 1], adB[kh][k & 1] + so + ((k - 2 * TM) >> 1) * 32 * 128);
    };
    // MFMA m: tile (i, j), product pr -- ORD 0: a tile's three products back to back (m / 3 = tile, m % 3 = pr);
    // ORD 1: product-major (every tile's pr 0, then every tile's pr 1, ...), so consecutive MFMAs never share an
    // accumulator; each accumulator still sums the same products in the same order (the same bits)
    auto mf = [&](const Frag &f, const Frag &u, auto M_) __attribute__((always_inline)) {
        constexpr int m = decltype(M_)::value, tl = ORD ? m % (TM * TN) : m / 3, pr = ORD ? m / (TM * TN) : m % 3;
        constexpr int i = tl / TN, j = tl % TN;
        if constexpr (ONE) {  // u: f's lo planes at scale
            if constexpr (pr == 0)
                hi[i][j] = p_mfma(u.a[i][1], f.b[j][0], hi[i][j]);
            else if constexpr (pr == 1)
                hi[i][j] = p_mfma(f.a[i][0], u.b[j][1], hi[i][j]);
            else
                hi[i][j] = p_mfma(f.a[i][0], f.b[j][0], hi[i][j]);
        } else if constexpr (pr == 0)
            lo[i][j] = p_mfma(f.a[i][1], f.b[j][0], lo[i][j]);
        else if constexpr (pr == 1)
            lo[i][j] = p_mfma(f.a[i][0], f.b[j][1], lo[i][j]);
        else
            hi[i][j] = p_mfma(f.a[i][0], f.b[j][0], hi[i][j]);
    };
    // half step: the 12 MFMAs on f, with the 8 reads of g (stage offset so, half KH) one behind each of the first 8
    // (sched_group_barrier: MFMA, read, MFMA, read, ...)
    auto half = [&](const Frag &f, Frag &g, uint32_t so, auto KH, auto READS) __attribute__((always_inline)) {
        Frag u;
        if constexpr (ONE) {
#pragma unroll
            for (int i = 0; i < TM; i++) u.a[i][1] = p_unscale(f.a[i][1]);
#pragma unroll
            for (int j = 0; j < TN; j++) u.b[j][1] = p_unscale(f.b[j][1]);
        }
        static_for<NM>([&](auto M_) __attribute__((always_inline)) {
            mf(f, u, M_);
            if constexpr (decltype(READS)::value && decltype(M_)::value < NR) rd(g, M_, so, KH);
        });
        if constexpr (decltype(READS)::value) {
            static_for<NR>([&](auto) __attribute__((always_inline)) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            });
            if constexpr (NM > NR) __builtin_amdgcn_sched_group_barrier(0x008, NM - NR, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    auto touch = [&](const Frag &f) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < TM; i++) asm volatile("" ::"v"(f.a[i][0]), "v"(f.a[i][1]));
#pragma unroll
        for (int j = 0; j < TN; j++) asm volatile("" ::"v"(f.b[j][0]), "v"(f.b[j][1]));
    };

    static_assert(NK >= NS - 1, "the prologue's k steps");
    constexpr int D = NS - 1;  // k steps in flight
    static_for<D>([&](auto KT) __attribute__((always_inline)) { issue(decltype(KT)::value, decltype(KT)::value); });
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G * (D - 1)) : "memory");  // step 0 landed
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    Frag f0, f1;
    static_for<NR>([&](auto K_) __attribute__((always_inline)) { rd(f0, K_, 0, IC<0>{}); });
    static_for<NK>([&](auto KT) __attribute__((always_inline)) {
        constexpr int kt = decltype(KT)::value, st = kt % NS, sn = (kt + 1) % NS;
        if constexpr (kt + D < NK && !(ABL & 1)) issue(kt + D, (kt + D) % NS);  // the stage read in step kt - 1
        // (ABL bit 1, a probe: no DMA in the loop -- the MFMA / fragment-read side alone, wrong results)
        __builtin_amdgcn_sched_barrier(0);
        half(f0, f1, (uint32_t)st * STG_B, IC<1>{}, IC<1>{});  // MFMAs of half 0, reads of half 1
        if constexpr (kt + 1 < NK) {
            touch(f1);  // the compiler's wait for f1 here, before the barrier
            // step kt + 1 landed: the steps issued after it (up to kt + D, those that exist) may stay in flight
            constexpr int later = (NK - 1 < kt + D ? NK - 1 : kt + D) - (kt + 1);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G * later) : "memory");
            __builtin_amdgcn_s_barrier();  // step kt + 1 published; every wave is past its reads of step kt - 1
            __builtin_amdgcn_sched_barrier(0);
            half(f1, f0, (uint32_t)sn * STG_B, IC<0>{}, IC<1>{});  // MFMAs of half 1, reads of the next half 0
        } else {
            half(f1, f0, 0u, IC<0>{}, IC<0>{});
        }
    });

    const float inv = p_pow2(-eA), invB = p_pow2(-eB);
    float *Ct = C + t * sC;
    if constexpr ((ABL & 2) != 0) {  // probe: no tile stores -- one sum per wave keeps the MFMAs live (wrong results)
        float sum = 0.0f;
#pragma unroll
        for (int i = 0; i < TM; i++)
#pragma unroll
            for (int j = 0; j < TN; j++)
#pragma unroll
                for (int r = 0; r < 16; r++) sum += hi[i][j][r] + lo[i][j][r];
        if (lane == 0 && m0 + w < M) Ct[(m0 + w) * N + n0] = sum;
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
                    const float v = (ONE ? hi[i][j][r] : hi[i][j][r] + lo[i][j][r] * P_LO_INV) * inv * invB;
                    Ct[row * N + col] = EPI == 1 ? p_relu(v + bv) : v;
                }
            }
        }
    }
}

template <int BM, int BN, int WGM, int WGN, int NS = 3, bool ONE = false, int ABL = 0, int ORD = 0>
hipError_t pq_launch(const void *A, const void *B, const uint32_t *amaxA, const uint32_t *amaxB, int64_t M, int N,
                     int K, int T, int64_t sA, int64_t sB, const float *bias, float *C, int64_t sC, hipStream_t s) {
    if (N % BN || K % 32 || K < 64) return hipErrorInvalidValue;
    const int64_t tiles_m = (M + BM - 1) / BM;
    const int tiles_n = N / BN;
    if (tiles_m * tiles_n > INT32_MAX) return hipErrorInvalidValue;
    const dim3 grid((unsigned)(tiles_m * tiles_n), T), block(64 * WGM * WGN);
    const auto *a = static_cast<const p_u32x4 *>(A);
    const auto *b = static_cast<const p_u32x4 *>(B);
#define PQ_K(NK)                                                                                                   \
    do {                                                                                                           \
        if (bias)                                                                                                  \
            hipLaunchKernelGGL((k_h3_pq<BM, BN, WGM, WGN, 1, NK, NS, ONE, ABL, ORD>), grid, block, 0, s, a, b, amaxA, amaxB, M, N, K, \
                               sA / 4, sB / 4, bias, C, sC, tiles_n);                                              \
        else                                                                                                       \
            hipLaunchKernelGGL((k_h3_pq<BM, BN, WGM, WGN, 0, NK, NS, ONE, ABL, ORD>), grid, block, 0, s, a, b, amaxA, amaxB, M, N, K, \
                               sA / 4, sB / 4, nullptr, C, sC, tiles_n);                                           \
    } while (0)
    switch (K) {  // the k loop is unrolled: one instantiation per depth (fc1's forward K = 576, input gradient 512)
        case 576: PQ_K(18); break;
        case 512: PQ_K(16); break;
        default: return hipErrorInvalidValue;
    }
#undef PQ_K
    return hipGetLastError();
}


// ---------------------------------------------------------------------------------------------------------------
// TN over plane operands with LDS-DMA staging (round 5; the weight gradient dz^T a3, merlin_h3_gemm_tn_gather_planes
// with cfg 20): slab[s][t][m][n] = sum over the split's rows k of A[t][k][m] B[t][k][n], A planes [Kd][M/8][2][8]
// (k_head_bwd's dz), B planes gathered by 64-column chunks (row k's chunk j is row bmap[k * N / 64 + j] of B seen
// as [*][64]: conv3's representatives).  The LDS images are k_h3_tn's -- per operand and plane [32 k rows][RC chunks
// of 8 columns], chunk c of row r at c ^ swz(r), fragments k-contiguous through ds_read_b64_tr_b16 -- but filled by
// DMA three k steps deep: a DMA writes its 64 lanes' 16-B chunks lane-linear, so each lane's source is the chunk
// whose image slot that is (the swizzle and the plane deinterleave are in the source addresses).  B's chunk rows
// come from bmap through a 3-slot LDS ring, itself filled by DMA four steps ahead, so the data DMA's addresses need
// no global load in the loop.  Rows past the split's end read a zero chunk; a split's step count is padded to a
// multiple of three (the ring's period: compile-time stages) with such steps.
// The DMAs are inline asm (s_mov_b32 m0 + global_load_lds_*): issued through the builtin, hipcc treats every LDS read
// that follows as possibly aliasing an in-flight DMA and waits vmcnt(0) before the first fragment read of each step
// (profiles/r05 .s of the first version), which serialises the pipeline; here the waits are all explicit: vmcnt
// counts this wave's DMAs in issue order and the barrier after each wait publishes every wave's.
// Same products in the same order as k_h3_tn / k_h3_tng: the same bits.
__device__ uint4 p_zero16[1] = {{0u, 0u, 0u, 0u}};

// m0 is a reserved register to LLVM (a clobber entry is ignored, with a warning), so the asm saves it in a scratch
// SGPR and puts it back behind the DMA: the compiler's view of m0 is unchanged by these statements whatever it keeps
// there.  (The DMA reads m0 at issue: the compiler's own code rewrites m0 right behind each global_load_lds too.)
__device__ __forceinline__ void p_dma16(const void *src, uint32_t lds) {  // lds: wave-uniform byte address
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds)
                 : "memory");
}
__device__ __forceinline__ void p_dma4(const void *src, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds)
                 : "memory");
}

template <int RC>
__device__ __forceinline__ int p_tr_swz(int row) {
    static_assert(RC % 16 == 0 || RC == 24 || RC == 8, "row chunks");  // 8 (128-B rows): as 24
    return RC % 16 == 0 ? (row & 3) << 2 : ((row >> 1) & 1) << 2;
}
typedef __bf16 p_bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 p_bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) p_bf16x4 lds_p_bf16x4;
typedef __attribute__((address_space(3))) int32_t lds_i32;

template <int BM, int BN, int WGM, int WGN>
__global__ __launch_bounds__(64 * WGM * WGN) void k_h3_tq(const p_u32x4 *__restrict__ A, const p_u32x4 *__restrict__ B,
                                                          const uint32_t *__restrict__ amaxA,
                                                          const uint32_t *__restrict__ amaxB, int64_t Kd, int M,
                                                          int N, int64_t sA, int64_t sB, int64_t kc, int tiles_n,
                                                          int tiles, int S, float *__restrict__ slab,
                                                          const int32_t *__restrict__ bmap) {
    constexpr int NT = 64 * WGM * WGN, NW = NT / 64;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int RCA = BM / 8, RCB = BN / 8;
    constexpr int PSA = 32 * RCA, PSB = 32 * RCB;  // chunks per plane image
    constexpr int STG = 2 * (PSA + PSB);
    constexpr uint32_t STG_B = STG * 16;
    static_assert((2 * PSA) % NT == 0 && (2 * PSB) % NT == 0, "whole DMA instructions per operand");
    constexpr int GA = 2 * PSA / NT, GB = 2 * PSB / NT, G = GA + GB + 1;  // + the index DMA
    constexpr int JB = BN / 64;   // 64-column chunks of B per tile (bmap entries per row)
    constexpr int XS = 64 * NW;   // index ring slot (ints; 32 * JB used)
    static_assert(32 * JB <= XS, "index slot");
    constexpr int NF = 2 * (TM + TN);             // fragments per half step (tiles x planes)
    constexpr int NR = 2 * NF, NM = 3 * TM * TN;  // tr reads (two per fragment) / MFMAs per half step
    __shared__ p_u32x4 lds[3 * STG];
    __shared__ int32_t ixr[3 * XS];

    const int P = p_xcd_tile(blockIdx.x, gridDim.x);
    const int t = P / (S * tiles), s = (P / tiles) % S, Lt = P % tiles;
    const int tm = Lt / tiles_n, tn = Lt - tm * tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int64_t k0 = (int64_t)s * kc, k1 = std::min<int64_t>(Kd, k0 + kc);
    const int eA = p_exp(p_amax(amaxA + t)), eB = p_exp(p_amax(amaxB + t));
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WGN, wn = w - (w / WGN) * WGN;
    const int nc = N / 64, j0 = n0 / 64;
    const int64_t rowA = M / 4;  // chunks per A row
    const p_u32x4 *At = A + t * sA, *Bt = B + t * sB;
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) p_u32x4 *)lds;
    const uint32_t ix0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) int32_t *)ixr;
    const uint32_t wbase = (uint32_t)__builtin_amdgcn_readfirstlane(w) * 64u;  // the wave's first slot

    // the thread's DMA slots: A (instructions 0 .. GA-1): row ra, chunk offset oa; B: row rb, ring entry xb, offset gp
    int ra[GA], rb[GB], xb[GB];
    uint32_t oa[GA], gp[GB];
#pragma unroll
    for (int i = 0; i < GA; i++) {
        const int q = i * NT + tid, p = q / PSA, rem = q - p * PSA, r = rem / RCA, cs = rem - r * RCA;
        const int c = cs ^ p_tr_swz<RCA>(r);
        ra[i] = r;
        oa[i] = (uint32_t)((m0 / 8 + c) * 2 + p);
    }
#pragma unroll
    for (int i = 0; i < GB; i++) {
        const int q = (GA + i) * NT + tid - 2 * PSA, p = q / PSB, rem = q - p * PSB, r = rem / RCB,
                  cs = rem - r * RCB;
        const int c = cs ^ p_tr_swz<RCB>(r), col = 8 * c;
        rb[i] = r;
        xb[i] = r * JB + (col >> 6);
        gp[i] = (uint32_t)(((col & 63) >> 3) * 2 + p);
    }
    // the index DMA: this thread's ring entry e = tid (< 32 JB used): row e / JB, chunk j0 + e % JB
    const int xr = tid / JB, xj = j0 + tid % JB;
    const int64_t nk = (k1 - k0 + 31) / 32, nk3 = (nk + 2) / 3 * 3;

    auto issue_ix = [&](int64_t kt, int slot) __attribute__((always_inline)) {
        const int64_t row = std::min<int64_t>(k0 + kt * 32 + (tid < 32 * JB ? xr : 0), k1 - 1);
        p_dma4(bmap + row * nc + (tid < 32 * JB ? xj : j0), ix0 + (uint32_t)(slot * XS) * 4u + wbase * 4u);
    };
    // this thread's chunk rows of a step from its index slot (read a step before they are used)
    auto read_ix = [&](int slot, int32_t (&x)[GB]) __attribute__((always_inline)) {
        const lds_i32 *xs = (const lds_i32 *)(uintptr_t)(ix0 + (uint32_t)(slot * XS) * 4u);
#pragma unroll
        for (int i = 0; i < GB; i++) x[i] = xs[xb[i]];
    };
    auto issue = [&](int64_t kt, int st, const int32_t (&x)[GB]) __attribute__((always_inline)) {
        const uint32_t base = lds0 + (uint32_t)(st * STG) * 16u + wbase * 16u;
        const int64_t kk = k0 + kt * 32;
        const bool full = kk + 32 <= k1;  // block-uniform
#pragma unroll
        for (int i = 0; i < GA; i++) {
            const p_u32x4 *src = full || kk + ra[i] < k1 ? At + (kk + ra[i]) * rowA + oa[i]
                                                          : reinterpret_cast<const p_u32x4 *>(p_zero16);
            p_dma16(src, base + (uint32_t)(i * NT) * 16u);
        }
#pragma unroll
        for (int i = 0; i < GB; i++) {
            const p_u32x4 *src = full || kk + rb[i] < k1 ? Bt + (int64_t)x[i] * 16 + gp[i]
                                                          : reinterpret_cast<const p_u32x4 *>(p_zero16);
            p_dma16(src, base + (uint32_t)((GA + i) * NT) * 16u);
        }
    };

    // fragment reads: fragment f < NF (A tiles x planes, then B tiles x planes), its two transposed halves
    const int fg = lane >> 4, fq = (lane >> 2) & 3, fp = lane & 3;
    struct Frag {
        p_bf16x4 v[NF][2];
    };
    auto rd = [&](Frag &g, auto K_, uint32_t so, auto KH) __attribute__((always_inline)) {
        constexpr int k = decltype(K_)::value, kh = decltype(KH)::value, f = k >> 1, h2 = k & 1;
        constexpr bool isA = f < 2 * TM;
        constexpr int tile = isA ? f >> 1 : (f - 2 * TM) >> 1, pl = f & 1;
        constexpr int RC = isA ? RCA : RCB;
        const int col0 = isA ? wm * WTM + tile * 32 : wn * WTN + tile * 32;
        const uint32_t img = lds0 + so + (uint32_t)(isA ? pl * PSA : 2 * PSA + pl * PSB) * 16u;
        const int chunk = ((col0 + 16 * (fg & 1)) >> 3) + (fp >> 1);
        const int row = 16 * kh + 8 * (fg >> 1) + 4 * h2 + fq;
        const uint32_t off = img + (uint32_t)((row * RC + (chunk ^ p_tr_swz<RC>(row))) * 16 + (fp & 1) * 8);
        g.v[f][h2] = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_p_bf16x4 *)(uintptr_t)off);
    };
    auto frag = [](const Frag &g, int f) __attribute__((always_inline)) {
        return __builtin_bit_cast(p_u32x4, p_bf16x8{g.v[f][0][0], g.v[f][0][1], g.v[f][0][2], g.v[f][0][3],
                                                   g.v[f][1][0], g.v[f][1][1], g.v[f][1][2], g.v[f][1][3]});
    };
    p_f32x16 hi[TM][TN], lo[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++) {
            hi[i][j] = p_f32x16{};
            lo[i][j] = p_f32x16{};
        }
    // MFMA m of a half step: tile (i, j) = (m / (3 TN), (m / 3) % TN), product m % 3 (k_h3_tn's order per tile)
    auto mf = [&](const Frag &f, auto M_) __attribute__((always_inline)) {
        constexpr int m = decltype(M_)::value, i = m / (3 * TN), j = (m / 3) % TN, pr = m % 3;
        constexpr int fa0 = 2 * i, fa1 = 2 * i + 1, fb0 = 2 * TM + 2 * j, fb1 = 2 * TM + 2 * j + 1;
        if constexpr (pr == 0)
            lo[i][j] = p_mfma(frag(f, fa1), frag(f, fb0), lo[i][j]);
        else if constexpr (pr == 1)
            lo[i][j] = p_mfma(frag(f, fa0), frag(f, fb1), lo[i][j]);
        else
            hi[i][j] = p_mfma(frag(f, fa0), frag(f, fb0), hi[i][j]);
    };
    constexpr int RPM = (NR + NM - 1) / NM;  // reads behind each MFMA
    auto half = [&](const Frag &f, Frag &g, uint32_t so, auto KH) __attribute__((always_inline)) {
        static_for<NM>([&](auto M_) __attribute__((always_inline)) {
            mf(f, M_);
            static_for<RPM>([&](auto R_) __attribute__((always_inline)) {
                constexpr int k = decltype(M_)::value * RPM + decltype(R_)::value;
                if constexpr (k < NR) rd(g, IC<k>{}, so, KH);
            });
        });
        static_for<NM>([&](auto M_) __attribute__((always_inline)) {
            constexpr int left = NR - decltype(M_)::value * RPM;
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            if constexpr (left > 0) __builtin_amdgcn_sched_group_barrier(0x100, left < RPM ? left : RPM, 0);
        });
        __builtin_amdgcn_sched_barrier(0);
    };
    auto touch = [&](const Frag &f) __attribute__((always_inline)) {
#pragma unroll
        for (int q = 0; q < NF; q++) asm volatile("" ::"v"(f.v[q][0]), "v"(f.v[q][1]));
    };
    auto publish = [&](auto CNT) __attribute__((always_inline)) {  // this wave's DMAs but the last CNT landed, then
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(decltype(CNT)::value) : "memory");  // every wave's
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };

    // prologue: indices of steps 0..2 (slot = step % 3); DMA of steps 0 and 1; once every wave has read slot 0, the
    // indices of step 3 into it
    int32_t x0[GB], x1[GB], x2[GB];  // chunk rows of the steps issued next (step k's in x[k % 3])
    issue_ix(0, 0);
    issue_ix(1, 1);
    issue_ix(2, 2);
    publish(IC<0>{});
    read_ix(0, x0);
    read_ix(1, x1);
    read_ix(2, x2);
    issue(0, 0, x0);
    issue(1, 1, x1);
    publish(IC<G - 1>{});  // DMA 0 landed (DMA 1 may not); every wave has read slots 0 .. 2
    issue_ix(3, 0);
    Frag f0, f1;
    static_for<NR>([&](auto K_) __attribute__((always_inline)) { rd(f0, K_, 0u, IC<0>{}); });
    // step kt (stage st = kt % 3): the indices of kt + 4 (slot (kt + 1) % 3, last read at step kt - 1), the DMA of
    // kt + 2 (stage (kt + 2) % 3, its chunk rows read a step ago), half 0, publish kt + 1 (the two DMA groups just
    // issued may stay in flight; the indices of kt + 3 have landed), read those, half 1
    auto step = [&](int64_t kt, auto ST, int32_t (&xu)[GB], int32_t (&xn)[GB]) __attribute__((always_inline)) {
        constexpr int st = decltype(ST)::value, sn = (st + 1) % 3, s2 = (st + 2) % 3;
        issue_ix(kt + 4, sn);
        issue(kt + 2, s2, xu);
        __builtin_amdgcn_sched_barrier(0);
        half(f0, f1, (uint32_t)st * STG_B, IC<1>{});
        touch(f1);
        publish(IC<G>{});
        read_ix(st, xn);  // slot st = (kt + 3) % 3
        half(f1, f0, (uint32_t)sn * STG_B, IC<0>{});
    };
    for (int64_t kt = 0; kt < nk3; kt += 3) {
        step(kt, IC<0>{}, x2, x0);
        step(kt + 1, IC<1>{}, x0, x1);
        step(kt + 2, IC<2>{}, x1, x2);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the padded steps' DMAs drained before the block ends

    const float inv = p_pow2(-eA), invB = p_pow2(-eB);
    float *St = slab + ((int64_t)s * (gridDim.x / (S * tiles)) + t) * (int64_t)M * N;
    const int fr = lane & 31, fh = lane >> 5;
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int row = m0 + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
                St[(int64_t)row * N + n0 + wn * WTN + j * 32 + fr] = (hi[i][j][r] + lo[i][j][r] * P_LO_INV) * inv * invB;
            }
}


// ---------------------------------------------------------------------------------------------------------------
// The update's forward over a3's planes with the rows gathered (round 5; merlin_h3_gemm_nt_heads_planes cfg 60):
// k_h3_pq's schedule (LDS-DMA three steps deep, K = 576 unrolled, fragment reads under the MFMAs) with A's rows read
// through the row map by 64-value chunks -- row m's chunk j is row amap[m * 9 + j] of A seen as [*][64] (conv3's
// patch representatives) -- and k_h3_ntp's epilogues (EPI 1 bias + ReLU; EPI 2 the same plus the policy / value
// heads' partial dot products, merlin_heads_combine's layout).  The block's 9 BM chunk rows are read into LDS once;
// a step's A sources are read from there one step ahead.  DMAs by inline asm as in k_h3_tq (no compiler-inserted
// vmcnt before LDS reads).  The same products in the same order as k_h3_ntpg: the same bits.
template <int BM, int BN, int WGM, int WGN, int EPI>
__global__ __launch_bounds__(64 * WGM * WGN) void k_h3_pqg(const p_u32x4 *__restrict__ A, const p_u32x4 *__restrict__ B,
                                                           const uint32_t *__restrict__ amaxA,
                                                           const uint32_t *__restrict__ amaxB, int64_t M, int N,
                                                           int64_t sA, int64_t sB, const float *__restrict__ bias,
                                                           float *__restrict__ C, int64_t sC, int tiles_n,
                                                           const int32_t *__restrict__ amap,
                                                           const float *__restrict__ hw0, const float *__restrict__ hw1,
                                                           int na, float *__restrict__ hpart) {
    constexpr int K = 576, NK = 18, KC = K / 64;
    constexpr int NT = 64 * WGM * WGN;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int NR = 2 * (TM + TN), NM = 3 * TM * TN;
    static_assert(NM >= NR, "a read behind every MFMA");
    constexpr int GA = BM * 8 / NT, GB = BN * 8 / NT, G = GA + GB;
    static_assert((BM * 8) % NT == 0 && (BN * 8) % NT == 0, "whole DMA instructions per thread");
    constexpr int STG = (BM + BN) * 8;
    constexpr uint32_t STG_B = STG * 16;
    __shared__ p_u32x4 lds[3 * STG];
    __shared__ int32_t gmap[BM * KC];

    const int t = blockIdx.y;
    const int L = p_xcd_tile(blockIdx.x, gridDim.x);
    const int tm = L / tiles_n, tn = L - tm * tiles_n;
    const int64_t m0 = (int64_t)tm * BM;
    const int n0 = tn * BN;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WGN, wn = w - (w / WGN) * WGN;
    const int eA = p_exp(p_amax(amaxA + t)), eB = p_exp(p_amax(amaxB + t));
    for (int e = tid; e < BM * KC; e += NT) {
        const int r = e / KC;
        gmap[e] = amap[std::min<int64_t>(m0 + r, M - 1) * KC + (e - r * KC)];
    }
    __syncthreads();
    const p_u32x4 *At = A + t * sA, *baseB = B + t * sB + (int64_t)n0 * (K / 4);
    int ga[GA];       // gmap entry base r * KC of the thread's A slots
    uint32_t ca[GA];  // their chunk within a k step
    uint32_t offB[GB];
#pragma unroll
    for (int i = 0; i < GA; i++) {
        const int q = i * NT + tid, r = q >> 3;
        ga[i] = r * KC;
        ca[i] = (uint32_t)((q & 7) ^ p_swz(r));
    }
#pragma unroll
    for (int i = 0; i < GB; i++) {
        const int q = i * NT + tid, r = q >> 3;
        offB[i] = (uint32_t)(r * (K / 4) + ((q & 7) ^ p_swz(r)));
    }
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) p_u32x4 *)lds;
    const uint32_t gm0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) int32_t *)gmap;
    const uint32_t wbase = (uint32_t)__builtin_amdgcn_readfirstlane(w) * 64u;
    // the chunk rows of step kt's A slots (plain LDS loads, read a step ahead of their issue)
    auto read_g = [&](int kt, int32_t (&g)[GA]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < GA; i++) g[i] = *(const lds_i32 *)(uintptr_t)(gm0 + (uint32_t)(ga[i] + kt / 2) * 4u);
    };
    auto issue = [&](int kt, int st, const int32_t (&g)[GA]) __attribute__((always_inline)) {
        const uint32_t base = lds0 + (uint32_t)(st * STG) * 16u + wbase * 16u;
#pragma unroll
        for (int i = 0; i < GA; i++)
            p_dma16(At + (int64_t)g[i] * 16 + 8 * (kt & 1) + ca[i], base + (uint32_t)(i * NT) * 16u);
#pragma unroll
        for (int i = 0; i < GB; i++) p_dma16(baseB + offB[i] + kt * 8, base + (uint32_t)((GA + i) * NT) * 16u);
    };

    const int fr = lane & 31, fh = lane >> 5;
    uint32_t adA[2][2], adB[2][2];
    {
        const int ra = wm * WTM + fr, rb = BM + wn * WTN + fr;
#pragma unroll
        for (int kh = 0; kh < 2; kh++)
#pragma unroll
            for (int p = 0; p < 2; p++) {
                const int c = 2 * (2 * kh + fh) + p;
                adA[kh][p] = lds0 + (uint32_t)(ra * 8 + (c ^ p_swz(ra))) * 16u;
                adB[kh][p] = lds0 + (uint32_t)(rb * 8 + (c ^ p_swz(rb))) * 16u;
            }
    }
    struct Frag {
        p_u32x4 a[TM][2], b[TN][2];
    };
    p_f32x16 hi[TM][TN], lo[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++) {
            hi[i][j] = p_f32x16{};
            lo[i][j] = p_f32x16{};
        }
    auto rd = [&](Frag &g, auto K_, uint32_t so, auto KH) __attribute__((always_inline)) {
        constexpr int k = decltype(K_)::value, kh = decltype(KH)::value;
        if constexpr (k < 2 * TM)
            lds_rd(g.a[k >> 1][k & 1], adA[kh][k & 1] + so + (k >> 1) * 32 * 128);
        else
            lds_rd(g.b[(k - 2 * TM) >> 1][k & 1], adB[kh][k & 1] + so + ((k - 2 * TM) >> 1) * 32 * 128);
    };
    auto mf = [&](const Frag &f, auto M_) __attribute__((always_inline)) {
        constexpr int m = decltype(M_)::value, i = m / (3 * TN), j = (m / 3) % TN, pr = m % 3;
        if constexpr (pr == 0)
            lo[i][j] = p_mfma(f.a[i][1], f.b[j][0], lo[i][j]);
        else if constexpr (pr == 1)
            lo[i][j] = p_mfma(f.a[i][0], f.b[j][1], lo[i][j]);
        else
            hi[i][j] = p_mfma(f.a[i][0], f.b[j][0], hi[i][j]);
    };
    auto half = [&](const Frag &f, Frag &g, uint32_t so, auto KH, auto READS) __attribute__((always_inline)) {
        static_for<NM>([&](auto M_) __attribute__((always_inline)) {
            mf(f, M_);
            if constexpr (decltype(READS)::value && decltype(M_)::value < NR) rd(g, M_, so, KH);
        });
        if constexpr (decltype(READS)::value) {
            static_for<NR>([&](auto) __attribute__((always_inline)) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            });
            if constexpr (NM > NR) __builtin_amdgcn_sched_group_barrier(0x008, NM - NR, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    auto touch = [&](const Frag &f) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < TM; i++) asm volatile("" ::"v"(f.a[i][0]), "v"(f.a[i][1]));
#pragma unroll
        for (int j = 0; j < TN; j++) asm volatile("" ::"v"(f.b[j][0]), "v"(f.b[j][1]));
    };

    int32_t g0[GA], g1[GA];  // chunk rows of the next issue (ping-pong, compile-time choice)
    read_g(0, g0);
    issue(0, 0, g0);
    read_g(1, g1);
    issue(1, 1, g1);
    read_g(2, g0);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    Frag f0, f1;
    static_for<NR>([&](auto K_) __attribute__((always_inline)) { rd(f0, K_, 0, IC<0>{}); });
    static_for<NK>([&](auto KT) __attribute__((always_inline)) {
        constexpr int kt = decltype(KT)::value, st = kt % 3, sn = (kt + 1) % 3;
        int32_t(&gu)[GA] = (kt % 2 == 0) ? g0 : g1;  // holds step kt + 2's rows
        int32_t(&gn)[GA] = (kt % 2 == 0) ? g1 : g0;
        if constexpr (kt + 2 < NK) issue(kt + 2, (kt + 2) % 3, gu);
        __builtin_amdgcn_sched_barrier(0);
        half(f0, f1, (uint32_t)st * STG_B, IC<1>{}, IC<1>{});
        if constexpr (kt + 1 < NK) {
            touch(f1);
            if constexpr (kt + 2 < NK)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (kt + 3 < NK) read_g(kt + 3, gn);
            half(f1, f0, (uint32_t)sn * STG_B, IC<0>{}, IC<1>{});
        } else {
            half(f1, f0, 0u, IC<0>{}, IC<0>{});
        }
    });

    const float inv = p_pow2(-eA), invB = p_pow2(-eB);
    float *Ct = C + t * sC;
    if constexpr (EPI == 2) {  // k_h3_ntp's heads epilogue (merlin_h3.hip h3_ntp_body EPI 2)
        static_assert(TN == 2 && WTN == 64, "heads epilogue: a wave tile 64 columns wide");
        const float *hw = t == 0 ? hw0 : hw1;
        const int nh = t == 0 ? na : 1;
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
        float *part = hpart + ((int64_t)(t * tiles_n + tn) * WGN + wn) * M * 4;
#pragma unroll
        for (int i = 0; i < TM; i++) {
            float pv[64];
#pragma unroll
            for (int q = 0; q < 64; q++) pv[q] = 0.0f;
#pragma unroll
            for (int j = 0; j < TN; j++) {
                const int col = n0 + wn * WTN + j * 32 + fr;
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const int64_t row = m0 + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
                    const float v = p_relu((hi[i][j][r] + lo[i][j][r] * P_LO_INV) * inv * invB + bv[j]);
                    if (row < M) Ct[row * N + col] = v;
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
                    const float v = (hi[i][j][r] + lo[i][j][r] * P_LO_INV) * inv * invB;
                    Ct[row * N + col] = EPI == 1 ? p_relu(v + bv) : v;
                }
            }
        }
    }
}

}  // namespace

// A, B: plane images (4 B per value, strides in values); cfg 60: 128 x 256 tiles (2 x 4 waves),
// 62: 128 x 192 (4 x 2 waves of 32 x 96: N = 576)
hipError_t launch_h3p_gemm_nt(const void *A, const uint32_t *amaxA, const void *B, const uint32_t *amaxB, int64_t M,
                              int N, int K, int T, int64_t a_stride, int64_t b_stride, const float *bias, float *C,
                              int64_t c_stride, int cfg, hipStream_t s, const int32_t *a_rows, const float *head_w0,
                              int n_actions, const float *head_w1, float *head_part) {
    if (M <= 0) return hipSuccess;
    if (a_stride % 4 || b_stride % 4) return hipErrorInvalidValue;
    if (a_rows) {  // the forward over a3's gathered planes (cfg 60 tiles, K = 576), bias + ReLU, heads optional
        constexpr int BM = 128, BN = 256;
        if (cfg != 60 || K != 576 || N % BN || !bias || !C) return hipErrorInvalidValue;
        if (head_part && (T != 2 || n_actions < 1 || n_actions > 4 || !head_w0 || !head_w1)) return hipErrorInvalidValue;
        const int64_t tiles_m = (M + BM - 1) / BM;
        const int tiles_n = N / BN;
        const dim3 grid((unsigned)(tiles_m * tiles_n), T), block(512);
        const auto *a = static_cast<const p_u32x4 *>(A);
        const auto *b = static_cast<const p_u32x4 *>(B);
        if (head_part)
            hipLaunchKernelGGL((k_h3_pqg<BM, BN, 2, 4, 2>), grid, block, 0, s, a, b, amaxA, amaxB, M, N, a_stride / 4,
                               b_stride / 4, bias, C, c_stride, tiles_n, a_rows, head_w0, head_w1, n_actions,
                               head_part);
        else
            hipLaunchKernelGGL((k_h3_pqg<BM, BN, 2, 4, 1>), grid, block, 0, s, a, b, amaxA, amaxB, M, N, a_stride / 4,
                               b_stride / 4, bias, C, c_stride, tiles_n, a_rows, nullptr, nullptr, 0, nullptr);
        return hipGetLastError();
    }
    switch (cfg) {
        case 60: return pq_launch<128, 256, 2, 4>(A, B, amaxA, amaxB, M, N, K, T, a_stride, b_stride, bias, C, c_stride, s);
        case 62: return pq_launch<128, 192, 4, 2>(A, B, amaxA, amaxB, M, N, K, T, a_stride, b_stride, bias, C, c_stride, s);
        // round 6: the same with a 4-stage ring (160 KB of LDS, three k steps in flight)
        case 63: return pq_launch<128, 192, 4, 2, 4>(A, B, amaxA, amaxB, M, N, K, T, a_stride, b_stride, bias, C, c_stride, s);
        // round 6: one accumulator per tile (ONE): 65: 256 x 192 tiles on a 2-stage ring (112 KB), 66: 62's 128 x 192
        // tile, 68: 256 x 256 over 4 waves (one per SIMD: 512 registers each; 8 waves spill), 69: 192 x 192 over 6
        // waves, 3 stages (144 KB)
        case 65: return pq_launch<256, 192, 4, 2, 2, true>(A, B, amaxA, amaxB, M, N, K, T, a_stride, b_stride, bias, C, c_stride, s);
        // 66: 62 with the MFMAs product-major (ORD 1: no two consecutive MFMAs on one accumulator; the same bits)
        case 66: return pq_launch<128, 192, 4, 2, 3, false, 0, 1>(A, B, amaxA, amaxB, M, N, K, T, a_stride, b_stride, bias, C, c_stride, s);
        case 68: return pq_launch<256, 256, 2, 2, 2, true>(A, B, amaxA, amaxB, M, N, K, T, a_stride, b_stride, bias, C, c_stride, s);
        case 69: return pq_launch<192, 192, 3, 2, 3, true>(A, B, amaxA, amaxB, M, N, K, T, a_stride, b_stride, bias, C, c_stride, s);
#ifdef MERLIN_PROBES  // ablations (ABL 1: no DMA in the k loop -- wrong results on purpose): 64 = 65's, 67 = 62's, 61 = 66's
        case 64: return pq_launch<256, 192, 4, 2, 2, true, 1>(A, B, amaxA, amaxB, M, N, K, T, a_stride, b_stride, bias, C, c_stride, s);
        case 67: return pq_launch<128, 192, 4, 2, 3, false, 1>(A, B, amaxA, amaxB, M, N, K, T, a_stride, b_stride, bias, C, c_stride, s);
        case 61: return pq_launch<128, 192, 4, 2, 3, false, 1, 1>(A, B, amaxA, amaxB, M, N, K, T, a_stride, b_stride, bias, C, c_stride, s);
        // ABL 2: no tile stores (the epilogue's share); ABL 3: neither DMA in the loop nor stores -- 70 / 71 = 62's,
        // 72 / 73 = 60's (the forward's 128 x 256 tile)
        case 70: return pq_launch<128, 192, 4, 2, 3, false, 2>(A, B, amaxA, amaxB, M, N, K, T, a_stride, b_stride, bias, C, c_stride, s);
        case 71: return pq_launch<128, 192, 4, 2, 3, false, 3>(A, B, amaxA, amaxB, M, N, K, T, a_stride, b_stride, bias, C, c_stride, s);
        case 72: return pq_launch<128, 256, 2, 4, 3, false, 2>(A, B, amaxA, amaxB, M, N, K, T, a_stride, b_stride, bias, C, c_stride, s);
        case 73: return pq_launch<128, 256, 2, 4, 3, false, 3>(A, B, amaxA, amaxB, M, N, K, T, a_stride, b_stride, bias, C, c_stride, s);
        case 74: return pq_launch<128, 256, 2, 4, 3, false, 1>(A, B, amaxA, amaxB, M, N, K, T, a_stride, b_stride, bias, C, c_stride, s);
#endif
        default: return hipErrorInvalidValue;
    }
}


// the weight gradient over plane operands with B's rows gathered (cfg 20: 128 x 192 tiles, 4 x 2 waves); slab as
// merlin_h3_gemm_tn's (S slabs of [T][M][N], summed in order by the caller's fold); strides in values
hipError_t launch_h3p_gemm_tn_gather(const void *A, const uint32_t *amaxA, const void *B, const uint32_t *amaxB,
                                     int64_t Kd, int M, int N, int T, int64_t a_stride, int64_t b_stride, int splits,
                                     float *slab, const int32_t *b_rows, int cfg, int *S_out, hipStream_t s) {
    // cfg 20: 128 x 192 tiles, 8 waves (the whole CU: 256 VGPRs x 2 waves per SIMD, 126 KB of LDS); cfg 21: 64 x 192,
    // 4 waves of the same wave tile (one per SIMD, ~99 KB of LDS), which leaves half of each SIMD's registers to
    // kernels queued beside it (conv3's backward sums)
    const int BM = cfg == 21 ? 64 : 128;
    constexpr int BN = 192, BK = 32;
    if ((cfg != 20 && cfg != 21) || M % BM || N % BN || N % 64 || a_stride % 4 || b_stride % 4 || !b_rows)
        return hipErrorInvalidValue;
    const int tiles_n = N / BN, tiles = (M / BM) * tiles_n;
    int S = std::max(1, splits);
    int64_t kc = (Kd + S - 1) / S;
    kc = (kc + BK - 1) / BK * BK;
    S = (int)std::max<int64_t>(1, (Kd + kc - 1) / kc);
    *S_out = S;
    if (cfg == 21)
        hipLaunchKernelGGL((k_h3_tq<64, BN, 2, 2>), dim3(tiles * S * T), dim3(256), 0, s,
                           static_cast<const p_u32x4 *>(A), static_cast<const p_u32x4 *>(B), amaxA, amaxB, Kd, M, N,
                           a_stride / 4, b_stride / 4, kc, tiles_n, tiles, S, slab, b_rows);
    else
        hipLaunchKernelGGL((k_h3_tq<128, BN, 4, 2>), dim3(tiles * S * T), dim3(512), 0, s,
                           static_cast<const p_u32x4 *>(A), static_cast<const p_u32x4 *>(B), amaxA, amaxB, Kd, M, N,
                           a_stride / 4, b_stride / 4, kc, tiles_n, tiles, S, slab, b_rows);
    return hipGetLastError();
}

}  // namespace merlin
