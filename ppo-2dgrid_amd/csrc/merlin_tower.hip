// merlin_tower.hip -- memory-bound glue of the CNN towers' GEMM formulation.
//
// Both CNNFeatureExtractor towers (src/actor_critic.py:6-21) run as
//   A2 = im2col(relu(conv1(frame)))   [T][n*25][512]  <- k_conv1_im2col_fwd (from tile codes)
//   Z2 = A2 @ W2t                     [T][n*25][64]   (hipBLASLt fp32, MFMA)
//   A3 = im2col(relu(Z2 + b2))        [T][n*9][576]   <- k_im2col3_fwd
//   Z3 = A3 @ W3t                     [T][n*9][64]    (hipBLASLt)
//   a3 = relu(Z3 + b3), rows (p3, co) feed fc1 with W4's columns permuted to (p3, co)
// with K orders (ky, kx, ci) so that every im2col row is 2 KB / 2.3 KB of contiguous
// floats and the GEMMs are plain row-major products.  conv1 is never evaluated as a
// convolution: each of its outputs is bias + 4 lookups in the per-tower table P
// (see merlin_conv1.hip for the derivation), recomputed wherever it is needed.
// Backward:
//   dA2 (= dZ2 @ W2t^T)  -> k_conv1_im2col_bwd: col2im + ReLU mask (z1 > 0 recomputed
//                           from P) + the class/quarter histogram -> dP, db1
//   dA3 (= dZ3 @ W3t^T)  -> k_col2im3_bwd: col2im + ReLU mask of conv2 -> dZ2
#include <algorithm>

#include "merlin_internal.h"

namespace merlin {
namespace {

constexpr int C1 = 32, NPOS1 = 169, NBIN = 20, NSLOT = 4;
constexpr int TAB = C1 * NSLOT * NBIN;    // floats per tower table (layout [co][slot][bin] in HBM)
constexpr int K2 = 512, P2 = 25;          // conv2: K = 4*4 taps x 32 ci, 5x5 outputs
constexpr int C2 = 64, K3 = 576, P3 = 9;  // conv3: K = 3*3 taps x 64 ci, 3x3 outputs
constexpr int MAXT = 2;
constexpr int BLK = 256;
constexpr int SLAB = C1 * (NSLOT * NBIN + 1);

__device__ __forceinline__ void load_codes(const uint32_t *__restrict__ codes, int64_t row, uint32_t w[8]) {
    const uint4 *c = reinterpret_cast<const uint4 *>(codes + row * MERLIN_OBS_WORDS);
    const uint4 a = c[0], b = c[1];
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
    w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}

// LDS table layout [t][slot*20 + bin][ci]: lanes with consecutive ci read consecutive words.
__device__ __forceinline__ void stage_tables(const float *__restrict__ tables, const float *__restrict__ bias,
                                             int T, float *tab, float *sb) {
    for (int k = threadIdx.x; k < T * TAB; k += blockDim.x) {
        const int t = k / TAB, r = k - t * TAB, co = r / (NSLOT * NBIN), e = r - co * (NSLOT * NBIN);
        tab[(t * NSLOT * NBIN + e) * C1 + co] = tables[k];
    }
    for (int k = threadIdx.x; k < T * C1; k += blockDim.x) sb[k] = bias[k];
}

// slot bins of the 169 conv1 output positions of one frame: bins[p] = 4 x u8 (slot*20 + cls*4 + q)
__device__ __forceinline__ void stage_bins(const uint32_t w[8], uint32_t *bins) {
    for (int p = threadIdx.x; p < NPOS1; p += blockDim.x) {
        const int oy = p / 13, ox = p - (p / 13) * 13;
        uint32_t packed = 0u;
#pragma unroll
        for (int dy = 0; dy < 2; dy++)
#pragma unroll
            for (int dx = 0; dx < 2; dx++) {
                const int qr = oy + dy, qc = ox + dx, cell = (qr >> 1) * 7 + (qc >> 1);
                const uint32_t cls = (w[cell >> 3] >> ((cell & 7) * 4)) & 0xfu;
                const int slot = dy * 2 + dx;
                packed |= (uint32_t)(slot * NBIN + (int)cls * 4 + (qr & 1) * 2 + (qc & 1)) << (8 * slot);
            }
        bins[p] = packed;
    }
}

__device__ __forceinline__ float conv1_z(const float *tab, const float *sb, int t, int ci, uint32_t b) {
    const float *tt = tab + t * NSLOT * NBIN * C1 + ci;
    return (((sb[t * C1 + ci] + tt[(b & 0xff) * C1]) + tt[((b >> 8) & 0xff) * C1]) + tt[((b >> 16) & 0xff) * C1]) +
           tt[(b >> 24) * C1];
}

// ---------------------------------------------------------------------------
// A2[t][s*25 + p2][(ky*4 + kx)*32 + ci] = relu(z1[t][ci][2oy+ky][2ox+kx])
__global__ __launch_bounds__(BLK, 2) void k_conv1_im2col_fwd(const uint32_t *__restrict__ codes,
                                                          const int64_t *__restrict__ index, int64_t n,
                                                          const float *__restrict__ tables,
                                                          const float *__restrict__ bias, int T,
                                                          float4 *__restrict__ out) {
    __shared__ float tab[MAXT * TAB];
    __shared__ float sb[MAXT * C1];
    __shared__ uint32_t bins[NPOS1];
    __shared__ __align__(16) float a1[MAXT * NPOS1 * C1];  // [t][pos][ci]
    stage_tables(tables, bias, T, tab, sb);
    for (int64_t s = blockIdx.x; s < n; s += gridDim.x) {
        uint32_t w[8];
        load_codes(codes, index ? index[s] : s, w);
        __syncthreads();  // previous sample's a1 fully consumed; tables staged
        stage_bins(w, bins);
        __syncthreads();
        for (int e = threadIdx.x; e < T * NPOS1 * C1; e += BLK) {
            const int t = e / (NPOS1 * C1), r = e - t * (NPOS1 * C1), p = r >> 5, ci = r & 31;
            a1[e] = fmaxf(conv1_z(tab, sb, t, ci, bins[p]), 0.0f);
        }
        __syncthreads();
        // 25 rows x 512 floats per tower, written as float4 (4 consecutive ci)
        for (int e = threadIdx.x; e < T * P2 * (K2 / 4); e += BLK) {
            const int t = e / (P2 * K2 / 4), r = e - t * (P2 * K2 / 4), p2 = r / (K2 / 4), k4 = r - p2 * (K2 / 4);
            const int tap = k4 >> 3, ci = (k4 & 7) * 4;
            const int oy = p2 / 5, ox = p2 - (p2 / 5) * 5, ky = tap >> 2, kx = tap & 3;
            const int pos = (2 * oy + ky) * 13 + (2 * ox + kx);
            out[((size_t)t * n + s) * (P2 * K2 / 4) + (size_t)p2 * (K2 / 4) + k4] =
                *reinterpret_cast<const float4 *>(a1 + (t * NPOS1 + pos) * C1 + ci);
        }
    }
}

// Backward of A2 = im2col(relu(conv1)) w.r.t. the tables and the bias:
//   dz1[t][ci][pos] = [z1 > 0] * sum_{(p2, tap) covering pos} dA2[t][s*25+p2][tap*32+ci]
//   dP[t][ci][slot][bin] += dz1 over the positions whose slot quarter falls in bin
// One wave per sample, lane = (tower, channel) = 64 lanes.  The lane walks the sample's
// 25 x 16 (p2, tap) gradient entries (each wave load = two 128-B rows, one per tower),
// tests the ReLU mask from 169 mask bits it computed once from the tables, and adds
// every entry into the 4 slot bins of its conv1 position.  The quarter index of each
// slot depends only on the tap's parity (static in the unrolled tap loop); the class is
// a 5-way select.  80 register bins per lane live across the wave's whole sample range.
constexpr int BWD_WAVES = 4;
__global__ __launch_bounds__(64 * BWD_WAVES, 2) void k_conv1_im2col_bwd(
    const uint32_t *__restrict__ codes, const int64_t *__restrict__ index, int64_t n,
    const float *__restrict__ tables, const float *__restrict__ bias, const float *__restrict__ dA, int T,
    float *__restrict__ slabs) {
    __shared__ float tab[MAXT * TAB];
    __shared__ float sb[MAXT * C1];
    __shared__ uint32_t bins_all[BWD_WAVES][NPOS1];
    __shared__ float red[64 * (NSLOT * NBIN + 1)];  // block fold of the 4 waves' bins
    stage_tables(tables, bias, T, tab, sb);
    for (int k = threadIdx.x; k < 64 * (NSLOT * NBIN + 1); k += blockDim.x) red[k] = 0.0f;
    __syncthreads();
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int t = lane >> 5, ci = lane & 31;
    const bool live = t < T;
    uint32_t *bins = bins_all[wv];
    float acc[NSLOT][4][4];  // [slot][class 1..4][parity group]; class 0 = group total - rest
    float tot[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int sl = 0; sl < NSLOT; sl++)
#pragma unroll
        for (int c = 0; c < 4; c++)
#pragma unroll
            for (int q = 0; q < 4; q++) acc[sl][c][q] = 0.0f;
    const int64_t gw = (int64_t)gridDim.x * BWD_WAVES;
    for (int64_t s = (int64_t)blockIdx.x * BWD_WAVES + wv; s < n; s += gw) {
        uint32_t w[8];
        load_codes(codes, index ? index[s] : s, w);
        // this wave's tile classes of the 4 slot quarters of the 169 positions (wave-private LDS)
        for (int p = lane; p < NPOS1; p += 64) {
            const int oy = p / 13, ox = p - (p / 13) * 13;
            uint32_t packed = 0u;
#pragma unroll
            for (int dy = 0; dy < 2; dy++)
#pragma unroll
                for (int dx = 0; dx < 2; dx++) {
                    const int qr = oy + dy, qc = ox + dx, cell = (qr >> 1) * 7 + (qc >> 1);
                    const uint32_t cls = (w[cell >> 3] >> ((cell & 7) * 4)) & 0xfu;
                    packed |= cls << (8 * (dy * 2 + dx));
                }
            bins[p] = packed;  // 4 x u8 classes (slot order)
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's own LDS writes are visible
        if (!live) continue;
        const float *tt = tab + t * NSLOT * NBIN * C1 + ci;
        const float b0 = sb[t * C1 + ci];
        const float *g = dA + ((size_t)t * n + s) * (P2 * K2) + ci;
        // positions in 4 parity groups (py, px): the taps covering a position and each slot's
        // quarter index are then compile-time constants
#pragma unroll
        for (int py = 0; py < 2; py++)
#pragma unroll
            for (int px = 0; px < 2; px++) {
                const int grp = py * 2 + px;
                for (int y = py; y < 13; y += 2)
                    for (int x = px; x < 13; x += 2) {
                        const int pos = y * 13 + x;
                        const uint32_t c4 = bins[pos];
                        // z1 > 0 ?  (ReLU mask, recomputed from the tables)
                        float z = b0;
#pragma unroll
                        for (int sl = 0; sl < 4; sl++) {
                            const int q = ((py + (sl >> 1)) & 1) * 2 + ((px + (sl & 1)) & 1);
                            z += tt[(sl * NBIN + (int)((c4 >> (8 * sl)) & 0xff) * 4 + q) * C1];
                        }
                        // col2im: taps ky in {py, py+2}, kx in {px, px+2}
                        float d = 0.0f;
#pragma unroll
                        for (int a = 0; a < 2; a++) {
                            const int ky = py + 2 * a, oy = (y - ky) >> 1;
                            if (y < ky || oy > 4) continue;
#pragma unroll
                            for (int b = 0; b < 2; b++) {
                                const int kx = px + 2 * b, ox = (x - kx) >> 1;
                                if (x < kx || ox > 4) continue;
                                d += g[(oy * 5 + ox) * K2 + (ky * 4 + kx) * C1];
                            }
                        }
                        d = z > 0.0f ? d : 0.0f;
                        tot[grp] += d;
#pragma unroll
                        for (int sl = 0; sl < 4; sl++) {
                            const uint32_t cls = (c4 >> (8 * sl)) & 0xff;
#pragma unroll
                            for (int c = 1; c < 5; c++) acc[sl][c - 1][grp] += (cls == (uint32_t)c) ? d : 0.0f;
                        }
                    }
            }
    }
    // fold the block's waves, then one slab per block
    if (live) {
        float *r = red + lane * (NSLOT * NBIN + 1);
#pragma unroll
        for (int sl = 0; sl < NSLOT; sl++)
#pragma unroll
            for (int grp = 0; grp < 4; grp++) {
                const int q = (((grp >> 1) + (sl >> 1)) & 1) * 2 + (((grp & 1) + (sl & 1)) & 1);
                float rest = 0.0f;
#pragma unroll
                for (int c = 1; c < 5; c++) {
                    atomicAdd(r + sl * NBIN + c * 4 + q, acc[sl][c - 1][grp]);
                    rest += acc[sl][c - 1][grp];
                }
                atomicAdd(r + sl * NBIN + q, tot[grp] - rest);
            }
        atomicAdd(r + NSLOT * NBIN, (tot[0] + tot[1]) + (tot[2] + tot[3]));
    }
    __syncthreads();
    float *dst = slabs + (size_t)blockIdx.x * T * SLAB;  // lane order t*32 + co == slab order
    for (int k = threadIdx.x; k < T * SLAB; k += blockDim.x) dst[k] = red[k];
}

__global__ __launch_bounds__(256) void k_slab_reduce(const float *__restrict__ slabs, int nslab, int T,
                                                     float *__restrict__ dtables, float *__restrict__ dbias) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= T * SLAB) return;
    float acc = 0.0f;
    for (int b = 0; b < nslab; b++) acc += slabs[(size_t)b * T * SLAB + k];
    const int t = k / SLAB, r = k - t * SLAB, co = r / (NSLOT * NBIN + 1), e = r - co * (NSLOT * NBIN + 1);
    if (e == NSLOT * NBIN)
        dbias[t * C1 + co] = acc;
    else
        dtables[(size_t)t * TAB + co * NSLOT * NBIN + e] = acc;
}

// ---------------------------------------------------------------------------
// A3[t][s*9 + p3][(ky*3 + kx)*64 + ci] = relu(Z2[t][s*25 + (oy+ky)*5 + ox+kx][ci] + b2[t][ci])
// one (tower, sample) per block iteration: 9 rows x 144 float4 out, 25 x 16 float4 in (L1-resident)
__global__ __launch_bounds__(BLK) void k_im2col3_fwd(const float4 *__restrict__ Z2, const float *__restrict__ b2,
                                                     int64_t n, int T, float4 *__restrict__ A3) {
    for (int64_t ts = blockIdx.x; ts < (int64_t)T * n; ts += gridDim.x) {
        const int t = (int)(ts / n);
        const float4 *z = Z2 + ts * (P2 * C2 / 4);
        float4 *o = A3 + ts * (P3 * K3 / 4);
        const float4 *bb = reinterpret_cast<const float4 *>(b2 + t * C2);
        for (int e = threadIdx.x; e < P3 * K3 / 4; e += BLK) {
            const int p3 = e / (K3 / 4), k4 = e - p3 * (K3 / 4), tap = k4 >> 4, ci4 = k4 & 15;
            const int oy = p3 / 3, ox = p3 - (p3 / 3) * 3, ky = tap / 3, kx = tap - (tap / 3) * 3;
            const float4 v = z[((oy + ky) * 5 + (ox + kx)) * (C2 / 4) + ci4];
            const float4 b = bb[ci4];
            o[e] = make_float4(fmaxf(v.x + b.x, 0.0f), fmaxf(v.y + b.y, 0.0f), fmaxf(v.z + b.z, 0.0f),
                               fmaxf(v.w + b.w, 0.0f));
        }
    }
}

// dZ2[t][s*25+p2][ci] = [Z2 + b2 > 0] * sum_{(p3, tap) covering p2} dA3[t][s*9+p3][tap*64+ci]
__global__ __launch_bounds__(BLK) void k_col2im3_bwd(const float4 *__restrict__ dA3, const float4 *__restrict__ Z2,
                                                     const float *__restrict__ b2, int64_t n, int T,
                                                     float4 *__restrict__ dZ2) {
    for (int64_t ts = blockIdx.x; ts < (int64_t)T * n; ts += gridDim.x) {
        const int t = (int)(ts / n);
        const float4 *base = dA3 + ts * (P3 * K3 / 4);
        const float4 *bb = reinterpret_cast<const float4 *>(b2 + t * C2);
        for (int e = threadIdx.x; e < P2 * C2 / 4; e += BLK) {
            const int p2 = e >> 4, ci4 = e & 15, y = p2 / 5, x = p2 - (p2 / 5) * 5;
            float4 g = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            for (int oy = max(0, y - 2); oy <= min(2, y); oy++)
                for (int ox = max(0, x - 2); ox <= min(2, x); ox++) {
                    const int tap = (y - oy) * 3 + (x - ox);
                    const float4 v = base[(oy * 3 + ox) * (K3 / 4) + tap * (C2 / 4) + ci4];
                    g.x += v.x;
                    g.y += v.y;
                    g.z += v.z;
                    g.w += v.w;
                }
            const float4 z = Z2[ts * (P2 * C2 / 4) + e];
            const float4 b = bb[ci4];
            dZ2[ts * (P2 * C2 / 4) + e] =
                make_float4(z.x + b.x > 0.0f ? g.x : 0.0f, z.y + b.y > 0.0f ? g.y : 0.0f,
                            z.z + b.z > 0.0f ? g.z : 0.0f, z.w + b.w > 0.0f ? g.w : 0.0f);
        }
    }
}

// Same map, written chunk-major dZ2c[t][ci/4][s*25+p2][ci%4] (the conv2 table histogram's
// input), raising *absmax (float bits) to max |dZ2| (the histogram's fixed-point scale).
// A block takes CF consecutive frames of one tower: their dA3 rows (CF x 20.7 KB) are staged
// in LDS with coalesced loads, and each 4-channel chunk's CF x 25 outputs are one contiguous
// run of the destination.
constexpr int CF = 2;
__global__ __launch_bounds__(BLK) void k_col2im3_bwd_chunked(const float4 *__restrict__ dA3,
                                                             const float4 *__restrict__ Z2,
                                                             const float *__restrict__ b2, int64_t n, int T,
                                                             float4 *__restrict__ dZ2c,
                                                             uint32_t *__restrict__ absmax) {
    __shared__ float4 tile[CF * P3 * K3 / 4];
    float amax = 0.0f;
    const int64_t groups = (n + CF - 1) / CF;
    for (int64_t tg = blockIdx.x; tg < (int64_t)T * groups; tg += gridDim.x) {
        const int t = (int)(tg / groups);
        const int64_t s0 = (tg - (int64_t)t * groups) * CF;
        const int nf = (int)std::min<int64_t>(CF, n - s0);
        const float4 *src = dA3 + ((size_t)t * n + s0) * (P3 * K3 / 4);
        __syncthreads();  // previous group's tile consumed
        for (int e = threadIdx.x; e < nf * (P3 * K3 / 4); e += BLK) tile[e] = src[e];
        __syncthreads();
        const float4 *bb = reinterpret_cast<const float4 *>(b2 + t * C2);
        for (int e = threadIdx.x; e < 16 * nf * P2; e += BLK) {
            const int ci4 = e / (nf * P2), r = e - ci4 * (nf * P2), f = r / P2, p2 = r - f * P2;
            const int y = p2 / 5, x = p2 - (p2 / 5) * 5;
            const float4 *tf = tile + f * (P3 * K3 / 4);
            float4 g = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            for (int oy = max(0, y - 2); oy <= min(2, y); oy++)
                for (int ox = max(0, x - 2); ox <= min(2, x); ox++) {
                    const int tap = (y - oy) * 3 + (x - ox);
                    const float4 v = tf[(oy * 3 + ox) * (K3 / 4) + tap * (C2 / 4) + ci4];
                    g.x += v.x;
                    g.y += v.y;
                    g.z += v.z;
                    g.w += v.w;
                }
            const float4 z = Z2[((size_t)t * n + s0 + f) * (P2 * C2 / 4) + p2 * 16 + ci4];
            const float4 b = bb[ci4];
            const float4 d = make_float4(z.x + b.x > 0.0f ? g.x : 0.0f, z.y + b.y > 0.0f ? g.y : 0.0f,
                                         z.z + b.z > 0.0f ? g.z : 0.0f, z.w + b.w > 0.0f ? g.w : 0.0f);
            dZ2c[(((size_t)t * 16 + ci4) * n + s0 + f) * P2 + p2] = d;
            amax = fmaxf(amax, fmaxf(fmaxf(fabsf(d.x), fabsf(d.y)), fmaxf(fabsf(d.z), fabsf(d.w))));
        }
    }
    // NaN/inf propagate as a non-finite max (the histogram then returns NaN)
    for (int off = 32; off > 0; off >>= 1) amax = fmaxf(amax, __shfl_xor(amax, off));
    if (amax != amax) amax = __int_as_float(0x7f800000);
    // skip the same-address atomic when the word already holds at least this wave's max (it only grows)
    if ((threadIdx.x & 63) == 0 &&
        __float_as_uint(amax) > __hip_atomic_load(absmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        atomicMax(absmax, __float_as_uint(amax));
}

int grid_cap(int64_t rows) { return (int)std::max<int64_t>(1, std::min<int64_t>(rows, 256 * 16)); }

}  // namespace

hipError_t launch_conv1_im2col_fwd(const uint32_t *codes, const int64_t *index, int64_t n, const float *tables,
                                   const float *bias, int T, float *A2, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int grid = (int)std::min<int64_t>(n, 256 * 4);
    hipLaunchKernelGGL(k_conv1_im2col_fwd, dim3(grid), dim3(BLK), 0, s, codes, index, n, tables, bias, T,
                       reinterpret_cast<float4 *>(A2));
    return hipGetLastError();
}

hipError_t launch_conv1_im2col_bwd(const uint32_t *codes, const int64_t *index, int64_t n, const float *tables,
                                   const float *bias, const float *dA2, int T, float *dtables, float *dbias,
                                   float *slabs, int max_slabs, hipStream_t s) {
    if (n <= 0) {
        hipError_t e = zero_async(dtables, sizeof(float) * T * TAB, s);
        return e == hipSuccess ? zero_async(dbias, sizeof(float) * T * C1, s) : e;
    }
    const int grid = (int)std::min<int64_t>((n + BWD_WAVES - 1) / BWD_WAVES, (int64_t)max_slabs);
    hipLaunchKernelGGL(k_conv1_im2col_bwd, dim3(grid), dim3(64 * BWD_WAVES), 0, s, codes, index, n, tables, bias,
                       dA2, T, slabs);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_slab_reduce, dim3((T * SLAB + 255) / 256), dim3(256), 0, s, slabs, grid, T, dtables,
                       dbias);
    return hipGetLastError();
}

hipError_t launch_im2col3_fwd(const float *Z2, const float *b2, int64_t n, int T, float *A3, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_im2col3_fwd, dim3(grid_cap((int64_t)T * n)), dim3(BLK), 0, s,
                       reinterpret_cast<const float4 *>(Z2), b2, n, T, reinterpret_cast<float4 *>(A3));
    return hipGetLastError();
}

hipError_t launch_col2im3_bwd(const float *dA3, const float *Z2, const float *b2, int64_t n, int T, int chunked,
                              float *dZ2, uint32_t *absmax, hipStream_t s) {
    if (chunked) {
        hipError_t e = zero_async(absmax, sizeof(uint32_t), s);
        if (e != hipSuccess || n <= 0) return e;
        const int64_t groups = (n + CF - 1) / CF;
        hipLaunchKernelGGL(k_col2im3_bwd_chunked, dim3(grid_cap((int64_t)T * groups)), dim3(BLK), 0, s,
                           reinterpret_cast<const float4 *>(dA3), reinterpret_cast<const float4 *>(Z2), b2, n,
                           T, reinterpret_cast<float4 *>(dZ2), absmax);
        return hipGetLastError();
    }
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_col2im3_bwd, dim3(grid_cap((int64_t)T * n)), dim3(BLK), 0, s,
                       reinterpret_cast<const float4 *>(dA3), reinterpret_cast<const float4 *>(Z2), b2, n, T,
                       reinterpret_cast<float4 *>(dZ2));
    return hipGetLastError();
}

}  // namespace merlin
