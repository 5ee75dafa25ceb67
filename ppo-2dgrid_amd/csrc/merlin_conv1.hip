// merlin_conv1.hip -- the CNN's first convolution computed from tile codes.
//
// CNNFeatureExtractor's conv1 (src/actor_critic.py:9-10: Conv2d(3, 32, k=8, s=4) on the
// 56x56 RGB frame / 255) only ever sees frames blitted from the 5 tiles of the
// minigrid atlas (7x7 tiles of 8x8 px).  An 8x8 window at stride 4 covers exactly
// 2x2 "quarter tiles" (4x4 px): window (oy, ox) covers quarter cells (oy+dy, ox+dx),
// dy,dx in {0,1}; quarter cell (qr, qc) is quarter (qr&1, qc&1) of tile
// (qr>>1, qc>>1).  Hence, exactly (up to fp32 summation order):
//   z1[co](oy,ox) = b[co] + sum_{slot=(dy,dx)} P[co][slot][cls*4 + q]
//   P[co][slot][cls*4+q] = sum_{c,ky,kx<4} W1[co][c][4dy+ky][4dx+kx] * A[cls][c][4qy+ky][4qx+kx]/255
// with cls = class of the tile under that quarter cell and q = its quarter index.
// P (2,560 floats per tower) is built from W1 by a tiny einsum on the host side of the
// autograd graph; these kernels do the lookups (forward, ReLU fused) and the
// transposed histogram (backward):  dP[co][slot][bin] = sum over (n, oy, ox) whose
// slot-quarter falls in `bin` of dz = da1 * (a1 > 0);  db[co] = sum dz.
// This replaces 1.04 MMAC per sample per tower in the forward and the same again in the
// weight gradient by 4 table reads per output, and the frame expansion entirely.
#include "merlin_internal.h"

namespace merlin {
namespace {

constexpr int C1 = 32;                 // conv1 output channels per tower
constexpr int NPOS = 169;              // 13 x 13 output positions
constexpr int NBIN = 20;               // 5 classes x 4 quarters
constexpr int TAB = C1 * 4 * NBIN;     // table floats per tower: [co][slot][bin]
constexpr int THREADS = 192;           // 3 waves: one thread per output position (169 live)
constexpr int MAXT = 2;                // towers (actor, critic)

__device__ __forceinline__ uint32_t nib(const uint32_t w[8], int cell) {
    return (w[cell >> 3] >> ((cell & 7) * 4)) & 0xfu;
}

// bins of output position p for the 4 slots: slot*20 + cls*4 + q
__device__ __forceinline__ void slot_bins(const uint32_t w[8], int oy, int ox, int b[4]) {
#pragma unroll
    for (int dy = 0; dy < 2; dy++)
#pragma unroll
        for (int dx = 0; dx < 2; dx++) {
            const int qr = oy + dy, qc = ox + dx;
            const uint32_t cls = nib(w, (qr >> 1) * 7 + (qc >> 1));
            const int slot = dy * 2 + dx;
            b[slot] = slot * NBIN + (int)cls * 4 + (qr & 1) * 2 + (qc & 1);
        }
}

__device__ __forceinline__ void load_codes(const uint32_t *__restrict__ codes, int64_t row, uint32_t w[8]) {
    const uint4 *c = reinterpret_cast<const uint4 *>(codes + row * MERLIN_OBS_WORDS);
    const uint4 a = c[0], b = c[1];
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
    w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}

// out[t][s][co][p] = relu(b[t][co] + sum_slot P[t][co][slot][bin_slot(p)])
__global__ __launch_bounds__(THREADS) void k_conv1_lut_fwd(const uint32_t *__restrict__ codes,
                                                           const int64_t *__restrict__ index, int64_t n,
                                                           const float *__restrict__ tables,
                                                           const float *__restrict__ bias, int T,
                                                           float *__restrict__ out) {
    __shared__ float tab[MAXT * TAB];
    __shared__ float sb[MAXT * C1];
    for (int k = threadIdx.x; k < T * TAB; k += THREADS) tab[k] = tables[k];
    for (int k = threadIdx.x; k < T * C1; k += THREADS) sb[k] = bias[k];
    __syncthreads();
    const int p = threadIdx.x;
    if (p >= NPOS) return;
    const int oy = p / 13, ox = p - (p / 13) * 13;
    for (int64_t s = blockIdx.x; s < n; s += gridDim.x) {
        uint32_t w[8];
        load_codes(codes, index ? index[s] : s, w);
        int b[4];
        slot_bins(w, oy, ox, b);
        for (int t = 0; t < T; t++) {
            float *o = out + ((size_t)t * n + s) * C1 * NPOS + p;
            const float *tt = tab + t * TAB;
#pragma unroll 8
            for (int co = 0; co < C1; co++) {
                const float *pc = tt + co * 4 * NBIN;
                const float z = (((sb[t * C1 + co] + pc[b[0]]) + pc[b[1]]) + pc[b[2]]) + pc[b[3]];
                o[(size_t)co * NPOS] = fmaxf(z, 0.0f);
            }
        }
    }
}

// Per block: dP/db partial slab over its samples.  Thread = output position p; for groups
// of 4 channels it accumulates dz into 4 slots x 5 classes x 4 channels registers (the
// quarter index q of each slot is fixed by p), then folds them into the block's LDS bins.
constexpr int CG = 4;
constexpr int SLAB = C1 * (4 * NBIN + 1);  // per tower: [co][80 bins + bias]

__global__ __launch_bounds__(THREADS) void k_conv1_lut_bwd(const uint32_t *__restrict__ codes,
                                                           const int64_t *__restrict__ index, int64_t n,
                                                           const float *__restrict__ act,
                                                           const float *__restrict__ grad, int T,
                                                           float *__restrict__ slabs) {
    __shared__ float bins[MAXT * SLAB];
    for (int k = threadIdx.x; k < T * SLAB; k += THREADS) bins[k] = 0.0f;
    __syncthreads();
    const int p = threadIdx.x;
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t s0 = (int64_t)blockIdx.x * per, s1 = min(n, s0 + per);
    if (p < NPOS) {
        const int oy = p / 13, ox = p - (p / 13) * 13;
        int qs[4];
#pragma unroll
        for (int dy = 0; dy < 2; dy++)
#pragma unroll
            for (int dx = 0; dx < 2; dx++) qs[dy * 2 + dx] = ((oy + dy) & 1) * 2 + ((ox + dx) & 1);
        for (int g = 0; g < T * C1; g += CG) {
            const int t = g / C1, co0 = g - t * C1;
            float acc[4][5][CG];
            float accb[CG];
#pragma unroll
            for (int j = 0; j < CG; j++) {
                accb[j] = 0.0f;
#pragma unroll
                for (int sl = 0; sl < 4; sl++)
#pragma unroll
                    for (int c = 0; c < 5; c++) acc[sl][c][j] = 0.0f;
            }
            for (int64_t s = s0; s < s1; s++) {
                uint32_t w[8];
                load_codes(codes, index ? index[s] : s, w);
                int cls[4];
#pragma unroll
                for (int dy = 0; dy < 2; dy++)
#pragma unroll
                    for (int dx = 0; dx < 2; dx++)
                        cls[dy * 2 + dx] = (int)nib(w, ((oy + dy) >> 1) * 7 + ((ox + dx) >> 1));
                const size_t base = (((size_t)t * n + s) * C1 + co0) * NPOS + p;
                float dz[CG];
#pragma unroll
                for (int j = 0; j < CG; j++) {
                    const float a = act[base + (size_t)j * NPOS];
                    const float gr = grad[base + (size_t)j * NPOS];
                    dz[j] = a > 0.0f ? gr : 0.0f;
                }
#pragma unroll
                for (int j = 0; j < CG; j++) {
                    accb[j] += dz[j];
#pragma unroll
                    for (int sl = 0; sl < 4; sl++)
#pragma unroll
                        for (int c = 0; c < 5; c++) acc[sl][c][j] += (cls[sl] == c) ? dz[j] : 0.0f;
                }
            }
#pragma unroll
            for (int j = 0; j < CG; j++) {
                float *bj = bins + t * SLAB + (co0 + j) * (4 * NBIN + 1);
                atomicAdd(bj + 4 * NBIN, accb[j]);
#pragma unroll
                for (int sl = 0; sl < 4; sl++)
#pragma unroll
                    for (int c = 0; c < 5; c++) atomicAdd(bj + sl * NBIN + c * 4 + qs[sl], acc[sl][c][j]);
            }
        }
    }
    __syncthreads();
    float *dst = slabs + (size_t)blockIdx.x * T * SLAB;
    for (int k = threadIdx.x; k < T * SLAB; k += THREADS) dst[k] = bins[k];
}

// fixed-order sum of the block slabs -> dtables [T][co][slot][bin], dbias [T][co]
__global__ __launch_bounds__(256) void k_conv1_lut_reduce(const float *__restrict__ slabs, int nslab, int T,
                                                          float *__restrict__ dtables,
                                                          float *__restrict__ dbias) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= T * SLAB) return;
    float acc = 0.0f;
    for (int b = 0; b < nslab; b++) acc += slabs[(size_t)b * T * SLAB + k];
    const int t = k / SLAB, r = k - t * SLAB, co = r / (4 * NBIN + 1), e = r - co * (4 * NBIN + 1);
    if (e == 4 * NBIN)
        dbias[t * C1 + co] = acc;
    else
        dtables[(size_t)t * TAB + co * 4 * NBIN + e] = acc;
}

}  // namespace

int conv1_slab_floats(int towers) { return towers * SLAB; }

hipError_t launch_conv1_lut_fwd(const uint32_t *codes, const int64_t *index, int64_t n, const float *tables,
                                const float *bias, int towers, float *out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int grid = (int)std::min<int64_t>(n, 256 * 8);
    hipLaunchKernelGGL(k_conv1_lut_fwd, dim3(grid), dim3(THREADS), 0, s, codes, index, n, tables, bias, towers,
                       out);
    return hipGetLastError();
}

hipError_t launch_conv1_lut_bwd(const uint32_t *codes, const int64_t *index, int64_t n, const float *act,
                                const float *grad, int towers, float *dtables, float *dbias, float *slabs,
                                int max_slabs, hipStream_t s) {
    if (n <= 0) {
        hipError_t e = zero_async(dtables, sizeof(float) * towers * TAB, s);
        if (e == hipSuccess) e = zero_async(dbias, sizeof(float) * towers * C1, s);
        return e;
    }
    const int grid = (int)std::min<int64_t>(n, (int64_t)max_slabs);
    hipLaunchKernelGGL(k_conv1_lut_bwd, dim3(grid), dim3(THREADS), 0, s, codes, index, n, act, grad, towers,
                       slabs);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int tot = towers * SLAB;
    hipLaunchKernelGGL(k_conv1_lut_reduce, dim3((tot + 255) / 256), dim3(256), 0, s, slabs, grid, towers, dtables,
                       dbias);
    return hipGetLastError();
}

}  // namespace merlin
