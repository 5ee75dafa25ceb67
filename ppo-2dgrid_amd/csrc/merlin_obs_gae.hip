// merlin_obs_gae.hip -- observation expansion and GAE / advantage normalisation.
//
// obs expansion: 7x7 tile-class nibbles -> the 56x56x3 RGBImgPartialObsWrapper
// frame (Grid.render blit, tile (i,j) -> img[8j:8j+8, 8i:8i+8]).  Write-bound:
// 32 B of codes in, 37,632 B (f32) or 9,408 B (u8) out per observation; every
// thread emits one 16-B float4 (4 pixels of one channel row, always inside one
// tile) from an LDS copy of the 5-tile atlas, so stores are fully coalesced.
//
// GAE: PPO.compute_gae (src/ppo.py:107-120) on [T][N]; per-env backward affine
// recurrence in the reference's fp32 op order (compiled with -ffp-contract=off):
//   delta = (r + (gamma*nv)*mask) - v,  gae = delta + ((gamma*lam)*mask)*gae
// Large N: one thread per env (coalesced [t][i] rows, loads software-pipelined).
// Small N (FOMAML single-env task rollouts): one wave per env, the T-long
// recurrence split into 64 chunks whose affine maps (A,B) are composed with a
// wavefront shuffle scan, then each lane replays its chunk sequentially.
#include "merlin_internal.h"

namespace merlin {
namespace {

__constant__ uint8_t c_atlas[MERLIN_OBS_TILES * 8 * 8 * 3];  // [tile][y][x][c]

constexpr int OBS_F4 = 3 * 56 * 14;  // float4 per NCHW observation (9408 floats)

__device__ __forceinline__ uint32_t tile_code(const uint32_t *__restrict__ codes, int64_t row,
                                              int cell) {
    const uint32_t w = codes[row * MERLIN_OBS_WORDS + (cell >> 3)];
    return (w >> ((cell & 7) * 4)) & 0xfu;
}

__global__ __launch_bounds__(256) void k_obs_expand_nchw(const uint32_t *__restrict__ codes,
                                                         const int64_t *__restrict__ index,
                                                         int64_t n, float4 *__restrict__ out,
                                                         float scale) {
    // LDS atlas as [tile][c][y][half] float4 (4 consecutive x of one channel row)
    __shared__ float4 atlas4[MERLIN_OBS_TILES * 3 * 8 * 2];
    for (int k = threadIdx.x; k < MERLIN_OBS_TILES * 3 * 8 * 2; k += blockDim.x) {
        const int h = k & 1, y = (k >> 1) & 7, c = (k >> 4) % 3, t = (k >> 4) / 3;
        const uint8_t *src = c_atlas + ((t * 8 + y) * 8 + h * 4) * 3 + c;
        atlas4[k] = make_float4((float)src[0] * scale, (float)src[3] * scale, (float)src[6] * scale,
                                (float)src[9] * scale);
    }
    __syncthreads();
    const int64_t total = n * OBS_F4;
    for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < total;
         f += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = f / OBS_F4;
        const int r = (int)(f - s * OBS_F4);
        const int c = r / 784;
        const int r2 = r - c * 784;
        const int y = r2 / 14;
        const int xq = r2 - y * 14;
        const int64_t src = index ? index[s] : s;
        const uint32_t code = tile_code(codes, src, (y >> 3) * 7 + (xq >> 1));
        out[f] = atlas4[((code * 3 + c) * 8 + (y & 7)) * 2 + (xq & 1)];
    }
}

__global__ __launch_bounds__(256) void k_obs_expand_nhwc_f32(const uint32_t *__restrict__ codes,
                                                             const int64_t *__restrict__ index,
                                                             int64_t n, float *__restrict__ out,
                                                             float scale) {
    const int64_t total = n * 9408;
    for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < total;
         f += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = f / 9408;
        const int o = (int)(f - s * 9408);
        const int y = o / 168, rem = o - y * 168, x = rem / 3, c = rem - x * 3;
        const int64_t src = index ? index[s] : s;
        const uint32_t code = tile_code(codes, src, (y >> 3) * 7 + (x >> 3));
        out[f] = (float)c_atlas[((code * 8 + (y & 7)) * 8 + (x & 7)) * 3 + c] * scale;
    }
}

__global__ __launch_bounds__(256) void k_obs_expand_u8(const uint32_t *__restrict__ codes,
                                                       const int64_t *__restrict__ index, int64_t n,
                                                       uint32_t *__restrict__ out) {
    const int64_t total = n * (9408 / 4);
    for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < total;
         f += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = f / 2352;
        const int o0 = (int)(f - s * 2352) * 4;
        const int64_t src = index ? index[s] : s;
        uint32_t word = 0u;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int o = o0 + b;
            const int y = o / 168, rem = o - y * 168, x = rem / 3, c = rem - x * 3;
            const uint32_t code = tile_code(codes, src, (y >> 3) * 7 + (x >> 3));
            word |= (uint32_t)c_atlas[((code * 8 + (y & 7)) * 8 + (x & 7)) * 3 + c] << (8 * b);
        }
        out[f] = word;
    }
}

int grid_for(int64_t work, int block) {
    int64_t g = (work + block - 1) / block;
    const int64_t cap = 256 * 16;  // 256 CUs x 16 blocks, grid-stride beyond
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (int)g;
}

// ---------------------------------------------------------------------------
// GAE
constexpr int GAE_BLK = 256;

__device__ __forceinline__ void block_reduce2(double &a, double &b, double *sh) {
    for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_down(a, o, 64);
        b += __shfl_down(b, o, 64);
    }
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (l == 0) {
        sh[2 * w] = a;
        sh[2 * w + 1] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const int nw = (blockDim.x + 63) >> 6;
        a = 0.0;
        b = 0.0;
        for (int k = 0; k < nw; k++) {
            a += sh[2 * k];
            b += sh[2 * k + 1];
        }
    }
}

// one thread per env
__global__ __launch_bounds__(GAE_BLK) void k_gae_thread(
    const float *__restrict__ rew, const float *__restrict__ val, const float *__restrict__ done,
    const float *__restrict__ last, float *__restrict__ adv, float *__restrict__ ret, int T, int N,
    float gf, float glf, double gamma, double *__restrict__ partials) {
    __shared__ double sh[2 * (GAE_BLK / 64)];
    const int i = blockIdx.x * GAE_BLK + threadIdx.x;
    double s1 = 0.0, s2 = 0.0;
    if (i < N) {
        const size_t n = (size_t)N;
        // t = T-1: next value is the bootstrap last_value, a Python float in the reference:
        // gamma * last_value is a double product cast to f32
        float vnext = val[(size_t)(T - 1) * n + i];
        float gae;
        {
            const size_t k = (size_t)(T - 1) * n + i;
            const float mask = 1.0f - done[k];
            const float gn = (float)(gamma * (double)last[i]);
            const float delta = (rew[k] + gn * mask) - vnext;
            gae = delta + (glf * mask) * 0.0f;
            adv[k] = gae;
            ret[k] = vnext + gae;
            s1 += (double)gae;
            s2 += (double)gae * (double)gae;
        }
        constexpr int U = 8;
        int t = T - 2;
        for (; t >= U - 1; t -= U) {  // software pipeline: issue U rows of loads, then the chain
            float r[U], v[U], d[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const size_t k = (size_t)(t - u) * n + i;
                r[u] = rew[k];
                v[u] = val[k];
                d[u] = done[k];
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                const size_t k = (size_t)(t - u) * n + i;
                const float mask = 1.0f - d[u];
                const float delta = (r[u] + (gf * vnext) * mask) - v[u];
                gae = delta + (glf * mask) * gae;
                adv[k] = gae;
                ret[k] = v[u] + gae;
                s1 += (double)gae;
                s2 += (double)gae * (double)gae;
                vnext = v[u];
            }
        }
        for (; t >= 0; t--) {
            const size_t k = (size_t)t * n + i;
            const float v = val[k];
            const float mask = 1.0f - done[k];
            const float delta = (rew[k] + (gf * vnext) * mask) - v;
            gae = delta + (glf * mask) * gae;
            adv[k] = gae;
            ret[k] = v + gae;
            s1 += (double)gae;
            s2 += (double)gae * (double)gae;
            vnext = v;
        }
    }
    if (partials) {
        block_reduce2(s1, s2, sh);
        if (threadIdx.x == 0) {
            partials[2 * blockIdx.x] = s1;
            partials[2 * blockIdx.x + 1] = s2;
        }
    }
}

// one wave per env: chunked affine scan across the 64 lanes
__global__ __launch_bounds__(64) void k_gae_wave(const float *__restrict__ rew,
                                                 const float *__restrict__ val,
                                                 const float *__restrict__ done,
                                                 const float *__restrict__ last,
                                                 float *__restrict__ adv, float *__restrict__ ret,
                                                 int T, int N, float gf, float glf, double gamma,
                                                 double *__restrict__ partials) {
    const int i = blockIdx.x;
    const int lane = threadIdx.x;
    const size_t n = (size_t)N;
    const int L = (T + 63) / 64;
    const int t0 = min(lane * L, T), t1 = min(t0 + L, T);
    // g_{t0} = B + A * g_{t1}
    float A = 1.0f, B = 0.0f;
    for (int t = t1 - 1; t >= t0; t--) {
        const size_t k = (size_t)t * n + i;
        const float mask = 1.0f - done[k];
        const float gn = (t == T - 1) ? (float)(gamma * (double)last[i]) : gf * val[k + n];
        const float delta = (rew[k] + gn * mask) - val[k];
        const float c = glf * mask;
        B = delta + c * B;
        A = c * A;
    }
    // inclusive suffix scan over lanes: (A,B)_l o (A,B)_{l+1} o ...
    float SA = A, SB = B;
    for (int o = 1; o < 64; o <<= 1) {
        const float nA = __shfl_down(SA, o, 64);
        const float nB = __shfl_down(SB, o, 64);
        if (lane + o < 64) {
            SB = SB + SA * nB;
            SA = SA * nA;
        }
    }
    // g entering this chunk from the right = suffix map of lane+1 applied to g_T = 0
    float gin = __shfl_down(SB, 1, 64);
    if (lane == 63) gin = 0.0f;
    double s1 = 0.0, s2 = 0.0;
    float gae = gin;
    for (int t = t1 - 1; t >= t0; t--) {
        const size_t k = (size_t)t * n + i;
        const float mask = 1.0f - done[k];
        const float v = val[k];
        const float gn = (t == T - 1) ? (float)(gamma * (double)last[i]) : gf * val[k + n];
        const float delta = (rew[k] + gn * mask) - v;
        gae = delta + (glf * mask) * gae;
        adv[k] = gae;
        ret[k] = v + gae;
        s1 += (double)gae;
        s2 += (double)gae * (double)gae;
    }
    if (partials) {
        for (int o = 32; o > 0; o >>= 1) {
            s1 += __shfl_down(s1, o, 64);
            s2 += __shfl_down(s2, o, 64);
        }
        if (lane == 0) {
            partials[2 * i] = s1;
            partials[2 * i + 1] = s2;
        }
    }
}

__global__ void k_reduce_partials(const double *__restrict__ partials, int np, double count,
                                  double *__restrict__ stats) {
    // fixed-order serial sum: deterministic; np is at most a few hundred
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        double a = 0.0, b = 0.0;
        for (int k = 0; k < np; k++) {
            a += partials[2 * k];
            b += partials[2 * k + 1];
        }
        stats[0] = count;
        stats[1] = a;
        stats[2] = b;
    }
}

__global__ __launch_bounds__(256) void k_adv_normalize(const float *adv, int64_t n,
                                                       const double *__restrict__ stats,
                                                       float *out) {
    const double cnt = stats[0];
    const double mean = stats[1] / cnt;
    double var = (stats[2] - stats[1] * mean) / (cnt - 1.0);
    if (var < 0.0) var = 0.0;
    const float mf = (float)mean;
    const float denom = (float)sqrt(var) + 1e-8f;  // adv.std() + 1e-8 in f32
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
         k += (int64_t)gridDim.x * blockDim.x)
        out[k] = (adv[k] - mf) / denom;
}

constexpr int WAVE_GAE_MAX_N = 256;

}  // namespace

hipError_t upload_atlas(const uint8_t *atlas_host) {
    return hipMemcpyToSymbol(HIP_SYMBOL(c_atlas), atlas_host, sizeof(c_atlas), 0,
                             hipMemcpyHostToDevice);
}

hipError_t launch_obs_expand_f32(const uint32_t *codes, const int64_t *index, int64_t n, float *out,
                                 float scale, int layout, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if (layout == MERLIN_LAYOUT_NCHW)
        hipLaunchKernelGGL(k_obs_expand_nchw, dim3(grid_for(n * OBS_F4, 256)), dim3(256), 0, s, codes,
                           index, n, reinterpret_cast<float4 *>(out), scale);
    else
        hipLaunchKernelGGL(k_obs_expand_nhwc_f32, dim3(grid_for(n * 9408, 256)), dim3(256), 0, s,
                           codes, index, n, out, scale);
    return hipGetLastError();
}

hipError_t launch_obs_expand_u8(const uint32_t *codes, const int64_t *index, int64_t n, uint8_t *out,
                                hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_obs_expand_u8, dim3(grid_for(n * 2352, 256)), dim3(256), 0, s, codes, index,
                       n, reinterpret_cast<uint32_t *>(out));
    return hipGetLastError();
}

int gae_partials_needed(int T, int N) {
    (void)T;
    return N <= WAVE_GAE_MAX_N ? N : (N + GAE_BLK - 1) / GAE_BLK;
}

hipError_t launch_gae(const float *rew, const float *val, const float *done, const float *last,
                      float *adv, float *ret, int T, int N, double gamma, double lam, double *stats,
                      double *partials, int max_partials, hipStream_t s) {
    const float gf = (float)gamma;
    const float glf = (float)(gamma * lam);  // Python float product, cast when it meets the f32 mask
    const int np = gae_partials_needed(T, N);
    double *p = (stats && np <= max_partials) ? partials : nullptr;
    if (stats && !p) return hipErrorInvalidValue;
    if (N <= WAVE_GAE_MAX_N)
        hipLaunchKernelGGL(k_gae_wave, dim3(N), dim3(64), 0, s, rew, val, done, last, adv, ret, T, N,
                           gf, glf, gamma, p);
    else
        hipLaunchKernelGGL(k_gae_thread, dim3((N + GAE_BLK - 1) / GAE_BLK), dim3(GAE_BLK), 0, s, rew,
                           val, done, last, adv, ret, T, N, gf, glf, gamma, p);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !stats) return e;
    hipLaunchKernelGGL(k_reduce_partials, dim3(1), dim3(64), 0, s, p, np, (double)T * (double)N,
                       stats);
    return hipGetLastError();
}

hipError_t launch_adv_normalize(const float *adv, int64_t n, const double *stats, float *out,
                                hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_adv_normalize, dim3(grid_for(n, 256)), dim3(256), 0, s, adv, n, stats, out);
    return hipGetLastError();
}

}  // namespace merlin
