// merlin_group_act.hip -- FOMAML's acting step: one frame per task, each task with its own policy weights
// (src/fomaml.py:54-108 collect_trajectory: fast_policy.act(state) per step; src/actor_critic.py:48-56 act).
//
// The batched FOMAML rollout (merlin/fomaml.py) steps G tasks (G = tasks_per_batch = 32 at cfg 5) with G different
// weight sets, one env each.  Through the generic torch / library path a step was ~15 launches of a few threads'
// work each (grouped conv2 lookups over 2 blocks, im2col, 4 batched GEMMs, log-softmax, Gumbel draw, copies): ~180 us
// per step, latency-bound (profiles/r05a_fomaml_kernel_stats.md).  Here a step is two launches plus the fused draw
// + env step (merlin_env_act_step):
//
//   k_group_conv   one block per (task, tower): the frame's 49 tile classes -> conv1 + conv2 by the tower's
//                  2,720-row table T2 (16 rows per conv2 position, merlin_conv2lut.hip's row layout) + b2, ReLU
//                  -> conv3 (9 x 64 outputs, 576 MACs each; the 4 waves split the 576-long reduction, summed in
//                  wave order) + b3, ReLU -> a3 [tower][576] in fc1's (p3, co) column order
//   k_group_fc1    one block per (task, tower, 64-column chunk of fc1): h = relu(b4 + W4p a3) of its 64 columns
//                  (16 waves of 4 columns, lanes over k, a fixed xor tree), then the head dot products of those 64
//                  columns (actor: the task's A logits' weights, critic: its value weights) summed in wave order;
//                  chunk 0 adds the task's head biases -> part[tower][chunk][task][4], the partial-sum layout
//                  merlin_env_act_step / merlin_act_draw read (then called with zero biases)
//
// fp32 throughout (products and sums in fp32, as the reference's CPU/torch forward; different summation order).
#include <algorithm>

#include "merlin_internal.h"

namespace merlin {
namespace {

constexpr int GA_NROW = 2720, GA_H = 512, GA_K = 576;
// k_group_conv's waves: conv3's 576-long reduction is split over GC_W waves (36 k values each, all loads of a wave's
// W3 slice issued before its FMAs); with 4 waves (round 5) each lane walked 144 k values in 18 dependent load batches
// and the launch took ~19 us at 32 tasks (profiles/r05b_fomaml_kernel_stats.md)
constexpr int GC_W = 16, GC_T = 64 * GC_W, GC_KW = GA_K / GC_W;

__global__ __launch_bounds__(GC_T) void k_group_conv(const uint32_t *__restrict__ codes, const float4 *__restrict__ T2,
                                                    const float *__restrict__ b2, const float *__restrict__ W3t,
                                                    const float *__restrict__ b3, float *__restrict__ a3, int shared) {
    __shared__ uint8_t cls[52];
    __shared__ float4 a2[25][16];
    __shared__ float red[GC_W][9][64];
    const int tt = blockIdx.x, g = tt >> 1;  // tower tt = 2 g (actor) / 2 g + 1 (critic) of task g
    const int wt = shared ? (tt & 1) : tt;   // its weights' tower (one weight set for every task when shared)
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // conv3's weights first (they do not depend on the frame): their load round trip overlaps the frame -> T2 chain
    const float *w3 = W3t + (size_t)wt * GA_K * 64 + lane;
    const int k0 = wv * GC_KW;
    float wk[GC_KW];
#pragma unroll
    for (int u = 0; u < GC_KW; u++) wk[u] = w3[(size_t)(k0 + u) * 64];
    if (tid < 49) {
        const uint32_t word = codes[(size_t)g * MERLIN_OBS_WORDS + (tid >> 3)];
        cls[tid] = (uint8_t)min((word >> ((tid & 7) * 4)) & 0xfu, 4u);
    }
    __syncthreads();
    // conv2 + b2 + ReLU at the 25 positions (16 float4 columns each)
    const float4 *tab = T2 + (size_t)wt * GA_NROW * 16;
    for (int e = tid; e < 25 * 16; e += GC_T) {
        const int p = e >> 4, q = e & 15, py = p / 5, px = p - py * 5;
        int w[9];
#pragma unroll
        for (int a = 0; a < 3; a++)
#pragma unroll
            for (int b = 0; b < 3; b++) w[a * 3 + b] = cls[(py + a) * 7 + px + b];
        float4 v[16];
#pragma unroll
        for (int ky = 0; ky < 4; ky++)
#pragma unroll
            for (int kx = 0; kx < 4; kx++) {
                const int a = ky >> 1, b = kx >> 1, j = 2 * a + b, c00 = w[a * 3 + b];
                int row;
                if (!(ky & 1) && !(kx & 1))
                    row = 4 * c00 + j;
                else if (!(ky & 1))
                    row = 20 + 4 * (5 * c00 + w[a * 3 + b + 1]) + j;
                else if (!(kx & 1))
                    row = 120 + 4 * (5 * c00 + w[(a + 1) * 3 + b]) + j;
                else
                    row = 220 + 4 * (125 * c00 + 25 * w[a * 3 + b + 1] + 5 * w[(a + 1) * 3 + b] + w[(a + 1) * 3 + b + 1]) +
                          j;
                v[ky * 4 + kx] = tab[(size_t)row * 16 + q];
            }
        float4 s = v[0];
#pragma unroll
        for (int i = 1; i < 16; i++) {
            s.x += v[i].x;
            s.y += v[i].y;
            s.z += v[i].z;
            s.w += v[i].w;
        }
        const float *bb = b2 + (size_t)wt * 64 + q * 4;
        a2[p][q] = make_float4(fmaxf(s.x + bb[0], 0.0f), fmaxf(s.y + bb[1], 0.0f), fmaxf(s.z + bb[2], 0.0f),
                               fmaxf(s.w + bb[3], 0.0f));
    }
    __syncthreads();
    // conv3: lane = output channel co, wave wv takes k = tap * 64 + ci in [36 wv, 36 wv + 36) for all 9 positions
    // (its 36 weights loaded before the FMAs: one load round trip per wave)
    const float *a2f = reinterpret_cast<const float *>(&a2[0][0]);
    float acc[9];
#pragma unroll
    for (int p3 = 0; p3 < 9; p3++) acc[p3] = 0.0f;
    // four consecutive k (one tap, ci .. ci + 3: k0 and the tap boundaries are multiples of 4) per LDS read
    // (ds_read_b128 instead of 4 ds_read_b32: the phase was LDS-issue-bound), each position's products added in
    // the same order as one k at a time -- the same bits
    static_assert(GC_KW % 4 == 0, "k in groups of 4");
#pragma unroll
    for (int u = 0; u < GC_KW; u += 4) {
        const int k = k0 + u, tap = k >> 6, ci = k & 63, ky = tap / 3, kx = tap - ky * 3;
#pragma unroll
        for (int p3 = 0; p3 < 9; p3++) {
            const int oy = p3 / 3, ox = p3 - oy * 3;
            const float4 v = *reinterpret_cast<const float4 *>(a2f + ((oy + ky) * 5 + ox + kx) * 64 + ci);
            acc[p3] += v.x * wk[u];
            acc[p3] += v.y * wk[u + 1];
            acc[p3] += v.z * wk[u + 2];
            acc[p3] += v.w * wk[u + 3];
        }
    }
#pragma unroll
    for (int p3 = 0; p3 < 9; p3++) red[wv][p3][lane] = acc[p3];
    __syncthreads();
    for (int e = tid; e < 9 * 64; e += GC_T) {
        const int p3 = e >> 6, co = e & 63;
        float s = red[0][p3][co];
#pragma unroll
        for (int v = 1; v < GC_W; v++) s += red[v][p3][co];  // wave order
        a3[(size_t)tt * GA_K + e] = fmaxf(s + b3[(size_t)wt * 64 + co], 0.0f);
    }
}

// 16 waves x 4 columns per 64-column chunk (round 6; 4 waves walked 16 columns in 4 dependent load rounds): each lane
// issues its 36 fc1 weights, the columns' biases and head weights at once -- one load round trip per step
constexpr int GF_W = 16, GF_T = 64 * GF_W;
__global__ __launch_bounds__(GF_T) void k_group_fc1(const float *__restrict__ a3, const float *__restrict__ W4p,
                                                    const float *__restrict__ b4, const float *__restrict__ Wa,
                                                    const float *__restrict__ ba, const float *__restrict__ Wc,
                                                    const float *__restrict__ bc, int G, int A,
                                                    float *__restrict__ part, int shared) {
    __shared__ float red[GF_W][4];
    const int j = blockIdx.x, tt = blockIdx.y, g = tt >> 1, tower = tt & 1;
    const int wt = shared ? tower : tt, wg = shared ? 0 : g;  // the weights' tower and task
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n0 = j * 64 + wv * 4;  // this wave's 4 columns
    const float *wrow = W4p + (size_t)wt * GA_H * GA_K + (size_t)n0 * GA_K + lane;
    float wr[4][9];
#pragma unroll
    for (int c = 0; c < 4; c++)
#pragma unroll
        for (int i = 0; i < 9; i++) wr[c][i] = wrow[(size_t)c * GA_K + 64 * i];
    float bn[4], hw[4][4];
    const int na = tower == 0 ? A : 1;  // the tower's head rows: the task's A logits (actor) or its value (critic)
    const float *hsrc = tower == 0 ? Wa + (size_t)wg * A * GA_H : Wc + (size_t)wg * GA_H;
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const int n = n0 + c;
        bn[c] = b4[(size_t)wt * GA_H + n];
#pragma unroll
        for (int a = 0; a < 4; a++) {  // loaded unconditionally (row clamped into the tower's heads), then masked
            const float x = hsrc[(size_t)(a < na ? a : 0) * GA_H + n];
            hw[c][a] = a < na ? x : 0.0f;
        }
    }
    float x[9];
#pragma unroll
    for (int i = 0; i < 9; i++) x[i] = a3[(size_t)tt * GA_K + lane + 64 * i];
    float d[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
        float s = 0.0f;
#pragma unroll
        for (int i = 0; i < 9; i++) s += wr[c][i] * x[i];
        d[c] = s;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
#pragma unroll
        for (int c = 0; c < 4; c++) d[c] += __shfl_xor(d[c], off);
    float hp[4] = {0.0f, 0.0f, 0.0f, 0.0f};  // this wave's head partials over its 4 columns
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const float h = fmaxf(d[c] + bn[c], 0.0f);
#pragma unroll
        for (int a = 0; a < 4; a++) hp[a] += h * hw[c][a];
    }
    if (lane == 0)
#pragma unroll
        for (int a = 0; a < 4; a++) red[wv][a] = hp[a];
    __syncthreads();
    if (tid < 4) {
        float s = red[0][tid];
#pragma unroll
        for (int v = 1; v < GF_W; v++) s += red[v][tid];  // wave order
        if (j == 0) s += tower == 0 ? (tid < A ? ba[(size_t)wg * A + tid] : 0.0f) : (tid == 0 ? bc[wg] : 0.0f);
        part[(((size_t)tower * gridDim.x + j) * G + g) * 4 + tid] = s;
    }
}

}  // namespace

hipError_t launch_group_act(const uint32_t *codes, int G, const float *T2, const float *b2, const float *W3t,
                            const float *b3, const float *W4p, const float *b4, const float *Wa, const float *ba,
                            const float *Wc, const float *bc, int A, float *a3, float *part, bool shared,
                            hipStream_t s) {
    if (G <= 0) return hipSuccess;
    if (A < 1 || A > 4) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_group_conv, dim3(2 * G), dim3(GC_T), 0, s, codes, reinterpret_cast<const float4 *>(T2), b2,
                       W3t, b3, a3, (int)shared);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_group_fc1, dim3(GA_H / 64, 2 * G), dim3(GF_T), 0, s, a3, W4p, b4, Wa, ba, Wc, bc, G, A, part,
                       (int)shared);
    return hipGetLastError();
}

}  // namespace merlin
