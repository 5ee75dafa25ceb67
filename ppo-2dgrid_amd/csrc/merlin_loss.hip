// merlin_loss.hip -- the PPO minibatch loss (src/ppo.py:136-150) and its gradient with
// respect to the policy heads' outputs, evaluated once per distinct frame of the minibatch.
//
// The update evaluates the towers once per distinct observation u of a minibatch
// (merlin/dedup.py); sample i reads frame u(i).  Per sample, with z = logits[u(i)]:
//   logp = z - logsumexp(z), p = softmax(z), H = -sum p * logp          (Categorical, entropy)
//   ratio = exp(logp[a] - logp_old), s1 = ratio * A, s2 = clamp(ratio, 1 - eps, 1 + eps) * A
//   loss = -mean(min(s1, s2)) + vf * mean((v - R)^2) - ent * mean(H)
// and the loss gradient is summed per frame over the frame's samples (CSR offs/order from
// merlin/windows.py; fixed shuffle tree + item order): dlogits[u], dvalue[u] go straight into
// the heads' backward, replacing ~80 small torch kernels (index_select / log_softmax / gather / clamp /
// min / means and their backward, index_add) per optimizer step.  The subgradients follow
// torch's: torch.min sends half of the gradient to each operand on ties, clamp passes it
// inside [lo, hi] only.  With the heads' biases passed in (logits / value then exclude them),
// their gradients come out of the same pass.  The five statistics are summed in f64, per block in a fixed tree
// and over blocks in block order (bitwise reproducible).  Every frame must own >= 1 sample.
#include "merlin_internal.h"

namespace merlin {
namespace {

constexpr int LOSS_WAVES = 4, LOSS_BLK = 64 * LOSS_WAVES;
constexpr int MAXA = 8;
constexpr int NSTAT = 5;  // -pi, (v - R)^2, H, logp_old - logp, clipped
constexpr int NSUM = NSTAT + MAXA + 1;  // + the heads' bias gradients (sum of every sample's dz, dv)

// atomicMax of the block's maxima m[j] (float bits of non-negative values) into dmax[j], j < A and j = MAXA; every
// thread of the 256-thread block calls it
// (atomic false: stored to dmax[j] instead, every j <= MAXA)
__device__ __forceinline__ void block_max9(const uint32_t (&m)[MAXA + 1], int A, uint32_t *__restrict__ dmax,
                                           bool atomic = true) {
    __shared__ uint32_t red9[MAXA + 1][4];
#pragma unroll
    for (int j = 0; j <= MAXA; j++) {
        uint32_t x = m[j];
        for (int o = 32; o > 0; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o));
        if ((threadIdx.x & 63) == 0) red9[j][threadIdx.x >> 6] = x;
    }
    __syncthreads();
    if (threadIdx.x <= MAXA) {
        const uint32_t *r = red9[threadIdx.x];
        const uint32_t x = max(max(r[0], r[1]), max(r[2], r[3]));
        if (!atomic)
            dmax[threadIdx.x] = x;
        else if ((threadIdx.x < (unsigned)A || threadIdx.x == MAXA) && x &&
                 x > __hip_atomic_load(dmax + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            atomicMax(dmax + threadIdx.x, x);
    }
}

// One lane per sample in frame-sorted order (position k -> sample order[k] of frame
// inv[order[k]]), one wave per item of 64 positions.  Each lane forms its sample's loss
// gradient wrt its frame's logits / value; a segmented inclusive scan over the wave (fixed
// shuffle tree, frame runs as segments) leaves each run's sum on its last lane, which writes
// it to the frame, or -- for a run that starts before the item / continues after it -- to the
// item's carry slot 0 / 1 (k_ppo_loss_fix adds those in item order).  A frame with thousands
// of samples is thus spread over many waves instead of one serial thread.
__global__ __launch_bounds__(LOSS_BLK) void k_ppo_loss(const float *__restrict__ logits,
                                                       const float *__restrict__ value,
                                                       const float *__restrict__ bias_a,
                                                       const float *__restrict__ bias_c, int A,
                                                       const int32_t *__restrict__ offs,
                                                       const int32_t *__restrict__ order,
                                                       const int64_t *__restrict__ inv, int64_t n,
                                                       const int64_t *__restrict__ sample_index,
                                                       const int64_t *__restrict__ actions,
                                                       const float *__restrict__ lp_old,
                                                       const float *__restrict__ adv,
                                                       const float *__restrict__ ret, float lo, float hi,
                                                       float clip, float vf2_n, float ent_n, float inv_n,
                                                       float *__restrict__ dlogits, float *__restrict__ dvalue,
                                                       float *__restrict__ carry, double *__restrict__ partial,
                                                       uint32_t *__restrict__ bmax) {
    __shared__ double red[NSUM][LOSS_BLK];
    const int lane = threadIdx.x & 63;
    const int64_t item = (int64_t)blockIdx.x * LOSS_WAVES + (threadIdx.x >> 6);
    const int64_t k = item * 64 + lane;
    const bool live = k < n;
    double st[NSUM];
#pragma unroll
    for (int q = 0; q < NSUM; q++) st[q] = 0.0;
    float g[MAXA + 1];
#pragma unroll
    for (int j = 0; j <= MAXA; j++) g[j] = 0.0f;
    int64_t u = -1;
    if (live) {
        const int i = order[k];
        u = inv[i];
        const int64_t gi = sample_index ? sample_index[i] : i;
        const int64_t a = actions[gi];
        const float lpo = lp_old[gi], Av = adv[gi], R = ret[gi];
        float z[MAXA], lp[MAXA], p[MAXA];
        float m = -INFINITY;
#pragma unroll
        for (int j = 0; j < MAXA; j++) {  // every logit load issued unconditionally (index clamped), then masked
            const int jj = j < A ? j : 0;
            const float x = logits[u * A + jj] + (bias_a ? bias_a[jj] : 0.0f);
            z[j] = j < A ? x : -INFINITY;
            m = fmaxf(m, z[j]);
        }
        float s = 0.0f;
#pragma unroll
        for (int j = 0; j < MAXA; j++) s += j < A ? expf(z[j] - m) : 0.0f;
        const float lse = m + logf(s);
        float H = 0.0f;
#pragma unroll
        for (int j = 0; j < MAXA; j++) {
            lp[j] = z[j] - lse;
            p[j] = j < A ? expf(lp[j]) : 0.0f;
            if (j < A) H -= fmaxf(lp[j], -3.402823466e38f) * p[j];  // _entropy clamps logp at finfo.min
        }
        float la = NAN;  // an action outside [0, A) poisons the loss instead of reading past z
#pragma unroll
        for (int j = 0; j < MAXA; j++)
            if (a == j && j < A) la = lp[j];
        const float ratio = expf(la - lpo);
        const float s1 = ratio * Av;
        const float s2 = fminf(fmaxf(ratio, lo), hi) * Av;
        const float g1 = s1 < s2 ? 1.0f : (s1 == s2 ? 0.5f : 0.0f);
        const float g2 = s2 < s1 ? 1.0f : (s1 == s2 ? 0.5f : 0.0f);
        const bool inr = ratio >= lo && ratio <= hi;
        const float dla = -inv_n * Av * (g1 + (inr ? g2 : 0.0f)) * ratio;
#pragma unroll
        for (int j = 0; j < MAXA; j++) {
            const float d_lp = (a == j ? dla : 0.0f) - dla * p[j];  // d logp[a] / dz_j
            const float d_h = ent_n * p[j] * (lp[j] + H);            // -ent/n * dH/dz_j, dH/dz_j = -p_j (logp_j + H)
            g[j] = j < A ? d_lp + d_h : 0.0f;
        }
        const float d = value[u] + (bias_c ? bias_c[0] : 0.0f) - R;
        g[MAXA] = vf2_n * d;
#pragma unroll
        for (int j = 0; j <= MAXA; j++) st[NSTAT + j] = (double)g[j];
        st[0] = -(double)(s1 != s1 || s2 != s2 ? NAN : fminf(s1, s2));  // torch.min keeps NaN
        st[1] = (double)(d * d);
        st[2] = (double)H;
        st[3] = (double)(lpo - la);
        st[4] = fabsf(ratio - 1.0f) > clip ? 1.0 : 0.0;
    }
    // segmented inclusive scan over the wave: head = first position of a frame run in this item
    const int64_t uprev = __shfl_up(u, 1);
    bool head = lane == 0 || u != uprev;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const bool hup = __shfl_up(head, d);
        float up[MAXA + 1];
#pragma unroll
        for (int j = 0; j <= MAXA; j++) up[j] = __shfl_up(g[j], d);
        if (lane >= d && !head) {
#pragma unroll
            for (int j = 0; j <= MAXA; j++) g[j] = up[j] + g[j];
        }
        head = head || (lane >= d && hup);
    }
    const int64_t unext = __shfl_down(u, 1);
    const bool last = live && (lane == 63 || unext != u);
    if (last) {
        const int64_t e0 = item * 64, e1 = e0 + 64;
        const bool from_before = offs[u] < e0, goes_after = offs[u + 1] > e1;
        float *dst = nullptr;
        if (from_before)
            dst = carry + ((size_t)item * 2 + 0) * (MAXA + 1);
        else if (goes_after)
            dst = carry + ((size_t)item * 2 + 1) * (MAXA + 1);
        if (dst) {
#pragma unroll
            for (int j = 0; j <= MAXA; j++) dst[j] = g[j];
        } else {
#pragma unroll
            for (int j = 0; j < MAXA; j++)
                if (j < A) dlogits[u * A + j] = g[j];
            dvalue[u] = g[MAXA];
        }
    }
    if (bmax) {  // block-uniform: max |.| of the frames this block finished (the spanning ones: k_ppo_loss_fix),
                 // stored per block (same-address atomics from every block serialised: +9 us per launch)
        uint32_t m[MAXA + 1];
        const bool fin = last && offs[u] >= item * 64 && offs[u + 1] <= item * 64 + 64;
#pragma unroll
        for (int j = 0; j <= MAXA; j++) m[j] = fin ? __float_as_uint(g[j]) & 0x7fffffffu : 0u;
        block_max9(m, A, bmax + (size_t)blockIdx.x * (MAXA + 1), false);
    }
#pragma unroll
    for (int q = 0; q < NSUM; q++) red[q][threadIdx.x] = st[q];
    __syncthreads();
    for (int w = LOSS_BLK / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
#pragma unroll
            for (int q = 0; q < NSUM; q++) red[q][threadIdx.x] += red[q][threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x < NSUM) partial[(size_t)blockIdx.x * NSUM + threadIdx.x] = red[threadIdx.x][0];
}

__device__ void loss_fix_frame(const int32_t *__restrict__ offs, int64_t u, int A, const float *__restrict__ carry,
                               float *__restrict__ dlogits, float *__restrict__ dvalue, uint32_t *m);

// frames whose samples span items j0 < j1: carry[j0][1] + sum_{j0 < j <= j1} carry[j][0].
// dmax (nullable, zeroed by the caller): dmax[j] = max over the frames of |dlogits[u][j]| (j < A) and dmax[MAXA] =
// max |dvalue[u]|, as float bits (atomicMax of non-negative floats) -- the bound merlin_head.hip's k_head_bwd
// derives dz's plane scale from, so that it can write dz as h3 planes in its one pass.  k_ppo_loss leaves the
// maxima over the frames each block finishes (bmax, nbmax blocks), this kernel adds the frames that span items.
__global__ __launch_bounds__(256) void k_ppo_loss_fix(const int32_t *__restrict__ offs, int64_t U, int A,
                                                      const float *__restrict__ carry, float *__restrict__ dlogits,
                                                      float *__restrict__ dvalue, uint32_t *__restrict__ dmax,
                                                      const uint32_t *__restrict__ bmax, int64_t nbmax) {
    const int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (!dmax) {
        if (u < U) loss_fix_frame(offs, u, A, carry, dlogits, dvalue, nullptr);
        return;
    }
    uint32_t m[MAXA + 1];
    if (u < U) {
        loss_fix_frame(offs, u, A, carry, dlogits, dvalue, m);
    } else {
#pragma unroll
        for (int j = 0; j <= MAXA; j++) m[j] = 0u;
    }
    if (blockIdx.x == 0)  // k_ppo_loss's per-block maxima, folded in by this block's threads
        for (int64_t b = threadIdx.x; b < nbmax; b += 256)
#pragma unroll
            for (int j = 0; j <= MAXA; j++) m[j] = max(m[j], bmax[b * (MAXA + 1) + j]);
    block_max9(m, A, dmax);
}

// one frame of k_ppo_loss_fix; m (nullable) receives |dlogits[u][j]| / |dvalue[u]| as float bits (0 for j >= A)
__device__ void loss_fix_frame(const int32_t *__restrict__ offs, int64_t u, int A, const float *__restrict__ carry,
                               float *__restrict__ dlogits, float *__restrict__ dvalue, uint32_t *m) {
    const int64_t j0 = offs[u] / 64, j1 = (offs[u + 1] - 1) / 64;
    if (j1 <= j0) {  // the frame's sum was written (and its max taken) by k_ppo_loss
        if (m) {
#pragma unroll
            for (int j = 0; j <= MAXA; j++) m[j] = 0u;
        }
        return;
    }
    float acc[MAXA + 1];
    const float *c = carry + ((size_t)j0 * 2 + 1) * (MAXA + 1);
#pragma unroll
    for (int j = 0; j <= MAXA; j++) acc[j] = c[j];
    // a hot frame (thousands of samples) spans many items: two independent partial sums over
    // alternate items keep twice the loads in flight; fixed join order (bitwise reproducible)
    float acc2[MAXA + 1];
#pragma unroll
    for (int j = 0; j <= MAXA; j++) acc2[j] = 0.0f;
    int64_t it = j0 + 1;
    for (; it + 1 <= j1; it += 2) {
        const float *c0 = carry + ((size_t)it * 2) * (MAXA + 1);
        const float *c1 = carry + ((size_t)(it + 1) * 2) * (MAXA + 1);
        float v0[MAXA + 1], v1[MAXA + 1];
#pragma unroll
        for (int j = 0; j <= MAXA; j++) {
            v0[j] = c0[j];
            v1[j] = c1[j];
        }
#pragma unroll
        for (int j = 0; j <= MAXA; j++) {
            acc[j] += v0[j];
            acc2[j] += v1[j];
        }
    }
    if (it <= j1) {
        c = carry + ((size_t)it * 2) * (MAXA + 1);
#pragma unroll
        for (int j = 0; j <= MAXA; j++) acc[j] += c[j];
    }
#pragma unroll
    for (int j = 0; j <= MAXA; j++) acc[j] += acc2[j];
#pragma unroll
    for (int j = 0; j < MAXA; j++)
        if (j < A) dlogits[u * A + j] = acc[j];
    dvalue[u] = acc[MAXA];
    if (m) {
#pragma unroll
        for (int j = 0; j <= MAXA; j++) m[j] = j < A || j == MAXA ? __float_as_uint(acc[j]) & 0x7fffffffu : 0u;
    }
}

// stats[q] += (sum over the block partials) / n; loss = -pi + vf * v - ent * H (means); the
// heads' bias gradients = the sums of every sample's dz / dv.  Thread t sums partials t, t + 256,
// ... in order, then a fixed LDS tree: the same bits every call.
__global__ __launch_bounds__(256) void k_ppo_loss_final(const double *__restrict__ partial, int64_t nblk, int A,
                                                        double inv_n, double vf_coef, double ent_coef,
                                                        double *__restrict__ stats, float *__restrict__ loss,
                                                        float *__restrict__ dbias_a, float *__restrict__ dbias_c) {
    __shared__ double red[NSUM][256];
    const int t = threadIdx.x;
    double acc[NSUM];
#pragma unroll
    for (int q = 0; q < NSUM; q++) acc[q] = 0.0;
    for (int64_t b = t; b < nblk; b += 256) {
#pragma unroll
        for (int q = 0; q < NSUM; q++) acc[q] += partial[(size_t)b * NSUM + q];
    }
#pragma unroll
    for (int q = 0; q < NSUM; q++) red[q][t] = acc[q];
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (t < w) {
#pragma unroll
            for (int q = 0; q < NSUM; q++) red[q][t] += red[q][t + w];
        }
        __syncthreads();
    }
    if (t < NSTAT && stats) stats[t] += red[t][0] * inv_n;
    if (t == 0 && loss)
        loss[0] = (float)(red[0][0] * inv_n + vf_coef * (red[1][0] * inv_n) - ent_coef * (red[2][0] * inv_n));
    if (t < A && dbias_a) dbias_a[t] = (float)red[NSTAT + t][0];
    if (t == 0 && dbias_c) dbias_c[0] = (float)red[NSTAT + MAXA][0];
}

}  // namespace

int64_t ppo_loss_workspace_doubles(int64_t n) {
    const int64_t items = (n + 63) / 64, blocks = (items + LOSS_WAVES - 1) / LOSS_WAVES;
    // block partials + f32 carries + the blocks' |gradient| maxima (u32)
    return blocks * NSUM + (items * 2 * (MAXA + 1) + 1) / 2 + (blocks * (MAXA + 1) + 1) / 2;
}

hipError_t launch_ppo_loss(const float *logits, const float *value, const float *bias_a, const float *bias_c,
                           int64_t U, int A, const int32_t *offs, const int32_t *order, const int64_t *inv, int64_t n,
                           const int64_t *sample_index, const int64_t *actions, const float *lp_old, const float *adv,
                           const float *ret, double clip_eps, double vf_coef, double ent_coef, float *dlogits,
                           float *dvalue, float *dbias_a, float *dbias_c, float *loss, double *stats,
                           double *workspace, hipStream_t s, uint32_t *dmax) {
    const int64_t items = (n + 63) / 64, nblk = (items + LOSS_WAVES - 1) / LOSS_WAVES;
    const double inv_n = n > 0 ? 1.0 / (double)n : 0.0;
    double *partial = workspace;
    float *carry = reinterpret_cast<float *>(workspace + nblk * NSUM);
    uint32_t *bmax = dmax ? reinterpret_cast<uint32_t *>(workspace + nblk * NSUM + (items * 2 * (MAXA + 1) + 1) / 2)
                          : nullptr;
    if (nblk > 0) {
        hipLaunchKernelGGL(k_ppo_loss, dim3((unsigned)nblk), dim3(LOSS_BLK), 0, s, logits, value, bias_a, bias_c, A, offs,
                           order, inv, n,
                           sample_index, actions, lp_old, adv, ret, (float)(1.0 - clip_eps), (float)(1.0 + clip_eps),
                           (float)clip_eps, (float)(2.0 * vf_coef * inv_n), (float)(ent_coef * inv_n),
                           (float)inv_n, dlogits, dvalue, carry, partial, bmax);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_ppo_loss_fix, dim3((unsigned)((U + 255) / 256)), dim3(256), 0, s, offs, U, A, carry,
                           dlogits, dvalue, dmax, bmax, nblk);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_ppo_loss_final, dim3(1), dim3(256), 0, s, partial, nblk, A, inv_n, vf_coef, ent_coef, stats,
                       loss, dbias_a, dbias_c);
    return hipGetLastError();
}

}  // namespace merlin
