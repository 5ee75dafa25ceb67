// merlin_internal.h -- shared declarations between the HIP translation units of
// libmerlin_hip.so (not part of the public ABI; see include/merlin_hip.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "merlin_hip.h"

namespace merlin {

// Env state in HBM, structure-of-arrays, one slot per env (index i < n):
//   walls   uint32[n][SP]   row bitmasks (bit x of row y = wall at (x, y)); SP = 16 or 32
//   agent   uint4[n]        x: ax | ay<<8 | dir<<16   y: step_count
//                           z: gx | gy<<8             w: last_x | last_y<<8 | stay<<16
//   rng_s   ulonglong2[n]   PCG64 128-bit state (x = low 64, y = high 64)
//   rng_i   ulonglong2[n]   PCG64 increment
//   rng_b   uint2[n]        (has32, buf32) -- numpy's persistent 32-bit half buffer
//   ep_ret  double[n]       running episode return (src/ppo.py:88 accumulates a Python float)
//   ep_len  int32[n]
//   visited uint32[n][SP]   exploration-bonus visit bitmask (only if enabled)
//   err     uint32[2]       device error bits, fallback-map counter
//   pg_*    the env's look-ahead map (merlin_env.hip k_env_refill): pg_walls uint32[n][SP],
//           pg_agent uint4[n] (agent format above), pg_rng_s / pg_rng_b (RNG state after it),
//           pg_valid uint8[n] (1 = the slot holds the env's next map)
//   rflag   uint8[n]        1 = reset due, its slot was empty (single-step launch; k_env_fallback)
//   bflag   uint8[ceil(n/64)] 1 = some env of that step block (SBLK envs, merlin_env.hip) is flagged
struct EnvDev {
    int n, size, sp, difficulty, max_steps;
    int stuck_on, max_stay;
    double penalty;
    int explore_on;
    double bonus;
    int reseed;  // never persist the advanced RNG state: every reset = reset(seed=...)
    uint32_t *walls;
    uint4 *agent;
    ulonglong2 *rng_s;
    ulonglong2 *rng_i;
    uint2 *rng_b;
    double *ep_ret;
    int32_t *ep_len;
    uint32_t *visited;
    uint32_t *err;
    uint32_t *pg_walls;
    uint4 *pg_agent;
    ulonglong2 *pg_rng_s;
    uint2 *pg_rng_b;
    uint8_t *pg_valid;
    uint8_t *rflag;
    uint8_t *bflag;
};

// step launches between two look-ahead refills (merlin_env_step)
constexpr int REFILL_EVERY = 16;

// ---------------------------------------------------------------------------------------------------------------
// The acting tail shared by merlin_act.hip (k_act_heads, k_act_draw) and the fused draw + env step
// (merlin_env.hip, merlin_env_act_step): log-softmax, argmax or the counter-keyed exponential-race draw.
constexpr int ACT_MAXA = 8;
constexpr int ACT_PARTS_UNROLL = 8;  // head-partial chunks summed with all loads in flight (act_from_parts)


__device__ __forceinline__ float relu_nan(float v) { return v != v ? v : fmaxf(v, 0.0f); }  // torch.relu keeps NaN

__device__ __forceinline__ uint64_t mix64(uint64_t x) {  // splitmix64 finaliser
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    x ^= x >> 31;
    return x;
}

// uniform in (0, 1]: 53 random bits of the hash of (seed, epoch, step, env, j)
__device__ __forceinline__ double uniform01(uint64_t seed, uint64_t epoch, uint64_t step, uint64_t env, int j) {
    uint64_t x = mix64(seed + 0x9e3779b97f4a7c15ull);
    x = mix64(x ^ (epoch + 0x632be59bd9b4e019ull));
    x = mix64(x ^ (step * 0x8cb92ba72f3d8dd7ull));
    x = mix64(x ^ (env * 0xd6e8feb86659fd93ull + (uint64_t)j));
    return (double)((x >> 11) + 1) * (1.0 / 9007199254740992.0);
}

// acc[j < A]: the actor's head dot products, acc[ACT_MAXA]: the critic's; biases added here.  Log-softmax, argmax or the
// exponential-race draw, action / logp / value of env k written.
__device__ __forceinline__ int act_finish(const float (&acc)[ACT_MAXA + 1], const float *__restrict__ ba,
                                           const float *__restrict__ bc, int A, int det, uint64_t seed, uint64_t ep,
                                           int64_t step, int64_t env_offset, int64_t k, int64_t *__restrict__ action,
                                           float *__restrict__ logp, float *__restrict__ value) {
    float zl[ACT_MAXA], m = -INFINITY;
    int amax = 0;
    float bj[ACT_MAXA];  // every bias load issued before any is used (index clamped into [0, A): no load behind a branch)
#pragma unroll
    for (int j = 0; j < ACT_MAXA; j++) bj[j] = ba[j < A ? j : 0];
#pragma unroll
    for (int j = 0; j < ACT_MAXA; j++) {
        zl[j] = j < A ? acc[j] + bj[j] : -INFINITY;
        if (zl[j] > m) {  // first maximum (torch.argmax)
            m = zl[j];
            amax = j;
        }
    }
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < ACT_MAXA; j++) s += j < A ? expf(zl[j] - m) : 0.0f;
    const float lse = m + logf(s);
    int a = amax;
    if (!det) {
        double best = -INFINITY;
#pragma unroll
        for (int j = 0; j < ACT_MAXA; j++) {
            if (j < A) {
                // log(p_j / E_j) = logp_j - log(-log u)
                const double sc = (double)(zl[j] - lse) -
                                  log(-log(uniform01(seed, ep, (uint64_t)step, (uint64_t)(env_offset + k), j)));
                if (sc > best) {
                    best = sc;
                    a = j;
                }
            }
        }
    }
    float la = zl[0] - lse;
#pragma unroll
    for (int j = 1; j < ACT_MAXA; j++)
        if (j == a) la = zl[j] - lse;
    // non-finite logits (a diverged update): Categorical(logits) raises in the reference;
    // here the action is the sentinel -1, which the next env step rejects
    // (MERLIN_DEVERR_BAD_ACTION, read once per rollout by merlin_env_errors)
    if (!isfinite(lse)) a = -1;
    action[k] = a;
    logp[k] = la;
    value[k] = acc[ACT_MAXA] + bc[0];
    return a;
}


// the fused draw of merlin_env_act_step: the heads' partial dot products of the acting GEMM's epilogue
// (part[t][p][k][4], P partials per env summed in order; tower 0: the actor's A <= 4 logits, tower 1: the critic's
// value in .x), drawn and written to action / logp / value, the action then stepped by the same thread
struct ActIn {
    const float4 *part;  // null: the actions are read from StepOut::actions
    int P;
    const float *ba, *bc;
    int A, det;
    uint64_t seed;
    const int64_t *epoch;
    int64_t step, env_offset;
    int64_t *action;
    float *logp, *value;
};

__device__ __forceinline__ int act_from_parts(const ActIn &c, int64_t n, int64_t k) {
    float4 a, v;
    if (c.P <= ACT_PARTS_UNROLL) {
        // the common widths (8 chunk partials: the acting GEMM's heads epilogue, merlin_group_act): every partial's
        // load issued first (indices clamped into [0, P): no load behind a branch, one round trip instead of P), then
        // the same ordered sums as the loop below -- the same bits
        float4 xs[ACT_PARTS_UNROLL];
        float ys[ACT_PARTS_UNROLL];  // the critic's partials: only their first lane is the value's
#pragma unroll
        for (int p = 0; p < ACT_PARTS_UNROLL; p++) {
            const int q = p < c.P ? p : 0;
            xs[p] = c.part[(int64_t)q * n + k];
            ys[p] = reinterpret_cast<const float *>(c.part + (int64_t)(c.P + q) * n + k)[0];
        }
        a = xs[0];
        v = make_float4(ys[0], 0.0f, 0.0f, 0.0f);
#pragma unroll
        for (int p = 1; p < ACT_PARTS_UNROLL; p++) {
            if (p < c.P) {
                a.x += xs[p].x;
                a.y += xs[p].y;
                a.z += xs[p].z;
                a.w += xs[p].w;
                v.x += ys[p];
            }
        }
    } else {
        a = c.part[k];
        v = c.part[(int64_t)c.P * n + k];
        for (int p = 1; p < c.P; p++) {
            const float4 x = c.part[(int64_t)p * n + k], y = c.part[(int64_t)(c.P + p) * n + k];
            a.x += x.x;
            a.y += x.y;
            a.z += x.z;
            a.w += x.w;
            v.x += y.x;
        }
    }
    float acc[ACT_MAXA + 1];
#pragma unroll
    for (int j = 0; j <= ACT_MAXA; j++) acc[j] = 0.0f;
    acc[0] = a.x;
    acc[1] = a.y;
    acc[2] = a.z;
    acc[3] = a.w;
    acc[ACT_MAXA] = v.x;
    const uint64_t ep = c.epoch ? (uint64_t)c.epoch[0] : 0ull;
    return act_finish(acc, c.ba, c.bc, c.A, c.det, c.seed, ep, c.step, c.env_offset, k, c.action, c.logp, c.value);
}

struct StepOut {
    const int64_t *actions;
    int64_t action_stride;
    int n_steps;
    int autoreset;
    uint32_t *obs;
    float *reward;
    uint8_t *term;
    uint8_t *trunc;
    float *done;
    double *ep_ret_out;
    int32_t *ep_len_out;
    ActIn act;  // act.part != null (n_steps == 1): the action of env i is drawn from the heads' partials first
    int no_fallback;  // single-step launches: no k_env_fallback pass; an empty slot raises MERLIN_DEVERR_SLOT_EMPTY
};

// Zero `bytes` bytes at p on stream s with a kernel (vector stores).  Every zero-fill of the library goes
// through this, never hipMemsetAsync: a memset node captured into a HIP graph replays with a wrong fill value on
// ROCm 7 (scripts/probe_graph_then.py: 0x80 per byte), and any entry point may end up inside a capture.
hipError_t zero_async(void *p, size_t bytes, hipStream_t s);
hipError_t launch_group_act(const uint32_t *codes, int G, const float *T2, const float *b2, const float *W3t,
                            const float *b3, const float *W4p, const float *b4, const float *Wa, const float *ba,
                            const float *Wc, const float *bc, int A, float *a3, float *part, bool shared, hipStream_t s);
hipError_t launch_h3p_gemm_nt(const void *A, const uint32_t *amaxA, const void *B, const uint32_t *amaxB, int64_t M,
                              int N, int K, int T, int64_t a_stride, int64_t b_stride, const float *bias, float *C,
                              int64_t c_stride, int cfg, hipStream_t s, const int32_t *a_rows = nullptr,
                              const float *head_w0 = nullptr, int n_actions = 0, const float *head_w1 = nullptr,
                              float *head_part = nullptr);
hipError_t launch_h3p_gemm_tn_gather(const void *A, const uint32_t *amaxA, const void *B, const uint32_t *amaxB,
                                     int64_t Kd, int M, int N, int T, int64_t a_stride, int64_t b_stride, int splits,
                                     float *slab, const int32_t *b_rows, int cfg, int *S_out, hipStream_t s);
hipError_t launch_env_reset(const EnvDev &E, const uint8_t *mask, uint32_t *obs, hipStream_t s);
hipError_t launch_env_step(const EnvDev &E, const StepOut &O, bool refill, hipStream_t s);
hipError_t launch_env_full_obs(const EnvDev &E, uint8_t *out, hipStream_t s);
hipError_t launch_env_refill(const EnvDev &E, bool full, hipStream_t s);
hipError_t upload_atlas(const uint8_t *atlas_host);
hipError_t launch_obs_expand_f32(const uint32_t *codes, const int64_t *index, int64_t n, float *out,
                                 float scale, int layout, hipStream_t s);
hipError_t launch_obs_expand_u8(const uint32_t *codes, const int64_t *index, int64_t n, uint8_t *out,
                                hipStream_t s);
hipError_t launch_gae(const float *rew, const float *val, const float *done, const float *last,
                      float *adv, float *ret, int T, int N, double gamma, double lam, double *stats,
                      double *partials, int max_partials, hipStream_t s);
hipError_t launch_adv_normalize(const float *adv, int64_t n, const double *stats, float *out,
                                hipStream_t s);
int gae_partials_needed(int T, int N);
int conv1_slab_floats(int towers);
hipError_t launch_conv1_lut_fwd(const uint32_t *codes, const int64_t *index, int64_t n, const float *tables,
                                const float *bias, int towers, float *out, hipStream_t s);
hipError_t launch_conv1_lut_bwd(const uint32_t *codes, const int64_t *index, int64_t n, const float *act,
                                const float *grad, int towers, float *dtables, float *dbias, float *slabs,
                                int max_slabs, hipStream_t s);
hipError_t launch_conv1_im2col_fwd(const uint32_t *codes, const int64_t *index, int64_t n, const float *tables,
                                   const float *bias, int T, float *A2, hipStream_t s);
hipError_t launch_conv1_im2col_bwd(const uint32_t *codes, const int64_t *index, int64_t n, const float *tables,
                                   const float *bias, const float *dA2, int T, float *dtables, float *dbias,
                                   float *slabs, int max_slabs, hipStream_t s);
hipError_t launch_im2col3_fwd(const float *Z2, const float *b2, int64_t n, int T, float *A3, hipStream_t s);
hipError_t launch_col2im3_bwd(const float *dA3, const float *Z2, const float *b2, int64_t n, int T, int chunked,
                              float *dZ2, uint32_t *absmax, hipStream_t s);
int conv2_lut_rows();
int conv2_lut_fblocks(int64_t n);
size_t conv2_lut_slab_bytes(int towers, int fblocks);
hipError_t launch_conv2_lut_fwd(const uint32_t *codes, const int64_t *index, int64_t n, const float *tables,
                                int towers, float *Z2, hipStream_t s, int64_t gstride = 0);
hipError_t launch_conv2_lut_bwd(const uint32_t *codes, int64_t n, const float *dZ2c, const uint32_t *absmax,
                                int towers, float *dT, void *slabs, hipStream_t s, int64_t gstride = 0);

hipError_t launch_patch_maps(const int32_t *kid, const int64_t *gkey, int64_t G, int64_t F, const int64_t *goff, int K,
                             int32_t *kmap, int32_t *rmap, int32_t *rep_row, hipStream_t s);
hipError_t launch_window_lut(const int32_t *rows, int64_t nw, const float *tab, int T, float *Z2w, hipStream_t s,
                             const float *b2 = nullptr);
hipError_t launch_window_conv3(const float *Q, int64_t nw, const int32_t *wid, const int64_t *groups, int64_t n,
                               const float *b3, int T, float *Y3, uint64_t *bits, uint32_t *amax,
                               const int32_t *rrow, int copy, hipStream_t s, uint32_t *colmax = nullptr,
                               uint32_t *bound = nullptr);
hipError_t launch_act_heads(const float *z, const float *b4, int64_t n, int H, const float *wa, const float *ba,
                            const float *wc, const float *bc, int A, int det, uint64_t seed, const int64_t *epoch,
                            int64_t step, int64_t env_offset, int64_t *action, float *logp, float *value,
                            hipStream_t s);
// the acting tail from the heads' partials of the acting GEMM's epilogue (merlin_h3.hip EPI 3), part [2][P][n][4]
hipError_t launch_act_draw(const float *part, int P, int64_t n, const float *ba, const float *bc, int A, int det,
                           uint64_t seed, const int64_t *epoch, int64_t step, int64_t env_offset, int64_t *action,
                           float *logp, float *value, hipStream_t s);
int64_t ppo_loss_workspace_doubles(int64_t n_samples);
hipError_t launch_ppo_loss(const float *logits, const float *value, const float *bias_a, const float *bias_c,
                           int64_t U, int A, const int32_t *offs, const int32_t *order, const int64_t *inv, int64_t n,
                           const int64_t *sample_index, const int64_t *actions, const float *lp_old, const float *adv,
                           const float *ret, double clip_eps, double vf_coef, double ent_coef, float *dlogits,
                           float *dvalue, float *dbias_a, float *dbias_c, float *loss, double *stats,
                           double *workspace, hipStream_t s, uint32_t *dmax = nullptr);
hipError_t launch_codes_conv3(const uint32_t *codes, int64_t n, const float *Q, const float *b3, int T, float *Y3,
                              uint32_t *amax, uint32_t *err, hipStream_t s);
hipError_t launch_x6_gemm_nt32(const float *A, const void *B, int64_t M, int N, int K, int T, int64_t a_stride,
                               int64_t b_stride, const float *bias, float *C, int64_t c_stride, int cfg, hipStream_t s);
hipError_t launch_x6_gemm_tn32(const float *A, const float *B, int64_t Kd, int M, int N, int T, int64_t a_stride,
                               int64_t b_stride, int splits, float *slab, int cfg, hipStream_t s, int *S_out);
hipError_t launch_stage_fwd(const float *W1, const float *b1, const float *W2, const float *atlas, const int16_t *idx,
                            int T, float *HT, float *T2, hipStream_t s);
hipError_t launch_stage_bwd(const float *W2, const float *HT, const float *dT2, const float *atlas,
                            const int16_t *koff, const int16_t *kv, int T, float *dH, float *dW1, float *db1,
                            float *dW2, double *ws, hipStream_t s);
// the window GEMM's backward (csrc/merlin_winbwd.hip): work = winbwd_work_floats(T, nw) floats of scratch
int64_t winbwd_work_floats(int T, int64_t nw);
hipError_t launch_winbwd(const float *a2w, const float *dQ, const float *W3r, int T, int64_t nw, float *da2w,
                         float *db2, float *dW3r, float *work, hipStream_t s, float *db3 = nullptr);
hipError_t launch_winfwd(const float *a2w, const float *W3r, int T, int64_t nw, float *Q, hipStream_t s);
// k_stage_bwd_w's partials (towers x taps x parts x outputs)
constexpr size_t STAGE_WS_DOUBLES = 2 * 4 * 10 * 2048;
hipError_t launch_heads_fwd(const float *h, int64_t n, int H, const float *wa, int A, const float *wc, const float *ba,
                            const float *bc, float *logits, float *value, hipStream_t s);
hipError_t launch_seg_sum(const float *src, const void *mask, int mask_bits, int64_t src_rows, const int32_t *idx,
                          const int32_t *key, int64_t nnz, const int32_t *slot, int S, int64_t L, const int32_t *fix,
                          int64_t nfix, int T, float *out, int64_t out_rows, float *carry, int acc_out, int fill, int role,
                          int32_t *mark, const int32_t *hfix, int32_t *cnt, hipStream_t s,
                          const int32_t *mrow = nullptr);

// GEMM epilogues (merlin_head.hip); partial sums use a per-device workspace of
// epilogue_work_floats() floats
constexpr int EPI_MAX_BLOCKS = 512;
size_t epilogue_work_floats();
bool epilogue_cols_ok(int cols);
int epilogue_max_act();
hipError_t launch_bias_relu(float *Z, const float *b, int64_t rows, int cols, int T, hipStream_t s);
hipError_t launch_relu_bwd_colsum(const float *Y, const float *dY, float *dZ, int64_t rows, int cols, int T,
                                  float *dbias, float *work, hipStream_t s);
hipError_t launch_colsum(const float *X, int64_t rows, int cols, int64_t row_stride, int64_t tower_stride, int T,
                         float *out, float *work, hipStream_t s);
hipError_t launch_head_bwd(const float *h, const float *dlogits, const float *dvalue, const float *wa,
                           const float *wc, int64_t n, int H, int A, float *dz, float *db4, float *dwa, float *dwc,
                           float *work, uint32_t *amax, hipStream_t s, const uint32_t *dmax = nullptr,
                           void *dz_planes = nullptr);

// atomicMax of each tower's block maximum (float bits of non-negative values) into amax[t], t < T <= 2; every
// thread of the 256-thread block calls it
__device__ __forceinline__ void block_amax2(const uint32_t mx[2], int T, uint32_t *amax) {
    __shared__ uint32_t red[2][4];
    uint32_t m0 = mx[0], m1 = mx[1];
    for (int o = 32; o > 0; o >>= 1) {
        m0 = max(m0, (uint32_t)__shfl_xor((int)m0, o));
        m1 = max(m1, (uint32_t)__shfl_xor((int)m1, o));
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = m0;
        red[1][threadIdx.x >> 6] = m1;
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)T) {
        const uint32_t *r = red[threadIdx.x];
        const uint32_t m = max(max(r[0], r[1]), max(r[2], r[3]));
        // the word only grows: a block whose max is not above it (most of them, once a few have reported) skips
        // the atomic -- thousands of same-address atomics serialise at the memory side
        if (m && m > __hip_atomic_load(amax + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            atomicMax(amax + threadIdx.x, m);
    }
}

// ---------------------------------------------------------------------------------------------------------------
// The h3 operand form (merlin_h3.hip's header comment): per tower one power-of-two scale 2^e from a bound on max |x|,
// per value an f16 hi plane and an f16 lo plane (x 2^11).  Shared by merlin_h3.hip's splits and the producers that
// write their output as planes directly (k_head_bwd's dz, conv3's representatives).
constexpr float H3_LO_SCALE = 2048.0f;
// the scale exponent e of a tensor whose max |x| (or a bound on it) has float bits `amax`: amax 2^e in [2^14, 2^15)
__device__ __forceinline__ int h3_exp(uint32_t amax) {
    if (amax == 0u) return 0;
    const int e = (int)((amax >> 23) & 0xffu) - 127;  // floor(log2) for a normal max (inf / nan: e = 128)
    return min(max(14 - e, -120), 115);                // e + 11 stays a normal power of two
}
__device__ __forceinline__ float pow2f(int e) { return __uint_as_float((uint32_t)(e + 127) << 23); }

// planes of two unscaled values a, b (sc = 2^e, sc2 = 2^(e + 11)): hi word (h of a, h of b) = f16(x'), lo word =
// f16(2^11 x' - 2^11 h), each by one v_fma_mix{lo,hi}_f16 (the mixed fma rounds its exact result once to f16; in
// the lo ones h is read as an f16 operand from its half of the hi word, so x' - h is never formed in f32): six
// vector instructions per pair (the compiler's version of the same expressions took nine, computing h twice)
__device__ __forceinline__ void h3_pair(float a, float b, float sc, float sc2, uint32_t &hi, uint32_t &lo) {
    const float m2048 = -H3_LO_SCALE, za = a * sc2, zb = b * sc2;
    uint32_t h, l;
    asm("v_fma_mixlo_f16 %0, %1, %2, 0" : "=v"(h) : "v"(a), "v"(sc));
    asm("v_fma_mixhi_f16 %0, %1, %2, 0" : "+v"(h) : "v"(b), "v"(sc));
    asm("v_fma_mixlo_f16 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(l) : "v"(h), "v"(m2048), "v"(za));
    asm("v_fma_mixhi_f16 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(l) : "v"(h), "v"(m2048), "v"(zb));
    hi = h;
    lo = l;
}

// 4 consecutive values (columns 4 q .. 4 q + 3 of a row) -> their halves of the row's plane image: hi at uint2 index
// 4 (q >> 1) + (q & 1), lo 2 uint2 further (a group of 8 values = a 16-B hi chunk + a 16-B lo chunk)
__device__ __forceinline__ void h3_store4(uint2 *__restrict__ row, int q, const float4 v, float sc, float sc2) {
    uint32_t h0, h1, l0, l1;
    h3_pair(v.x, v.y, sc, sc2, h0, l0);
    h3_pair(v.z, v.w, sc, sc2, h1, l1);
    const int o = 4 * (q >> 1) + (q & 1);
    row[o] = make_uint2(h0, h1);
    row[o + 2] = make_uint2(l0, l1);
}

// h3_store4 with adjacent lanes paired (lane q and q ^ 1, both active, holding the two halves of one 8-value group):
// one 16-B store per lane instead of two 8-B ones -- the even lane writes the group's hi chunk, the odd lane its lo
// chunk (uint4 index q of the row's plane image), after one exchange of two words
__device__ __forceinline__ void h3_store4_pair(uint4 *__restrict__ row, int q, const float4 v, float sc, float sc2) {
    uint32_t h0, h1, l0, l1;
    h3_pair(v.x, v.y, sc, sc2, h0, l0);
    h3_pair(v.z, v.w, sc, sc2, h1, l1);
    const bool odd = q & 1;
    const uint32_t r0 = (uint32_t)__shfl_xor((int)(odd ? h0 : l0), 1);
    const uint32_t r1 = (uint32_t)__shfl_xor((int)(odd ? h1 : l1), 1);
    row[q] = odd ? make_uint4(r0, r1, l0, l1) : make_uint4(h0, h1, r0, r1);
}

// fc1 on the bf16 matrix cores in exact three-plane form (merlin_gemm.hip, merlin_x6.h)
hipError_t launch_x6_split(const float *x, int64_t n, void *planes, hipStream_t s);
hipError_t launch_x6_join(const void *planes, int64_t n, float *x, hipStream_t s);
hipError_t launch_x6_gemm_nt(const float *A, const void *B, int64_t M, int N, int K, int T, int64_t a_stride,
                             int64_t b_stride, const float *bias, float *C, int64_t c_stride, int cfg, hipStream_t s);
hipError_t launch_x6_gemm_tn(const float *A, const float *B, int64_t Kd, int M, int N, int T, int64_t a_stride,
                             int64_t b_stride, int splits, float *slab, float *out, int cfg, hipStream_t s);
int x6_tn_max_splits();
// out[e] = sum over s < S of slab[s][e], in slab order (total % 4 == 0)
hipError_t launch_x6_fold(const float *slab, int S, int64_t total, float *out, hipStream_t s);
// fc1 on the f16 matrix cores in two-plane form (merlin_h3.hip)
hipError_t launch_h3_amax(const float *x, int64_t n, int T, int64_t stride, uint32_t *amax, hipStream_t s);
hipError_t launch_h3_split(const float *x, int64_t n, int T, const uint32_t *amax, void *planes, hipStream_t s);
// a_planes (nullable): receives A's planes ([T][M][K/8][2][8] f16, A's byte layout), written by the first column
// tile's blocks
hipError_t launch_h3_gemm_nt(const float *A, const uint32_t *amaxA, const void *B, const uint32_t *amaxB, int64_t M,
                             int N, int K, int T, int64_t a_stride, int64_t b_stride, const float *bias, float *C,
                             int64_t c_stride, void *a_planes, int cfg, hipStream_t s,
                             const int32_t *a_rows = nullptr, const float *head_w0 = nullptr, int n_actions = 0,
                             const float *head_w1 = nullptr, float *head_part = nullptr, bool a_is_planes = false);
// head_part (nullable; pipelined cfgs 10 / 12 / 13 with bias, 2 towers): the heads' dot products of h folded into the
// forward GEMM's epilogue, h3_heads_parts(N, cfg) float4 partials per row and tower, [2][parts][M][4]; summed by
// launch_heads_combine into logits [M][n_actions] and value [M]
int h3_heads_parts(int N, int cfg);
hipError_t launch_heads_combine(const float *part, int P, int64_t M, int na, float *logits, float *value,
                                hipStream_t s);
// planes: A and B are plane images (an NT's a_planes) instead of fp32 tensors
// a_rows / b_rows (nullable): the operand's rows gathered by 64-value chunks -- row r's chunk j is row
// rows[r * (K or N) / 64 + j] of the operand seen as [*][64] (k_h3_ntp GA, k_h3_tn GB; pipelined NT cfgs and TN
// cfgs 0-2 only)
hipError_t launch_h3_gemm_tn(const void *A, const uint32_t *amaxA, const void *B, const uint32_t *amaxB, int64_t Kd,
                             int M, int N, int T, int64_t a_stride, int64_t b_stride, int splits, float *slab,
                             float *out, bool planes, int cfg, hipStream_t s, const int32_t *b_rows = nullptr,
                             bool a_planes = false, bool b_planes = false);

// clip_grad_norm_ + Adam step over a parameter list (merlin_optim.hip)
constexpr int OPT_MAX_TENSORS = 32;
int64_t opt_blocks(int n, const int64_t *numel);
hipError_t launch_clip_adam(int n, float *const *params, float *const *grads, float *const *exp_avg,
                            float *const *exp_avg_sq, float *const *steps, const int64_t *numel, double lr, double beta1,
                            double beta2, double eps, float max_norm, float *norm_out, double *partial, hipStream_t s);

}  // namespace merlin
