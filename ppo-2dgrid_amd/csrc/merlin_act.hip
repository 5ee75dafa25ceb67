// merlin_act.hip -- the acting path's tail: fc1's bias + ReLU, both heads, the categorical
// log-probabilities and the action sample, one wave per env (src/actor_critic.py:48-55:
// CNNActorCritic.act; src/ppo.py:69-71 stores action, log-prob and value).
//
// Input is fc1's pre-activation of both towers, z[t][k][:] (a plain bmm, no epilogue).  Lane l
// owns columns 4l.., 4l + 256.. of the hidden layer: h = relu(z + b4), the actor's A dot
// products and the critic's one are summed per lane, then over the wave by a fixed xor tree.
// Lane 0 forms logp = logits - logsumexp(logits) and draws the action by exponential races,
// argmax_j p_j / E_j with E_j ~ Exp(1) (the law of Categorical(logits).sample(); torch's
// multinomial uses the same race), from a counter-based generator keyed by (seed, *epoch,
// step, global env index = env_offset + env, j: a data-parallel shard draws what one process
// over the concatenated envs would): no RNG state, so the rollout replays as a HIP graph with a fresh draw per
// replay once the caller bumps *epoch.  deterministic = argmax of the logits (first maximum,
// as torch.argmax).  Non-finite logits give action -1 (see below).  Writes action int64,
// logp[action] and value straight into the rollout
// storage: the 2 head GEMMs + ~17 small torch kernels + 3 copies of the per-step tail become one
// launch.
#include <algorithm>

#include "merlin_internal.h"

namespace merlin {
namespace {

constexpr int ACT_WAVES = 4;
constexpr int MAXA = ACT_MAXA;
__global__ __launch_bounds__(64 * ACT_WAVES) void k_act_heads(const float4 *__restrict__ z,
                                                              const float4 *__restrict__ b4, int64_t n, int H4,
                                                              const float4 *__restrict__ wa,
                                                              const float *__restrict__ ba,
                                                              const float4 *__restrict__ wc,
                                                              const float *__restrict__ bc, int A, int det,
                                                              uint64_t seed, const int64_t *__restrict__ epoch,
                                                              int64_t step, int64_t env_offset,
                                                              int64_t *__restrict__ action,
                                                              float *__restrict__ logp, float *__restrict__ value) {
    const int lane = threadIdx.x & 63;
    const uint64_t ep = epoch ? (uint64_t)epoch[0] : 0ull;
    for (int64_t k = (int64_t)blockIdx.x * ACT_WAVES + (threadIdx.x >> 6); k < n;
         k += (int64_t)gridDim.x * ACT_WAVES) {
        float acc[MAXA + 1];
#pragma unroll
        for (int j = 0; j <= MAXA; j++) acc[j] = 0.0f;
        for (int c = lane; c < H4; c += 64) {
            const float4 z0 = z[(size_t)k * H4 + c], z1 = z[((size_t)n + k) * H4 + c];
            const float4 c0 = b4[c], c1 = b4[H4 + c];
            const float4 h0 = make_float4(relu_nan(z0.x + c0.x), relu_nan(z0.y + c0.y), relu_nan(z0.z + c0.z),
                                          relu_nan(z0.w + c0.w));
            const float4 h1 = make_float4(relu_nan(z1.x + c1.x), relu_nan(z1.y + c1.y), relu_nan(z1.z + c1.z),
                                          relu_nan(z1.w + c1.w));
#pragma unroll
            for (int j = 0; j < MAXA; j++) {
                if (j < A) {
                    const float4 w = wa[(size_t)j * H4 + c];
                    acc[j] += h0.x * w.x + h0.y * w.y + h0.z * w.z + h0.w * w.w;
                }
            }
            const float4 w = wc[c];
            acc[MAXA] += h1.x * w.x + h1.y * w.y + h1.z * w.z + h1.w * w.w;
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
            for (int j = 0; j <= MAXA; j++) acc[j] += __shfl_xor(acc[j], off);
        }
        if (lane == 0) act_finish(acc, ba, bc, A, det, seed, ep, step, env_offset, k, action, logp, value);
    }
}

// The same tail from the heads' partial dot products of the acting GEMM's epilogue (merlin_h3.hip EPI 3: h is
// never written): part[t][p][k][4], P partials per env summed in order (tower 0: the actor's A <= 4 logits, tower 1:
// the critic's value in .x).  One thread per env.
__global__ __launch_bounds__(256) void k_act_draw(const float4 *__restrict__ part, int P, int64_t n,
                                                  const float *__restrict__ ba, const float *__restrict__ bc, int A,
                                                  int det, uint64_t seed, const int64_t *__restrict__ epoch,
                                                  int64_t step, int64_t env_offset, int64_t *__restrict__ action,
                                                  float *__restrict__ logp, float *__restrict__ value) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    const ActIn c{part, P, ba, bc, A, det, seed, epoch, step, env_offset, action, logp, value};
    act_from_parts(c, n, k);
}

}  // namespace

hipError_t launch_act_heads(const float *z, const float *b4, int64_t n, int H, const float *wa, const float *ba,
                            const float *wc, const float *bc, int A, int det, uint64_t seed, const int64_t *epoch,
                            int64_t step, int64_t env_offset, int64_t *action, float *logp, float *value,
                            hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int grid = (int)std::min<int64_t>((n + ACT_WAVES - 1) / ACT_WAVES, 256 * 8);
    hipLaunchKernelGGL(k_act_heads, dim3(grid), dim3(64 * ACT_WAVES), 0, s, reinterpret_cast<const float4 *>(z),
                       reinterpret_cast<const float4 *>(b4), n, H / 4, reinterpret_cast<const float4 *>(wa), ba,
                       reinterpret_cast<const float4 *>(wc), bc, A, det, seed, epoch, step, env_offset, action, logp,
                       value);
    return hipGetLastError();
}

hipError_t launch_act_draw(const float *part, int P, int64_t n, const float *ba, const float *bc, int A, int det,
                           uint64_t seed, const int64_t *epoch, int64_t step, int64_t env_offset, int64_t *action,
                           float *logp, float *value, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if (P < 1 || A < 1 || A > 4) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_act_draw, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<const float4 *>(part), P, n, ba, bc, A, det, seed, epoch, step, env_offset,
                       action, logp, value);
    return hipGetLastError();
}

}  // namespace merlin
