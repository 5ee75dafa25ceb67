// merlin_capi.hip -- host side of libmerlin_hip.so: the extern "C" ABI declared
// in include/merlin_hip.h, env-context lifetime, numpy SeedSequence seeding and
// the library's own restatement of minigrid's tile renderer (the atlas).
#include <math.h>
#include <string.h>

#include <mutex>
#include <string>

#include <algorithm>

#include "merlin_internal.h"

struct merlin_env {
    merlin::EnvDev dev;
    int device;
    bool has_state;
    int steps_since_refill;  // merlin_env_step launches since the last look-ahead refill
    int refill_every;        // 0: the caller launches refills (merlin_env_refill)
    bool no_fallback = false;  // merlin_env_set_step_fallback(0): with refill_every 0, no k_env_fallback pass
    // reseed mode (every reset is reset(seed=task_seed)) after a full reset: every look-ahead slot holds its env's
    // seed map and no reset consumes it, so the periodic refills and the fallback pass would find nothing to do and
    // are left out (an empty slot would still raise MERLIN_DEVERR_SLOT_EMPTY); cleared when merlin_env_seed makes
    // the slots stale (round 6: FOMAML's 32-env task rollouts, two graph nodes fewer per step)
    bool seed_slots_full = false;
};

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

int hip_fail(hipError_t e, const char *what) {
    return fail(MERLIN_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(expr)                                  \
    do {                                               \
        hipError_t _e = (expr);                        \
        if (_e != hipSuccess) return hip_fail(_e, #expr); \
    } while (0)

// ---------------------------------------------------------------------------
// numpy SeedSequence(seed).generate_state(4, uint64) -> PCG64 seeding
// (numpy/random/bit_generator.pyx mix_entropy / generate_state,
//  numpy/random/_pcg64.pyx -> pcg64_set_seed -> pcg_setseq_128_srandom_r).
struct U128 {
    uint64_t hi, lo;
};

U128 mul128(U128 a, U128 b) {
    const unsigned __int128 x = ((unsigned __int128)a.hi << 64) | a.lo;
    const unsigned __int128 y = ((unsigned __int128)b.hi << 64) | b.lo;
    const unsigned __int128 z = x * y;
    return {(uint64_t)(z >> 64), (uint64_t)z};
}

U128 add128(U128 a, U128 b) {
    const unsigned __int128 x = ((unsigned __int128)a.hi << 64) | a.lo;
    const unsigned __int128 y = ((unsigned __int128)b.hi << 64) | b.lo;
    const unsigned __int128 z = x + y;
    return {(uint64_t)(z >> 64), (uint64_t)z};
}

void seed_pcg64(uint64_t seed, U128 &state, U128 &inc) {
    uint32_t ent[2];
    int n = 0;
    if (seed == 0) ent[n++] = 0;
    for (uint64_t s = seed; s; s >>= 32) ent[n++] = (uint32_t)s;
    uint32_t pool[4];
    uint32_t hc = 0x43b0d7e5u;
    auto hashmix = [&hc](uint32_t v) {
        v ^= hc;
        hc *= 0x931e8875u;
        v *= hc;
        v ^= v >> 16;
        return v;
    };
    auto mix = [](uint32_t x, uint32_t y) {
        uint32_t r = 0xca01f9ddu * x - 0x4973f715u * y;
        return r ^ (r >> 16);
    };
    for (int i = 0; i < 4; i++) pool[i] = hashmix(i < n ? ent[i] : 0u);
    for (int s = 0; s < 4; s++)
        for (int d = 0; d < 4; d++)
            if (s != d) pool[d] = mix(pool[d], hashmix(pool[s]));
    uint32_t w[8];
    uint32_t hb = 0x8b51f9ddu;
    for (int i = 0; i < 8; i++) {
        uint32_t v = pool[i & 3] ^ hb;
        hb *= 0x58f38dedu;
        v *= hb;
        w[i] = v ^ (v >> 16);
    }
    const uint64_t v0 = (uint64_t)w[0] | ((uint64_t)w[1] << 32), v1 = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
    const uint64_t v2 = (uint64_t)w[4] | ((uint64_t)w[5] << 32), v3 = (uint64_t)w[6] | ((uint64_t)w[7] << 32);
    const U128 initstate{v0, v1}, initseq{v2, v3};
    inc = {(initseq.hi << 1) | (initseq.lo >> 63), (initseq.lo << 1) | 1u};
    const U128 mult{0x2360ed051fc65da4ULL, 0x4385df649fccf645ULL};
    state = inc;  // step from state 0: 0 * mult + inc
    state = add128(state, initstate);
    state = add128(mul128(state, mult), inc);
}

// ---------------------------------------------------------------------------
// minigrid 3.0.0 Grid.render_tile(obj, agent_dir, highlight, tile_size=8, subdivs=3)
// with minigrid.utils.rendering fill_coords / point_in_rect / point_in_triangle /
// rotate_fn / highlight_img / downsample, keeping numpy's dtypes: float32
// triangle vertices and their dot products, float64 sample points, uint8
// canvas, float64 means, truncating cast into the uint8 frame.
struct Tri {
    float ax, ay, v0x, v0y, v1x, v1y, dot00, dot01, dot11, inv;
    Tri() {
        const float a[2] = {0.12f, 0.19f}, b[2] = {0.87f, 0.50f}, c[2] = {0.12f, 0.81f};
        ax = a[0];
        ay = a[1];
        v0x = c[0] - a[0];
        v0y = c[1] - a[1];
        v1x = b[0] - a[0];
        v1y = b[1] - a[1];
        dot00 = v0x * v0x + v0y * v0y;
        dot01 = v0x * v1x + v0y * v1y;
        dot11 = v1x * v1x + v1y * v1y;
        const float den = dot00 * dot11 - dot01 * dot01;
        inv = 1.0f / den;
    }
    bool in(double x, double y) const {
        const double v2x = x - (double)ax, v2y = y - (double)ay;
        const double dot02 = (double)v0x * v2x + (double)v0y * v2y;
        const double dot12 = (double)v1x * v2x + (double)v1y * v2y;
        const double u = ((double)dot11 * dot02 - (double)dot01 * dot12) * (double)inv;
        const double v = ((double)dot00 * dot12 - (double)dot01 * dot02) * (double)inv;
        return (u >= 0) && (v >= 0) && (u + v) < 1;
    }
};

void render_tile(int obj /*0 none 1 wall 2 goal*/, bool agent, bool highlight, uint8_t out[8][8][3]) {
    static uint8_t img[24][24][3];
    memset(img, 0, sizeof(img));
    auto fill_rect = [](double xmin, double xmax, double ymin, double ymax, const uint8_t col[3]) {
        for (int y = 0; y < 24; y++)
            for (int x = 0; x < 24; x++) {
                const double yf = (y + 0.5) / 24, xf = (x + 0.5) / 24;
                if (xf >= xmin && xf <= xmax && yf >= ymin && yf <= ymax) memcpy(img[y][x], col, 3);
            }
    };
    const uint8_t grey[3] = {100, 100, 100}, green[3] = {0, 255, 0}, red[3] = {255, 0, 0};
    fill_rect(0, 0.031, 0, 1, grey);
    fill_rect(0, 1, 0, 0.031, grey);
    if (obj == 1) fill_rect(0, 1, 0, 1, grey);
    if (obj == 2) fill_rect(0, 1, 0, 1, green);
    if (agent) {
        const Tri tri;
        const double theta = 0.5 * M_PI * 3;  // agent_dir = 3 in get_pov_render
        const double c = cos(-theta), s = sin(-theta);
        for (int y = 0; y < 24; y++)
            for (int x = 0; x < 24; x++) {
                const double yf = (y + 0.5) / 24, xf = (x + 0.5) / 24;
                const double px = xf - 0.5, py = yf - 0.5;
                const double x2 = (0.5 + px * c) - py * s;
                const double y2 = (0.5 + py * c) + px * s;
                if (tri.in(x2, y2)) memcpy(img[y][x], red, 3);
            }
    }
    if (highlight)
        for (int y = 0; y < 24; y++)
            for (int x = 0; x < 24; x++)
                for (int k = 0; k < 3; k++) {
                    const uint8_t p = img[y][x][k];
                    double v = (double)p + 0.30 * (double)(uint8_t)(255 - p);
                    v = v < 0 ? 0 : (v > 255 ? 255 : v);
                    img[y][x][k] = (uint8_t)v;
                }
    for (int Y = 0; Y < 8; Y++)
        for (int X = 0; X < 8; X++)
            for (int k = 0; k < 3; k++) {
                double m[3];
                for (int sy = 0; sy < 3; sy++) {
                    const uint8_t *r0 = img[3 * Y + sy][3 * X];
                    m[sy] = (((double)r0[k] + (double)r0[3 + k]) + (double)r0[6 + k]) / 3.0;
                }
                out[Y][X][k] = (uint8_t)(((m[0] + m[1]) + m[2]) / 3.0);
            }
}

uint8_t g_atlas[MERLIN_OBS_TILES][8][8][3];
std::once_flag g_atlas_once;

void build_atlas() {
    std::call_once(g_atlas_once, [] {
        render_tile(0, false, false, g_atlas[0]);  // not visible: empty, no highlight
        render_tile(0, false, true, g_atlas[1]);   // visible empty
        render_tile(1, false, true, g_atlas[2]);   // visible wall
        render_tile(2, false, true, g_atlas[3]);   // visible goal
        render_tile(0, true, true, g_atlas[4]);    // agent (view cell (3,6), agent_dir 3)
    });
}

// per-device one-time init: atlas upload + GAE partials workspace
struct DeviceWs {
    bool ready = false;
    double *partials = nullptr;
    int max_partials = 0;
    float *conv1_slabs = nullptr;
    int max_slabs = 0;
    void *lut2_slabs = nullptr;  // conv2 table histogram: per-block 4-channel u64 slices
    float *epi_work = nullptr;   // GEMM epilogues: per-block column-sum partials
    double *stage_part = nullptr;  // conv tables' adjoint: the 625-combination type's partial dW2 sums
    uint32_t *tower_err = nullptr;  // device error flags of the tower kernels (merlin_tower_errors)
};
constexpr int MAX_DEV = 64;
DeviceWs g_dev[MAX_DEV];
std::mutex g_dev_mu;
constexpr int WS_PARTIALS = 1 << 16;
constexpr int WS_SLABS = 1024;  // conv1 backward: per-block partial slabs (1024 x 2 towers x 2592 floats)

int device_ws(DeviceWs **out) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    if (dev < 0 || dev >= MAX_DEV) return fail(MERLIN_E_UNSUPPORTED, "device index out of range");
    std::lock_guard<std::mutex> lk(g_dev_mu);
    DeviceWs &w = g_dev[dev];
    if (!w.ready) {
        build_atlas();
        HIP_TRY(merlin::upload_atlas(&g_atlas[0][0][0][0]));
        HIP_TRY(hipMalloc(&w.partials, sizeof(double) * 2 * WS_PARTIALS));
        w.max_partials = WS_PARTIALS;
        HIP_TRY(hipMalloc(&w.conv1_slabs, sizeof(float) * (size_t)WS_SLABS * merlin::conv1_slab_floats(2)));
        w.max_slabs = WS_SLABS;
        HIP_TRY(hipMalloc(&w.lut2_slabs, merlin::conv2_lut_slab_bytes(2, merlin::conv2_lut_fblocks(INT64_MAX / 64))));
        HIP_TRY(hipMalloc(&w.epi_work, sizeof(float) * merlin::epilogue_work_floats()));
        HIP_TRY(hipMalloc(&w.stage_part, sizeof(double) * merlin::STAGE_WS_DOUBLES));
        HIP_TRY(hipMalloc(&w.tower_err, sizeof(uint32_t)));
        HIP_TRY(hipMemset(w.tower_err, 0, sizeof(uint32_t)));  // once, outside any capture
        HIP_TRY(hipDeviceSynchronize());
        w.ready = true;
    }
    *out = &w;
    return MERLIN_OK;
}


// zero_async's kernel: a 16-B aligned body by grid-stride uint4 stores; the unaligned head and the tail (< 16 B each)
// by block 0's first lanes, byte stores
__global__ void k_zero_fill(uint8_t *__restrict__ p, uint32_t head, size_t n16, uint32_t tail) {
    uint4 *v = reinterpret_cast<uint4 *>(p + head);
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256)
        v[i] = make_uint4(0u, 0u, 0u, 0u);
    if (blockIdx.x == 0) {
        if (threadIdx.x < head) p[threadIdx.x] = 0;
        if (threadIdx.x < tail) p[head + n16 * 16 + threadIdx.x] = 0;
    }
}
}  // namespace

hipError_t merlin::zero_async(void *p, size_t bytes, hipStream_t s) {
    if (bytes == 0) return hipSuccess;
    auto *b = static_cast<uint8_t *>(p);
    size_t head = (16 - (reinterpret_cast<uintptr_t>(b) & 15)) & 15;
    if (head > bytes) head = bytes;
    const size_t n16 = (bytes - head) / 16;
    const size_t tail = bytes - head - n16 * 16;
    const int grid = (int)std::max<size_t>(1, std::min<size_t>((n16 + 255) / 256, 2048));
    hipLaunchKernelGGL(k_zero_fill, dim3(grid), dim3(256), 0, s, b, (uint32_t)head, n16, (uint32_t)tail);
    return hipGetLastError();
}

extern "C" {

int merlin_version(void) { return MERLIN_ABI_VERSION; }

const char *merlin_last_error(void) { return g_err.c_str(); }

int merlin_tile_atlas(uint8_t *out_host) {
    if (!out_host) return fail(MERLIN_E_INVALID, "null output");
    build_atlas();
    memcpy(out_host, g_atlas, sizeof(g_atlas));
    return MERLIN_OK;
}

int64_t merlin_env_config_layout(int64_t *offsets_host, int32_t n_fields) {
    const int64_t off[MERLIN_ENV_CONFIG_FIELDS] = {
        (int64_t)offsetof(merlin_env_config, num_envs),     (int64_t)offsetof(merlin_env_config, size),
        (int64_t)offsetof(merlin_env_config, difficulty),   (int64_t)offsetof(merlin_env_config, max_steps),
        (int64_t)offsetof(merlin_env_config, stuck_penalty), (int64_t)offsetof(merlin_env_config, max_stay),
        (int64_t)offsetof(merlin_env_config, penalty),      (int64_t)offsetof(merlin_env_config, exploration_bonus),
        (int64_t)offsetof(merlin_env_config, bonus),        (int64_t)offsetof(merlin_env_config, reseed_each_reset)};
    if (offsets_host)
        for (int i = 0; i < n_fields && i < MERLIN_ENV_CONFIG_FIELDS; i++) offsets_host[i] = off[i];
    return (int64_t)sizeof(merlin_env_config);
}

int merlin_env_create(const merlin_env_config *cfg, merlin_env **out) {
    if (!cfg || !out) return fail(MERLIN_E_INVALID, "null argument");
    *out = nullptr;
    if (cfg->num_envs <= 0) return fail(MERLIN_E_INVALID, "num_envs must be > 0");
    if (cfg->size < 5 || cfg->size > 32)
        return fail(MERLIN_E_UNSUPPORTED, "grid size must be in [5, 32]");
    if (cfg->difficulty < MERLIN_EASY || cfg->difficulty > MERLIN_HARDEST)
        return fail(MERLIN_E_INVALID, "unknown difficulty");
    if (cfg->difficulty == MERLIN_HARDEST && cfg->size < 9)
        return fail(MERLIN_E_UNSUPPORTED, "hardest needs size >= 9 (integers(2, mid-1))");
    if (cfg->difficulty == MERLIN_HARD && cfg->size < 6)
        return fail(MERLIN_E_UNSUPPORTED, "hard needs size >= 6");
    DeviceWs *ws = nullptr;
    int rc = device_ws(&ws);
    if (rc) return rc;
    merlin_env *e = new merlin_env();
    e->refill_every = merlin::REFILL_EVERY;
    merlin::EnvDev &d = e->dev;
    d.n = cfg->num_envs;
    d.size = cfg->size;
    d.sp = cfg->size <= 16 ? 16 : 32;
    d.difficulty = cfg->difficulty;
    d.max_steps = cfg->max_steps > 0 ? cfg->max_steps : 4 * cfg->size * cfg->size;
    d.stuck_on = cfg->stuck_penalty ? 1 : 0;
    d.max_stay = cfg->max_stay > 0 ? cfg->max_stay : 3;
    d.penalty = cfg->penalty;
    d.explore_on = cfg->exploration_bonus ? 1 : 0;
    d.bonus = cfg->bonus;
    d.reseed = cfg->reseed_each_reset ? 1 : 0;
    (void)hipGetDevice(&e->device);
    const size_t n = (size_t)d.n;
    hipError_t err = hipSuccess;
    auto alloc = [&](void **p, size_t bytes) {
        if (err == hipSuccess) err = hipMalloc(p, bytes);
        if (err == hipSuccess) err = hipMemset(*p, 0, bytes);
    };
    alloc((void **)&d.walls, n * d.sp * sizeof(uint32_t));
    alloc((void **)&d.agent, n * sizeof(uint4));
    alloc((void **)&d.rng_s, n * sizeof(ulonglong2));
    alloc((void **)&d.rng_i, n * sizeof(ulonglong2));
    alloc((void **)&d.rng_b, n * sizeof(uint2));
    alloc((void **)&d.ep_ret, n * sizeof(double));
    alloc((void **)&d.ep_len, n * sizeof(int32_t));
    alloc((void **)&d.err, 2 * sizeof(uint32_t));
    alloc((void **)&d.pg_walls, n * d.sp * sizeof(uint32_t));
    alloc((void **)&d.pg_agent, n * sizeof(uint4));
    alloc((void **)&d.pg_rng_s, n * sizeof(ulonglong2));
    alloc((void **)&d.pg_rng_b, n * sizeof(uint2));
    alloc((void **)&d.pg_valid, n * sizeof(uint8_t));
    alloc((void **)&d.rflag, n * sizeof(uint8_t));
    alloc((void **)&d.bflag, (n + 63) / 64);  // one flag per step block (merlin_env.hip SBLK >= 64 envs)
    if (d.explore_on) alloc((void **)&d.visited, n * d.sp * sizeof(uint32_t));
    if (err != hipSuccess) {
        merlin_env_destroy(e);
        return hip_fail(err, "hipMalloc(env state)");
    }
    *out = e;
    return MERLIN_OK;
}

int merlin_env_destroy(merlin_env *e) {
    if (!e) return MERLIN_OK;
    merlin::EnvDev &d = e->dev;
    void *ptrs[] = {d.walls, d.agent, d.rng_s, d.rng_i, d.rng_b, d.ep_ret, d.ep_len, d.err, d.visited,
                    d.pg_walls, d.pg_agent, d.pg_rng_s, d.pg_rng_b, d.pg_valid, d.rflag, d.bflag};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    delete e;
    return MERLIN_OK;
}

int merlin_env_num_envs(const merlin_env *e) { return e ? e->dev.n : -1; }
int merlin_env_size(const merlin_env *e) { return e ? e->dev.size : -1; }

int merlin_env_seed(merlin_env *e, const uint64_t *seeds, int32_t n, void *stream) {
    if (!e || !seeds) return fail(MERLIN_E_INVALID, "null argument");
    if (n != e->dev.n) return fail(MERLIN_E_INVALID, "seed count must equal num_envs");
    hipStream_t s = (hipStream_t)stream;
    const size_t N = (size_t)n;
    ulonglong2 *st = new ulonglong2[N];
    ulonglong2 *inc = new ulonglong2[N];
    for (size_t i = 0; i < N; i++) {
        U128 a, b;
        seed_pcg64(seeds[i], a, b);
        st[i] = make_ulonglong2(a.lo, a.hi);
        inc[i] = make_ulonglong2(b.lo, b.hi);
    }
    hipError_t err = hipMemcpyAsync(e->dev.rng_s, st, N * sizeof(ulonglong2), hipMemcpyHostToDevice, s);
    if (err == hipSuccess)
        err = hipMemcpyAsync(e->dev.rng_i, inc, N * sizeof(ulonglong2), hipMemcpyHostToDevice, s);
    if (err == hipSuccess) err = merlin::zero_async(e->dev.rng_b, N * sizeof(uint2), s);
    if (err == hipSuccess) err = merlin::zero_async(e->dev.pg_valid, N, s);  // look-ahead maps are stale
    e->seed_slots_full = false;
    if (err == hipSuccess) err = hipStreamSynchronize(s);  // host staging buffers are freed below
    delete[] st;
    delete[] inc;
    if (err != hipSuccess) return hip_fail(err, "merlin_env_seed");
    return MERLIN_OK;
}

int merlin_env_reset(merlin_env *e, const uint8_t *mask, uint32_t *obs, void *stream) {
    if (!e) return fail(MERLIN_E_INVALID, "null env");
    HIP_TRY(merlin::launch_env_reset(e->dev, mask, obs, (hipStream_t)stream));  // + look-ahead refill
    e->steps_since_refill = 0;
    if (!mask) {
        e->has_state = true;
        e->seed_slots_full = e->dev.reseed != 0;  // the reset's full refill filled every slot with its seed map
    }
    return MERLIN_OK;
}

int merlin_env_step(merlin_env *e, const int64_t *actions, int32_t n_steps, int64_t action_stride,
                    uint32_t *obs, float *reward, uint8_t *term, uint8_t *trunc, float *done,
                    double *ep_ret, int32_t *ep_len, int32_t autoreset, void *stream) {
    if (!e || !actions) return fail(MERLIN_E_INVALID, "null argument");
    if (!e->has_state) return fail(MERLIN_E_INVALID, "merlin_env_step before merlin_env_reset");
    if (n_steps <= 0) return MERLIN_OK;
    if (action_stride < e->dev.n && n_steps > 1)
        return fail(MERLIN_E_INVALID, "action_stride must be >= num_envs");
    merlin::StepOut o{};
    o.actions = actions;
    o.action_stride = action_stride;
    o.n_steps = n_steps;
    o.autoreset = autoreset;
    o.obs = obs;
    o.reward = reward;
    o.term = term;
    o.trunc = trunc;
    o.done = done;
    o.ep_ret_out = ep_ret;
    o.ep_len_out = ep_len;
    const bool refill = !e->seed_slots_full && e->refill_every > 0 && ++e->steps_since_refill >= e->refill_every;
    if (refill) e->steps_since_refill = 0;
    o.no_fallback = e->seed_slots_full || (e->no_fallback && e->refill_every == 0);
    HIP_TRY(merlin::launch_env_step(e->dev, o, refill, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_env_act_step(merlin_env *e, const float *head_part, int32_t n_parts, const float *b_actor,
                        const float *b_critic, int32_t act_dim, int32_t deterministic, uint64_t seed,
                        const int64_t *epoch, int64_t step, int64_t env_offset, int64_t *action, float *logp,
                        float *value, uint32_t *obs, float *reward, uint8_t *term, uint8_t *trunc, float *done,
                        double *ep_ret, int32_t *ep_len, void *stream) {
    if (!e || !head_part || !b_actor || !b_critic || !action || !logp || !value)
        return fail(MERLIN_E_INVALID, "null argument");
    if (!e->has_state) return fail(MERLIN_E_INVALID, "merlin_env_act_step before merlin_env_reset");
    if (n_parts < 1 || act_dim < 1 || act_dim > 4) return fail(MERLIN_E_INVALID, "n_parts >= 1, act_dim in [1, 4]");
    if (!deterministic && !epoch) return fail(MERLIN_E_INVALID, "a sampled action needs the epoch counter");
    merlin::StepOut o{};
    o.actions = action;
    o.action_stride = e->dev.n;
    o.n_steps = 1;
    o.autoreset = 1;
    o.obs = obs;
    o.reward = reward;
    o.term = term;
    o.trunc = trunc;
    o.done = done;
    o.ep_ret_out = ep_ret;
    o.ep_len_out = ep_len;
    o.act = merlin::ActIn{reinterpret_cast<const float4 *>(head_part), n_parts, b_actor, b_critic, act_dim,
                          deterministic ? 1 : 0, seed, epoch, step, env_offset, action, logp, value};
    const bool refill = !e->seed_slots_full && e->refill_every > 0 && ++e->steps_since_refill >= e->refill_every;
    if (refill) e->steps_since_refill = 0;
    o.no_fallback = e->seed_slots_full || (e->no_fallback && e->refill_every == 0);
    HIP_TRY(merlin::launch_env_step(e->dev, o, refill, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_group_act(const uint32_t *codes, int32_t groups, const float *T2, const float *b2, const float *W3t,
                     const float *b3, const float *W4p, const float *b4, const float *Wa, const float *ba,
                     const float *Wc, const float *bc, int32_t act_dim, float *a3_ws, float *head_part,
                     int32_t shared_weights, void *stream) {
    if (groups < 0) return fail(MERLIN_E_INVALID, "negative group count");
    if (act_dim < 1 || act_dim > 4) return fail(MERLIN_E_INVALID, "act_dim must be in [1, 4]");
    if (groups > 0 && (!codes || !T2 || !b2 || !W3t || !b3 || !W4p || !b4 || !Wa || !ba || !Wc || !bc || !a3_ws ||
                       !head_part))
        return fail(MERLIN_E_INVALID, "null argument");
    HIP_TRY(merlin::launch_group_act(codes, groups, T2, b2, W3t, b3, W4p, b4, Wa, ba, Wc, bc, act_dim, a3_ws,
                                     head_part, shared_weights != 0, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_env_set_step_fallback(merlin_env *e, int32_t on) {
    if (!e) return fail(MERLIN_E_INVALID, "null env");
    e->no_fallback = on == 0;
    return MERLIN_OK;
}

int merlin_env_set_refill_interval(merlin_env *e, int32_t every) {
    if (!e) return fail(MERLIN_E_INVALID, "null env");
    if (every < 0) return fail(MERLIN_E_INVALID, "refill interval must be >= 0");
    e->refill_every = every;
    e->steps_since_refill = 0;
    return MERLIN_OK;
}

int merlin_env_refill(merlin_env *e, void *stream) {
    if (!e) return fail(MERLIN_E_INVALID, "null env");
    HIP_TRY(merlin::launch_env_refill(e->dev, false, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_env_full_obs(merlin_env *e, uint8_t *out, void *stream) {
    if (!e || !out) return fail(MERLIN_E_INVALID, "null argument");
    HIP_TRY(merlin::launch_env_full_obs(e->dev, out, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_env_get_state(merlin_env *e, uint32_t *walls, int32_t *agent, uint64_t *rng, void *stream) {
    if (!e) return fail(MERLIN_E_INVALID, "null env");
    hipStream_t s = (hipStream_t)stream;
    const merlin::EnvDev &d = e->dev;
    const size_t n = (size_t)d.n;
    if (walls) {
        uint32_t *tmp = new uint32_t[n * d.sp];
        hipError_t err = hipMemcpyAsync(tmp, d.walls, n * d.sp * 4, hipMemcpyDeviceToHost, s);
        if (err == hipSuccess) err = hipStreamSynchronize(s);
        if (err == hipSuccess)
            for (size_t i = 0; i < n; i++)
                for (int y = 0; y < d.size; y++) walls[i * d.size + y] = tmp[i * d.sp + y];
        delete[] tmp;
        if (err != hipSuccess) return hip_fail(err, "get_state(walls)");
    }
    if (agent) {
        uint4 *tmp = new uint4[n];
        hipError_t err = hipMemcpyAsync(tmp, d.agent, n * sizeof(uint4), hipMemcpyDeviceToHost, s);
        if (err == hipSuccess) err = hipStreamSynchronize(s);
        if (err == hipSuccess)
            for (size_t i = 0; i < n; i++) {
                int32_t *a = agent + i * 8;
                a[0] = tmp[i].x & 0xff;
                a[1] = (tmp[i].x >> 8) & 0xff;
                a[2] = (tmp[i].x >> 16) & 3;
                a[3] = (int32_t)tmp[i].y;
                a[4] = tmp[i].z & 0xff;
                a[5] = (tmp[i].z >> 8) & 0xff;
                a[6] = (int32_t)(tmp[i].w >> 16);
                a[7] = 0;
            }
        delete[] tmp;
        if (err != hipSuccess) return hip_fail(err, "get_state(agent)");
    }
    if (rng) {
        ulonglong2 *a = new ulonglong2[n], *b = new ulonglong2[n];
        uint2 *c = new uint2[n];
        hipError_t err = hipMemcpyAsync(a, d.rng_s, n * sizeof(ulonglong2), hipMemcpyDeviceToHost, s);
        if (err == hipSuccess) err = hipMemcpyAsync(b, d.rng_i, n * sizeof(ulonglong2), hipMemcpyDeviceToHost, s);
        if (err == hipSuccess) err = hipMemcpyAsync(c, d.rng_b, n * sizeof(uint2), hipMemcpyDeviceToHost, s);
        if (err == hipSuccess) err = hipStreamSynchronize(s);
        if (err == hipSuccess)
            for (size_t i = 0; i < n; i++) {
                uint64_t *r = rng + i * 5;
                r[0] = a[i].y;
                r[1] = a[i].x;
                r[2] = b[i].y;
                r[3] = b[i].x;
                r[4] = ((uint64_t)c[i].x << 32) | c[i].y;
            }
        delete[] a;
        delete[] b;
        delete[] c;
        if (err != hipSuccess) return hip_fail(err, "get_state(rng)");
    }
    return MERLIN_OK;
}

int merlin_env_errors(merlin_env *e, uint32_t *flags, uint32_t *fallbacks, void *stream) {
    if (!e) return fail(MERLIN_E_INVALID, "null env");
    hipStream_t s = (hipStream_t)stream;
    uint32_t h[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(h, e->dev.err, sizeof(h), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    HIP_TRY(merlin::zero_async(e->dev.err, sizeof(h), s));
    if (flags) *flags = h[0];
    if (fallbacks) *fallbacks = h[1];
    return MERLIN_OK;
}

int merlin_obs_expand_f32(const uint32_t *codes, const int64_t *index, int64_t n, float *out, float scale,
                          int32_t layout, void *stream) {
    if ((!codes || !out) && n > 0) return fail(MERLIN_E_INVALID, "null argument");
    if (layout != MERLIN_LAYOUT_NCHW && layout != MERLIN_LAYOUT_NHWC)
        return fail(MERLIN_E_INVALID, "unknown layout");
    DeviceWs *ws = nullptr;
    int rc = device_ws(&ws);
    if (rc) return rc;
    HIP_TRY(merlin::launch_obs_expand_f32(codes, index, n, out, scale, layout, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_obs_expand_u8(const uint32_t *codes, const int64_t *index, int64_t n, uint8_t *out, void *stream) {
    if ((!codes || !out) && n > 0) return fail(MERLIN_E_INVALID, "null argument");
    DeviceWs *ws = nullptr;
    int rc = device_ws(&ws);
    if (rc) return rc;
    HIP_TRY(merlin::launch_obs_expand_u8(codes, index, n, out, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_gae(const float *rew, const float *val, const float *done, const float *last, float *adv,
               float *ret, int32_t T, int32_t N, double gamma, double lam, double *stats, void *stream) {
    if (!rew || !val || !done || !last || !adv || !ret) return fail(MERLIN_E_INVALID, "null argument");
    if (T <= 0 || N <= 0) return fail(MERLIN_E_INVALID, "T and N must be > 0");
    DeviceWs *ws = nullptr;
    int rc = device_ws(&ws);
    if (rc) return rc;
    if (stats && merlin::gae_partials_needed(T, N) > ws->max_partials)
        return fail(MERLIN_E_UNSUPPORTED, "too many envs for the GAE stats workspace");
    HIP_TRY(merlin::launch_gae(rew, val, done, last, adv, ret, T, N, gamma, lam, stats, ws->partials,
                               ws->max_partials, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_adv_normalize(const float *adv, int64_t n, const double *stats, float *out, void *stream) {
    if (!adv || !stats || !out) return fail(MERLIN_E_INVALID, "null argument");
    HIP_TRY(merlin::launch_adv_normalize(adv, n, stats, out, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_conv1_lut_fwd(const uint32_t *codes, const int64_t *index, int64_t n, const float *tables,
                         const float *bias, int32_t towers, float *out, void *stream) {
    if ((!codes || !tables || !bias || !out) && n > 0) return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    HIP_TRY(merlin::launch_conv1_lut_fwd(codes, index, n, tables, bias, towers, out, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_conv1_lut_bwd(const uint32_t *codes, const int64_t *index, int64_t n, const float *act,
                         const float *grad, int32_t towers, float *dtables, float *dbias, void *stream) {
    if (!dtables || !dbias || ((!codes || !act || !grad) && n > 0)) return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    DeviceWs *ws = nullptr;
    int rc = device_ws(&ws);
    if (rc) return rc;
    HIP_TRY(merlin::launch_conv1_lut_bwd(codes, index, n, act, grad, towers, dtables, dbias, ws->conv1_slabs,
                                         ws->max_slabs, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_tower_conv2_im2col_fwd(const uint32_t *codes, const int64_t *index, int64_t n, const float *tables,
                                  const float *bias, int32_t towers, float *A2, void *stream) {
    if ((!codes || !tables || !bias || !A2) && n > 0) return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    HIP_TRY(merlin::launch_conv1_im2col_fwd(codes, index, n, tables, bias, towers, A2, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_tower_conv2_im2col_bwd(const uint32_t *codes, const int64_t *index, int64_t n, const float *tables,
                                  const float *bias, const float *dA2, int32_t towers, float *dtables,
                                  float *dbias, void *stream) {
    if (!dtables || !dbias || ((!codes || !tables || !bias || !dA2) && n > 0))
        return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    DeviceWs *ws = nullptr;
    int rc = device_ws(&ws);
    if (rc) return rc;
    HIP_TRY(merlin::launch_conv1_im2col_bwd(codes, index, n, tables, bias, dA2, towers, dtables, dbias,
                                            ws->conv1_slabs, ws->max_slabs, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_tower_conv3_im2col_fwd(const float *Z2, const float *b2, int64_t n, int32_t towers, float *A3,
                                  void *stream) {
    if ((!Z2 || !b2 || !A3) && n > 0) return fail(MERLIN_E_INVALID, "null argument");
    HIP_TRY(merlin::launch_im2col3_fwd(Z2, b2, n, towers, A3, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_tower_conv3_col2im_bwd(const float *dA3, const float *Z2, const float *b2, int64_t n, int32_t towers,
                                  float *dZ2, void *stream) {
    if ((!dA3 || !Z2 || !b2 || !dZ2) && n > 0) return fail(MERLIN_E_INVALID, "null argument");
    HIP_TRY(merlin::launch_col2im3_bwd(dA3, Z2, b2, n, towers, 0, dZ2, nullptr, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_tower_conv3_col2im_bwd_chunked(const float *dA3, const float *Z2, const float *b2, int64_t n,
                                          int32_t towers, float *dZ2c, uint32_t *absmax, void *stream) {
    if (!absmax || ((!dA3 || !Z2 || !b2 || !dZ2c) && n > 0)) return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1) return fail(MERLIN_E_INVALID, "towers must be >= 1");
    HIP_TRY(merlin::launch_col2im3_bwd(dA3, Z2, b2, n, towers, 1, dZ2c, absmax, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_tower_conv2_lut_rows(void) { return merlin::conv2_lut_rows(); }

int merlin_tower_conv2_lut_fwd(const uint32_t *codes, const int64_t *index, int64_t n, const float *tables,
                               int32_t towers, float *Z2, void *stream) {
    if ((!codes || !tables || !Z2) && n > 0) return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    HIP_TRY(merlin::launch_conv2_lut_fwd(codes, index, n, tables, towers, Z2, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_tower_conv2_lut_bwd(const uint32_t *codes, int64_t n, const float *dZ2c, const uint32_t *absmax,
                               int32_t towers, float *dtables, void *stream) {
    if (!dtables || ((!codes || !dZ2c || !absmax) && n > 0)) return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    DeviceWs *ws = nullptr;
    int rc = device_ws(&ws);
    if (rc) return rc;
    HIP_TRY(merlin::launch_conv2_lut_bwd(codes, n, dZ2c, absmax, towers, dtables, ws->lut2_slabs,
                                         (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_tower_conv2_lut_fwd_grouped(const uint32_t *codes, int64_t n, int64_t group_frames, const float *tables,
                                       int32_t towers, float *Z2, void *stream) {
    if ((!codes || !tables || !Z2) && n > 0) return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 2 || towers % 2 || group_frames <= 0) return fail(MERLIN_E_INVALID, "bad grouping");
    if (n != (int64_t)(towers / 2) * group_frames) return fail(MERLIN_E_INVALID, "n != groups * group_frames");
    HIP_TRY(merlin::launch_conv2_lut_fwd(codes, nullptr, n, tables, towers, Z2, (hipStream_t)stream, group_frames));
    return MERLIN_OK;
}

int64_t merlin_tower_conv2_lut_slab_bytes(int32_t towers, int64_t group_frames) {
    return (int64_t)merlin::conv2_lut_slab_bytes(towers, merlin::conv2_lut_fblocks(group_frames));
}

int merlin_tower_conv2_lut_bwd_grouped(const uint32_t *codes, int64_t group_frames, const float *dZ2c,
                                       const uint32_t *absmax, int32_t towers, float *dtables, void *slabs,
                                       void *stream) {
    if (!dtables || ((!codes || !dZ2c || !absmax || !slabs) && group_frames > 0))
        return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 2 || towers % 2) return fail(MERLIN_E_INVALID, "bad grouping");
    HIP_TRY(merlin::launch_conv2_lut_bwd(codes, group_frames, dZ2c, absmax, towers, dtables, slabs,
                                         (hipStream_t)stream, group_frames));
    return MERLIN_OK;
}

int merlin_tower_window_lut(const int32_t *rows, int64_t nw, const float *tables, int32_t towers, float *Z2w,
                            void *stream) {
    if ((!rows || !tables || !Z2w) && nw > 0) return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    HIP_TRY(merlin::launch_window_lut(rows, nw, tables, towers, Z2w, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_minibatch_patch_maps(const int32_t *kid, const int64_t *group_keys, int64_t n_groups, int64_t n_frames,
                                const int64_t *group_offsets, int32_t n_patches, int32_t *kmap, int32_t *rmap,
                                int32_t *rep_row, void *stream) {
    if (n_groups < 0 || n_frames < 1 || n_patches < 1) return fail(MERLIN_E_INVALID, "bad shape");
    if (n_groups > 0 && (!kid || !group_keys || !group_offsets || !kmap || !rmap || !rep_row))
        return fail(MERLIN_E_INVALID, "null argument");
    if (n_groups * 9 > INT32_MAX) return fail(MERLIN_E_UNSUPPORTED, "more than 2^31 rows");
    HIP_TRY(merlin::launch_patch_maps(kid, group_keys, n_groups, n_frames, group_offsets, n_patches, kmap, rmap,
                                      rep_row, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_tower_window_lut_bias_relu(const int32_t *rows, int64_t nw, const float *tables, int32_t towers,
                                      const float *b2, float *a2w, void *stream) {
    if ((!rows || !tables || !a2w || !b2) && nw > 0) return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    HIP_TRY(merlin::launch_window_lut(rows, nw, tables, towers, a2w, (hipStream_t)stream, b2));
    return MERLIN_OK;
}

int merlin_tower_window_conv3(const float *Q, int64_t nw, const int32_t *wid, const int64_t *groups, int64_t n,
                              const float *b3, int32_t towers, float *Y3, void *stream) {
    if ((!Q || !wid || !b3 || !Y3) && n > 0) return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    HIP_TRY(merlin::launch_window_conv3(Q, nw, wid, groups, n, b3, towers, Y3, nullptr, nullptr, nullptr, 0,
                                        (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_tower_window_conv3_bits(const float *Q, int64_t nw, const int32_t *wid, const int64_t *groups, int64_t n,
                                   const float *b3, int32_t towers, float *Y3, uint64_t *relu_bits, uint32_t *amax,
                                   void *stream) {
    if ((!Q || !wid || !b3 || !Y3 || !relu_bits) && n > 0) return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    HIP_TRY(merlin::launch_window_conv3(Q, nw, wid, groups, n, b3, towers, Y3, relu_bits, amax, nullptr, 0,
                                        (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_tower_window_conv3_reuse(const float *Q, int64_t nw, const int32_t *wid, const int64_t *groups, int64_t n,
                                    const float *b3, int32_t towers, float *Y3, uint64_t *relu_bits, uint32_t *amax,
                                    const int32_t *rep_row, int32_t copy, void *stream) {
    if ((!rep_row || !Y3 || (!(copy & 4) && (!Q || !wid || !b3))) && n > 0)
        return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    if (copy < 0 || copy > 7) return fail(MERLIN_E_INVALID, "copy must be 0..7");
    HIP_TRY(merlin::launch_window_conv3(Q, nw, wid, groups, n, b3, towers, Y3, relu_bits, amax, rep_row, copy,
                                        (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_tower_window_conv3_planes(const float *Q, int64_t nw, const int32_t *wid, const int64_t *groups, int64_t n,
                                     const float *b3, int32_t towers, void *Y3_planes, uint64_t *relu_bits,
                                     const int32_t *rep_row, uint32_t *colmax_ws, uint32_t *bound, void *stream) {
    if ((!rep_row || !Y3_planes || !Q || !wid || !b3 || !relu_bits || !colmax_ws || !bound) && n > 0)
        return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    if (n > 0 && nw <= 0) return fail(MERLIN_E_INVALID, "no windows");
    HIP_TRY(merlin::launch_window_conv3(Q, nw, wid, groups, n, b3, towers, static_cast<float *>(Y3_planes), relu_bits,
                                        nullptr, rep_row, 0, (hipStream_t)stream, colmax_ws, bound));
    return MERLIN_OK;
}

int64_t merlin_tower_all_windows(void) { return 458752; }  // 4^9 + 3 * 4^8 (merlin_window.hip k_codes_conv3)

int merlin_tower_codes_conv3_amax(const uint32_t *codes, int64_t n, const float *Qall, const float *b3,
                                  int32_t towers, float *Y3, uint32_t *amax, void *stream) {
    if ((!codes || !Qall || !b3 || !Y3) && n > 0) return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    DeviceWs *ws = nullptr;
    if (int r = device_ws(&ws)) return r;
    HIP_TRY(merlin::launch_codes_conv3(codes, n, Qall, b3, towers, Y3, amax, ws->tower_err, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_tower_errors(uint32_t *flags, void *stream) {
    DeviceWs *ws = nullptr;
    if (int r = device_ws(&ws)) return r;
    hipStream_t s = (hipStream_t)stream;
    uint32_t h = 0;
    HIP_TRY(hipMemcpyAsync(&h, ws->tower_err, sizeof(h), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    HIP_TRY(merlin::zero_async(ws->tower_err, sizeof(h), s));
    if (flags) *flags = h;
    return MERLIN_OK;
}

int merlin_tower_codes_conv3(const uint32_t *codes, int64_t n, const float *Qall, const float *b3, int32_t towers,
                             float *Y3, void *stream) {
    return merlin_tower_codes_conv3_amax(codes, n, Qall, b3, towers, Y3, nullptr, stream);
}

static int segment_sum_fused(const float *src, const void *mask, int64_t src_rows, const int32_t *idx,
                             const int32_t *key, int64_t nnz, const int32_t *slot, int32_t sub, int64_t item_len,
                             const int32_t *fix, int64_t n_fix, int32_t towers, float *out, int64_t out_rows,
                             float *carry, int32_t flags, int32_t *mark, const int32_t *head_fix, int32_t *counters,
                             const int32_t *mask_rows, void *stream) {
    if (!out && out_rows > 0) return fail(MERLIN_E_INVALID, "null output");
    if (nnz > 0 && (!src || !idx || !key || !carry)) return fail(MERLIN_E_INVALID, "null argument");
    if (n_fix > 0 && !fix) return fail(MERLIN_E_INVALID, "null fix-up list");
    if ((head_fix == nullptr) != (counters == nullptr)) return fail(MERLIN_E_INVALID, "head_fix and counters go together");
    if (counters && nnz > 0 && n_fix != (nnz + item_len - 1) / item_len)
        return fail(MERLIN_E_INVALID, "in-launch fix-ups need one fix row per item");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    if (item_len <= 0 || sub <= 0) return fail(MERLIN_E_INVALID, "item_len and sub must be > 0");
    if (flags & ~(MERLIN_SEG_ACCUMULATE | MERLIN_SEG_NO_FILL | MERLIN_SEG_MASK_BITS | MERLIN_SEG_ROLE_MASK))
        return fail(MERLIN_E_INVALID, "unknown flags");
    HIP_TRY(merlin::launch_seg_sum(src, mask, (flags & MERLIN_SEG_MASK_BITS) ? 1 : 0, src_rows, idx, key, nnz, slot,
                                   sub, item_len, fix, n_fix, towers, out, out_rows, carry,
                                   (flags & MERLIN_SEG_ACCUMULATE) ? 1 : 0, (flags & MERLIN_SEG_NO_FILL) ? 0 : 1,
                                   (flags & MERLIN_SEG_ROLE_MASK) >> MERLIN_SEG_ROLE_SHIFT, mark, head_fix, counters,
                                   (hipStream_t)stream, mask_rows));
    return MERLIN_OK;
}

int merlin_segment_sum_fused(const float *src, const void *mask, int64_t src_rows, const int32_t *idx,
                             const int32_t *key, int64_t nnz, const int32_t *slot, int32_t sub, int64_t item_len,
                             const int32_t *fix, int64_t n_fix, int32_t towers, float *out, int64_t out_rows,
                             float *carry, int32_t flags, int32_t *mark, const int32_t *head_fix, int32_t *counters,
                             void *stream) {
    return segment_sum_fused(src, mask, src_rows, idx, key, nnz, slot, sub, item_len, fix, n_fix, towers, out,
                             out_rows, carry, flags, mark, head_fix, counters, nullptr, stream);
}

int merlin_segment_sum_mask_rows(const float *src, const void *mask, int64_t src_rows, const int32_t *idx,
                                 const int32_t *key, int64_t nnz, const int32_t *slot, int32_t sub, int64_t item_len,
                                 const int32_t *fix, int64_t n_fix, int32_t towers, float *out, int64_t out_rows,
                                 float *carry, int32_t flags, int32_t *mark, const int32_t *head_fix,
                                 int32_t *counters, const int32_t *mask_rows, void *stream) {
    if (nnz > 0 && (!mask || !mask_rows || !(flags & MERLIN_SEG_MASK_BITS)))
        return fail(MERLIN_E_INVALID, "mask_rows needs MERLIN_SEG_MASK_BITS words");
    return segment_sum_fused(src, mask, src_rows, idx, key, nnz, slot, sub, item_len, fix, n_fix, towers, out,
                             out_rows, carry, flags, mark, head_fix, counters, mask_rows, stream);
}

int merlin_segment_sum_marked(const float *src, const void *mask, int64_t src_rows, const int32_t *idx,
                              const int32_t *key, int64_t nnz, const int32_t *slot, int32_t sub, int64_t item_len,
                              const int32_t *fix, int64_t n_fix, int32_t towers, float *out, int64_t out_rows,
                              float *carry, int32_t flags, int32_t *mark, void *stream) {
    return merlin_segment_sum_fused(src, mask, src_rows, idx, key, nnz, slot, sub, item_len, fix, n_fix, towers, out,
                                    out_rows, carry, flags, mark, nullptr, nullptr, stream);
}

int merlin_segment_sum_masked(const float *src, const void *mask, int64_t src_rows, const int32_t *idx,
                              const int32_t *key, int64_t nnz, const int32_t *slot, int32_t sub, int64_t item_len,
                              const int32_t *fix, int64_t n_fix, int32_t towers, float *out, int64_t out_rows,
                              float *carry, int32_t flags, void *stream) {
    return merlin_segment_sum_marked(src, mask, src_rows, idx, key, nnz, slot, sub, item_len, fix, n_fix, towers, out,
                                     out_rows, carry, flags, nullptr, stream);
}

int merlin_segment_sum(const float *src, int64_t src_rows, const int32_t *idx, const int32_t *key, int64_t nnz,
                       const int32_t *slot, int32_t sub, int64_t item_len, const int32_t *fix, int64_t n_fix,
                       int32_t towers, float *out, int64_t out_rows, float *carry, int32_t accumulate,
                       void *stream) {
    return merlin_segment_sum_masked(src, nullptr, src_rows, idx, key, nnz, slot, sub, item_len, fix, n_fix, towers,
                                     out, out_rows, carry, accumulate ? MERLIN_SEG_ACCUMULATE : 0, stream);
}

int merlin_act_heads(const float *z, const float *b4, int64_t n, int32_t hidden, const float *w_actor,
                     const float *b_actor, const float *w_critic, const float *b_critic, int32_t act_dim,
                     int32_t deterministic, uint64_t seed, const int64_t *epoch, int64_t step, int64_t env_offset,
                     int64_t *action, float *logp, float *value, void *stream) {
    if (n < 0) return fail(MERLIN_E_INVALID, "negative size");
    if (act_dim < 1 || act_dim > 8) return fail(MERLIN_E_INVALID, "act_dim must be in [1, 8]");
    if (hidden <= 0 || hidden % 4) return fail(MERLIN_E_INVALID, "hidden must be a positive multiple of 4");
    if (n > 0 && (!z || !b4 || !w_actor || !b_actor || !w_critic || !b_critic || !action || !logp || !value))
        return fail(MERLIN_E_INVALID, "null argument");
    HIP_TRY(merlin::launch_act_heads(z, b4, n, hidden, w_actor, b_actor, w_critic, b_critic, act_dim,
                                     deterministic ? 1 : 0, seed, epoch, step, env_offset, action, logp, value,
                                     (hipStream_t)stream));
    return MERLIN_OK;
}

int64_t merlin_ppo_loss_workspace(int64_t n_samples) { return merlin::ppo_loss_workspace_doubles(n_samples); }

int merlin_ppo_loss(const float *logits, const float *value, const float *bias_actor, const float *bias_critic,
                    int64_t n_frames, int32_t act_dim, const int32_t *offs, const int32_t *order,
                    const int64_t *frame_of, int64_t n_samples, const int64_t *sample_index, const int64_t *actions,
                    const float *logp_old, const float *adv, const float *ret, double clip_eps, double vf_coef,
                    double ent_coef, float *dlogits, float *dvalue, float *dbias_actor, float *dbias_critic,
                    float *loss, double *stats, double *workspace, void *stream) {
    return merlin_ppo_loss_absmax(logits, value, bias_actor, bias_critic, n_frames, act_dim, offs, order, frame_of,
                                  n_samples, sample_index, actions, logp_old, adv, ret, clip_eps, vf_coef, ent_coef,
                                  dlogits, dvalue, dbias_actor, dbias_critic, loss, stats, workspace, nullptr, stream);
}

int merlin_ppo_loss_absmax(const float *logits, const float *value, const float *bias_actor, const float *bias_critic,
                           int64_t n_frames, int32_t act_dim, const int32_t *offs, const int32_t *order,
                           const int64_t *frame_of, int64_t n_samples, const int64_t *sample_index,
                           const int64_t *actions, const float *logp_old, const float *adv, const float *ret,
                           double clip_eps, double vf_coef, double ent_coef, float *dlogits, float *dvalue,
                           float *dbias_actor, float *dbias_critic, float *loss, double *stats, double *workspace,
                           uint32_t *grad_absmax, void *stream) {
    if (n_frames < 0 || n_samples < 0) return fail(MERLIN_E_INVALID, "negative size");
    if (n_frames > n_samples) return fail(MERLIN_E_INVALID, "every frame needs at least one sample");
    if (act_dim < 1 || act_dim > 8) return fail(MERLIN_E_INVALID, "act_dim must be in [1, 8]");
    if (!workspace) return fail(MERLIN_E_INVALID, "null workspace");
    if (n_frames > 0 && (!logits || !value || !offs || !dlogits || !dvalue))
        return fail(MERLIN_E_INVALID, "null argument");
    if (n_samples > 0 && (!order || !frame_of || !actions || !logp_old || !adv || !ret))
        return fail(MERLIN_E_INVALID, "null argument");
    if (n_samples > INT32_MAX) return fail(MERLIN_E_INVALID, "n_samples exceeds int32");
    HIP_TRY(merlin::launch_ppo_loss(logits, value, bias_actor, bias_critic, n_frames, act_dim, offs, order, frame_of,
                                    n_samples, sample_index, actions, logp_old, adv, ret, clip_eps, vf_coef, ent_coef,
                                    dlogits, dvalue, dbias_actor, dbias_critic, loss, stats, workspace,
                                    (hipStream_t)stream, grad_absmax));
    return MERLIN_OK;
}

int merlin_tower_bias_relu(float *z, const float *bias, int64_t rows, int32_t cols, int32_t towers, void *stream) {
    if ((!z || !bias) && rows > 0) return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    if (cols <= 0 || cols % 4) return fail(MERLIN_E_INVALID, "cols must be a positive multiple of 4");
    HIP_TRY(merlin::launch_bias_relu(z, bias, rows, cols, towers, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_tower_relu_bwd(const float *y, const float *dy, float *dz, int64_t rows, int32_t cols, int32_t towers,
                          float *dbias, void *stream) {
    if (!dbias || ((!y || !dy || !dz) && rows > 0)) return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    if (!merlin::epilogue_cols_ok(cols)) return fail(MERLIN_E_UNSUPPORTED, "cols must be 4 x a divisor of 256");
    DeviceWs *ws = nullptr;
    int rc = device_ws(&ws);
    if (rc) return rc;
    HIP_TRY(merlin::launch_relu_bwd_colsum(y, dy, dz, rows, cols, towers, dbias, ws->epi_work, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_tower_colsum(const float *x, int64_t rows, int32_t cols, int64_t row_stride, int64_t tower_stride,
                        int32_t towers, float *out, void *stream) {
    if (!out || (!x && rows > 0)) return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    if (!merlin::epilogue_cols_ok(cols)) return fail(MERLIN_E_UNSUPPORTED, "cols must be 4 x a divisor of 256");
    if (row_stride < cols || row_stride % 4 || tower_stride % 4) return fail(MERLIN_E_INVALID, "bad strides");
    DeviceWs *ws = nullptr;
    int rc = device_ws(&ws);
    if (rc) return rc;
    HIP_TRY(merlin::launch_colsum(x, rows, cols, row_stride, tower_stride, towers, out, ws->epi_work,
                                  (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_tower_head_bwd(const float *h, const float *dlogits, const float *dvalue, const float *w_actor,
                          const float *w_critic, int64_t n, int32_t hidden, int32_t act_dim, float *dz, float *dbias,
                          float *dw_actor, float *dw_critic, uint32_t *amax, void *stream) {
    if (!dbias || !dw_actor || !dw_critic || ((!h || !dlogits || !dvalue || !w_actor || !w_critic || !dz) && n > 0))
        return fail(MERLIN_E_INVALID, "null argument");
    if (act_dim < 1 || act_dim > merlin::epilogue_max_act()) return fail(MERLIN_E_UNSUPPORTED, "act_dim must be 1..8");
    if (!merlin::epilogue_cols_ok(hidden)) return fail(MERLIN_E_UNSUPPORTED, "hidden must be 4 x a divisor of 256");
    DeviceWs *ws = nullptr;
    int rc = device_ws(&ws);
    if (rc) return rc;
    HIP_TRY(merlin::launch_head_bwd(h, dlogits, dvalue, w_actor, w_critic, n, hidden, act_dim, dz, dbias, dw_actor,
                                    dw_critic, ws->epi_work, amax, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_tower_head_bwd_planes(const float *h, const float *dlogits, const float *dvalue, const float *w_actor,
                                 const float *w_critic, int64_t n, int32_t hidden, int32_t act_dim, void *dz_planes,
                                 float *dbias, float *dw_actor, float *dw_critic, const uint32_t *grad_absmax,
                                 uint32_t *dz_bound, void *stream) {
    if (!dbias || !dw_actor || !dw_critic || !grad_absmax || !dz_bound ||
        ((!h || !dlogits || !dvalue || !w_actor || !w_critic || !dz_planes) && n > 0))
        return fail(MERLIN_E_INVALID, "null argument");
    if (act_dim < 1 || act_dim > 8) return fail(MERLIN_E_UNSUPPORTED, "act_dim must be 1..8");
    if (!merlin::epilogue_cols_ok(hidden) || hidden % 8) return fail(MERLIN_E_UNSUPPORTED, "hidden must be 8 x a divisor of 128");
    DeviceWs *ws = nullptr;
    int rc = device_ws(&ws);
    if (rc) return rc;
    HIP_TRY(merlin::launch_head_bwd(h, dlogits, dvalue, w_actor, w_critic, n, hidden, act_dim, nullptr, dbias,
                                    dw_actor, dw_critic, ws->epi_work, dz_bound, (hipStream_t)stream, grad_absmax,
                                    dz_planes));
    return MERLIN_OK;
}

int merlin_tower_heads_fwd(const float *h, int64_t n, int32_t hidden, const float *w_actor, int32_t act_dim,
                           const float *w_critic, const float *b_actor, const float *b_critic, float *logits,
                           float *value, void *stream) {
    if ((!h || !w_actor || !w_critic || !logits || !value) && n > 0) return fail(MERLIN_E_INVALID, "null argument");
    if (n < 0) return fail(MERLIN_E_INVALID, "n must be >= 0");
    if (act_dim < 1 || act_dim > merlin::epilogue_max_act()) return fail(MERLIN_E_UNSUPPORTED, "act_dim must be 1..8");
    if (hidden != 512) return fail(MERLIN_E_UNSUPPORTED, "hidden must be 512");
    HIP_TRY(merlin::launch_heads_fwd(h, n, hidden, w_actor, act_dim, w_critic, b_actor, b_critic, logits, value,
                                     (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_x6_split(const float *x, int64_t n, void *planes, void *stream) {
    if ((!x || !planes) && n > 0) return fail(MERLIN_E_INVALID, "null argument");
    if (n < 0 || n % 8) return fail(MERLIN_E_INVALID, "n must be a non-negative multiple of 8");
    HIP_TRY(merlin::launch_x6_split(x, n, planes, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_stage_tables_fwd(const float *W1, const float *b1, const float *W2, const float *atlas, const int16_t *idx,
                            int32_t towers, float *HT, float *T2, void *stream) {
    if (!W1 || !b1 || !W2 || !atlas || !idx || !HT || !T2) return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    HIP_TRY(merlin::launch_stage_fwd(W1, b1, W2, atlas, idx, towers, HT, T2, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_stage_tables_bwd(const float *W2, const float *HT, const float *dT2, const float *atlas,
                            const int16_t *koff, const int16_t *kv, int32_t towers, float *dH, float *dW1, float *db1,
                            float *dW2, void *stream) {
    if (!W2 || !HT || !dT2 || !atlas || !koff || !kv || !dH || !dW1 || !db1 || !dW2)
        return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    DeviceWs *ws = nullptr;
    int rc = device_ws(&ws);
    if (rc != MERLIN_OK) return rc;
    HIP_TRY(merlin::launch_stage_bwd(W2, HT, dT2, atlas, koff, kv, towers, dH, dW1, db1, dW2, ws->stage_part,
                                     (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_window_gemm_fwd(const float *a2w, const float *W3r, int32_t towers, int64_t nw, float *Q, void *stream) {
    if (!a2w || !W3r || !Q) return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    if (nw < 0) return fail(MERLIN_E_INVALID, "nw must be >= 0");
    HIP_TRY(merlin::launch_winfwd(a2w, W3r, towers, nw, Q, (hipStream_t)stream));
    return MERLIN_OK;
}

int64_t merlin_window_gemm_bwd_work(int32_t towers, int64_t nw) {
    if (towers < 1 || towers > 2 || nw <= 0) return -1;
    return merlin::winbwd_work_floats(towers, nw);
}

int merlin_window_gemm_bwd(const float *a2w, const float *dQ, const float *W3r, int32_t towers, int64_t nw,
                           float *da2w, float *db2, float *dW3r, float *db3, float *work, int64_t work_floats,
                           void *stream) {
    if (!a2w || !dQ || !W3r || !da2w || !db2 || !dW3r || !work) return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    if (nw <= 0) return fail(MERLIN_E_INVALID, "nw must be > 0");
    if (work_floats < merlin::winbwd_work_floats(towers, nw)) return fail(MERLIN_E_INVALID, "work too small");
    HIP_TRY(merlin::launch_winbwd(a2w, dQ, W3r, towers, nw, da2w, db2, dW3r, work, (hipStream_t)stream, db3));
    return MERLIN_OK;
}

int merlin_x6_join(const void *planes, int64_t n, float *x, void *stream) {
    if ((!x || !planes) && n > 0) return fail(MERLIN_E_INVALID, "null argument");
    if (n < 0 || n % 8) return fail(MERLIN_E_INVALID, "n must be a non-negative multiple of 8");
    HIP_TRY(merlin::launch_x6_join(planes, n, x, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_x6_gemm_nt(const float *A, const void *B, int64_t M, int32_t N, int32_t K, int32_t towers, int64_t a_stride,
                      int64_t b_stride, const float *bias, float *C, int64_t c_stride, int32_t cfg, void *stream) {
    if (M < 0 || N <= 0 || K <= 0) return fail(MERLIN_E_INVALID, "bad shape");
    if (M > 0 && (!A || !B || !C)) return fail(MERLIN_E_INVALID, "null argument");
    if (K % 32) return fail(MERLIN_E_UNSUPPORTED, "K must be a multiple of 32");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    if (a_stride % 4 || b_stride % 8) return fail(MERLIN_E_INVALID, "tower strides: A multiple of 4, B of 8");
    const hipError_t e = merlin::launch_x6_gemm_nt(A, B, M, N, K, towers, a_stride, b_stride, bias, C, c_stride, cfg,
                                                   (hipStream_t)stream);
    if (e == hipErrorInvalidValue) return fail(MERLIN_E_UNSUPPORTED, "N not a multiple of the tile width / bad cfg");
    HIP_TRY(e);
    return MERLIN_OK;
}

int64_t merlin_x6_tn_slab_floats(int32_t M, int32_t N, int32_t towers, int32_t splits) {
    return (int64_t)std::max(1, splits) * towers * M * N;
}

int merlin_x6_gemm_tn(const float *A, const float *B, int64_t Kd, int32_t M, int32_t N, int32_t towers, int64_t a_stride,
                      int64_t b_stride, int32_t splits, float *slab, float *out, int32_t cfg, void *stream) {
    if (Kd < 0 || M <= 0 || N <= 0) return fail(MERLIN_E_INVALID, "bad shape");
    if (!out || (Kd > 0 && (!A || !B || !slab))) return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    if (splits < 1 || splits > merlin::x6_tn_max_splits()) return fail(MERLIN_E_INVALID, "splits out of range");
    if (M % 8 || N % 8 || a_stride % 4 || b_stride % 4) return fail(MERLIN_E_INVALID, "M, N: multiples of 8");
    const hipError_t e = merlin::launch_x6_gemm_tn(A, B, Kd, M, N, towers, a_stride, b_stride, splits, slab, out, cfg,
                                                   (hipStream_t)stream);
    if (e == hipErrorInvalidValue) return fail(MERLIN_E_UNSUPPORTED, "M / N not multiples of the tile / bad cfg");
    HIP_TRY(e);
    return MERLIN_OK;
}

int merlin_h3_amax(const float *x, int64_t n, int32_t towers, int64_t stride, uint32_t *amax, void *stream) {
    if (!amax || (n > 0 && !x)) return fail(MERLIN_E_INVALID, "null argument");
    // n == 0: zero amax[0 .. towers) only (any count up to 2^20: a rollout's per-step scales at once)
    if (towers < 1 || (n > 0 && towers > 2) || towers > (1 << 20))
        return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    if (n < 0 || n % 4 || stride % 4 || (towers > 1 && stride < n)) return fail(MERLIN_E_INVALID, "n, stride: multiples of 4");
    HIP_TRY(merlin::launch_h3_amax(x, n, towers, stride, amax, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_h3_split(const float *x, int64_t n, int32_t towers, const uint32_t *amax, void *planes, void *stream) {
    if ((!x || !planes || !amax) && n > 0) return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    if (n < 0 || n % 8) return fail(MERLIN_E_INVALID, "n must be a non-negative multiple of 8");
    HIP_TRY(merlin::launch_h3_split(x, n, towers, amax, planes, (hipStream_t)stream));
    return MERLIN_OK;
}

static int h3_gemm_nt(const float *A, const uint32_t *amax_a, const void *B, const uint32_t *amax_b, int64_t M,
                      int32_t N, int32_t K, int32_t towers, int64_t a_stride, int64_t b_stride, const float *bias,
                      float *C, int64_t c_stride, void *a_planes, const int32_t *a_rows, int32_t cfg, void *stream,
                      const float *head_w0 = nullptr, int32_t n_actions = 0, const float *head_w1 = nullptr,
                      float *head_part = nullptr, bool a_is_planes = false) {
    if (M < 0 || N <= 0 || K <= 0) return fail(MERLIN_E_INVALID, "bad shape");
    if (M > 0 && (!A || !B || (!C && !head_part) || !amax_a || !amax_b)) return fail(MERLIN_E_INVALID, "null argument");
    if (K % 32) return fail(MERLIN_E_UNSUPPORTED, "K must be a multiple of 32");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    if (a_stride % 4 || b_stride % 8) return fail(MERLIN_E_INVALID, "tower strides: A multiple of 4, B of 8");
    const hipError_t e = merlin::launch_h3_gemm_nt(A, amax_a, B, amax_b, M, N, K, towers, a_stride, b_stride, bias, C,
                                                   c_stride, a_planes, cfg, (hipStream_t)stream, a_rows, head_w0,
                                                   n_actions, head_w1, head_part, a_is_planes);
    if (e == hipErrorInvalidValue)
        return fail(MERLIN_E_UNSUPPORTED, "N not a multiple of the tile width / bad cfg / unsupported gather");
    HIP_TRY(e);
    return MERLIN_OK;
}

int merlin_h3_gemm_nt(const float *A, const uint32_t *amax_a, const void *B, const uint32_t *amax_b, int64_t M,
                      int32_t N, int32_t K, int32_t towers, int64_t a_stride, int64_t b_stride, const float *bias,
                      float *C, int64_t c_stride, void *a_planes, int32_t cfg, void *stream) {
    return h3_gemm_nt(A, amax_a, B, amax_b, M, N, K, towers, a_stride, b_stride, bias, C, c_stride, a_planes, nullptr,
                      cfg, stream);
}

int merlin_h3_gemm_nt_planes(const void *A_planes, const uint32_t *amax_a, const void *B, const uint32_t *amax_b,
                             int64_t M, int32_t N, int32_t K, int32_t towers, int64_t a_stride, int64_t b_stride,
                             const float *bias, float *C, int64_t c_stride, int32_t cfg, void *stream) {
#ifdef MERLIN_PROBES
    if (cfg < 60 || cfg >= 80) return fail(MERLIN_E_UNSUPPORTED, "plane-operand cfgs are 60..79 (probe build)");
#else
    if (cfg < 60 || cfg >= 70) return fail(MERLIN_E_UNSUPPORTED, "plane-operand cfgs are 60..69");
#endif
    return h3_gemm_nt(static_cast<const float *>(A_planes), amax_a, B, amax_b, M, N, K, towers, a_stride, b_stride,
                      bias, C, c_stride, nullptr, nullptr, cfg, stream);
}

int merlin_h3_gemm_nt_gather(const float *A, const uint32_t *amax_a, const void *B, const uint32_t *amax_b, int64_t M,
                             int32_t N, int32_t K, int32_t towers, int64_t a_stride, int64_t b_stride,
                             const float *bias, float *C, int64_t c_stride, const int32_t *a_rows, int32_t cfg,
                             void *stream) {
    if (M > 0 && !a_rows) return fail(MERLIN_E_INVALID, "null argument");
    if (K % 64) return fail(MERLIN_E_UNSUPPORTED, "gathered rows: K must be a multiple of 64");
    return h3_gemm_nt(A, amax_a, B, amax_b, M, N, K, towers, a_stride, b_stride, bias, C, c_stride, nullptr, a_rows,
                      cfg, stream);
}

static int h3_gemm_tn(const void *A, const uint32_t *amax_a, const void *B, const uint32_t *amax_b, int64_t Kd,
                      int32_t M, int32_t N, int32_t towers, int64_t a_stride, int64_t b_stride, int32_t splits,
                      float *slab, float *out, bool planes, int32_t cfg, void *stream, const int32_t *b_rows = nullptr,
                      bool a_planes = false, bool b_planes = false) {
    if (Kd < 0 || M <= 0 || N <= 0) return fail(MERLIN_E_INVALID, "bad shape");
    if (!out || (Kd > 0 && (!A || !B || !slab || !amax_a || !amax_b))) return fail(MERLIN_E_INVALID, "null argument");
    if (towers < 1 || towers > 2) return fail(MERLIN_E_INVALID, "towers must be 1 or 2");
    if (splits < 1 || splits > merlin::x6_tn_max_splits()) return fail(MERLIN_E_INVALID, "splits out of range");
    if (M % 8 || N % 8 || a_stride % 4 || b_stride % 4) return fail(MERLIN_E_INVALID, "M, N: multiples of 8");
    const hipError_t e = merlin::launch_h3_gemm_tn(A, amax_a, B, amax_b, Kd, M, N, towers, a_stride, b_stride, splits,
                                                   slab, out, planes, cfg, (hipStream_t)stream, b_rows, a_planes,
                                                   b_planes);
    if (e == hipErrorInvalidValue) return fail(MERLIN_E_UNSUPPORTED, "M / N not multiples of the tile / bad cfg");
    HIP_TRY(e);
    return MERLIN_OK;
}

int merlin_h3_gemm_tn(const float *A, const uint32_t *amax_a, const float *B, const uint32_t *amax_b, int64_t Kd,
                      int32_t M, int32_t N, int32_t towers, int64_t a_stride, int64_t b_stride, int32_t splits,
                      float *slab, float *out, int32_t cfg, void *stream) {
    return h3_gemm_tn(A, amax_a, B, amax_b, Kd, M, N, towers, a_stride, b_stride, splits, slab, out, false, cfg,
                      stream);
}

int merlin_h3_gemm_nt_heads(const float *A, const uint32_t *amax_a, const void *B, const uint32_t *amax_b, int64_t M,
                            int32_t N, int32_t K, int64_t a_stride, int64_t b_stride, const float *bias, float *C,
                            int64_t c_stride, const int32_t *a_rows, const float *head_w0, int32_t n_actions,
                            const float *head_w1, float *head_partials, int32_t cfg, void *stream) {
    if (M > 0 && (!bias || !head_w0 || !head_w1 || !head_partials)) return fail(MERLIN_E_INVALID, "null argument");
    if (n_actions < 1 || n_actions > 4) return fail(MERLIN_E_UNSUPPORTED, "heads epilogue: 1..4 actions");
    if (merlin::h3_heads_parts(N, cfg) == 0) return fail(MERLIN_E_UNSUPPORTED, "heads epilogue: cfg 10, 12 or 13");
    if (a_rows && K % 64) return fail(MERLIN_E_UNSUPPORTED, "gathered rows: K must be a multiple of 64");
    return h3_gemm_nt(A, amax_a, B, amax_b, M, N, K, 2, a_stride, b_stride, bias, C, c_stride, nullptr, a_rows, cfg,
                      stream, head_w0, n_actions, head_w1, head_partials);
}

int32_t merlin_h3_heads_parts(int32_t N, int32_t cfg) { return merlin::h3_heads_parts(N, cfg); }

int merlin_act_draw(const float *partials, int32_t parts, int64_t n, const float *b_actor, const float *b_critic,
                    int32_t n_actions, int32_t deterministic, uint64_t seed, const int64_t *epoch, int64_t step,
                    int64_t env_offset, int64_t *action, float *logp, float *value, void *stream) {
    if (n < 0 || parts < 1 || n_actions < 1 || n_actions > 4) return fail(MERLIN_E_INVALID, "bad shape");
    if (n > 0 && (!partials || !b_actor || !b_critic || !action || !logp || !value))
        return fail(MERLIN_E_INVALID, "null argument");
    HIP_TRY(merlin::launch_act_draw(partials, parts, n, b_actor, b_critic, n_actions, deterministic, seed, epoch, step,
                                    env_offset, action, logp, value, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_heads_combine(const float *partials, int32_t parts, int64_t M, int32_t n_actions, float *logits,
                         float *value, void *stream) {
    if (M < 0 || parts < 1 || n_actions < 1 || n_actions > 4) return fail(MERLIN_E_INVALID, "bad shape");
    if (M > 0 && (!partials || !logits || !value)) return fail(MERLIN_E_INVALID, "null argument");
    HIP_TRY(merlin::launch_heads_combine(partials, parts, M, n_actions, logits, value, (hipStream_t)stream));
    return MERLIN_OK;
}

int merlin_h3_gemm_tn_gather(const float *A, const uint32_t *amax_a, const float *B, const uint32_t *amax_b, int64_t Kd,
                             int32_t M, int32_t N, int32_t towers, int64_t a_stride, int64_t b_stride, int32_t splits,
                             float *slab, float *out, const int32_t *b_rows, int32_t cfg, void *stream) {
    if (Kd > 0 && !b_rows) return fail(MERLIN_E_INVALID, "null argument");
    if (N % 64) return fail(MERLIN_E_UNSUPPORTED, "gathered rows: N must be a multiple of 64");
    return h3_gemm_tn(A, amax_a, B, amax_b, Kd, M, N, towers, a_stride, b_stride, splits, slab, out, false, cfg, stream,
                      b_rows);
}

int merlin_h3_gemm_nt_heads_planes(const void *A_planes, const uint32_t *amax_a, const void *B,
                                   const uint32_t *amax_b, int64_t M, int32_t N, int32_t K, int64_t a_stride,
                                   int64_t b_stride, const float *bias, float *C, int64_t c_stride,
                                   const int32_t *a_rows, const float *head_w0, int32_t n_actions,
                                   const float *head_w1, float *head_partials, int32_t cfg, void *stream) {
    if (M > 0 && (!bias || !C || !a_rows || (head_partials && (!head_w0 || !head_w1))))
        return fail(MERLIN_E_INVALID, "null argument");
    if (head_partials && (n_actions < 1 || n_actions > 4))
        return fail(MERLIN_E_UNSUPPORTED, "heads epilogue: 1..4 actions");
    if (merlin::h3_heads_parts(N, cfg) == 0) return fail(MERLIN_E_UNSUPPORTED, "planes forward: cfg 10, 12 or 13");
    if (K % 64) return fail(MERLIN_E_UNSUPPORTED, "gathered rows: K must be a multiple of 64");
    return h3_gemm_nt(static_cast<const float *>(A_planes), amax_a, B, amax_b, M, N, K, 2, a_stride, b_stride, bias,
                      C, c_stride, nullptr, a_rows, cfg, stream, head_w0, n_actions, head_w1, head_partials, true);
}

int merlin_h3_gemm_tn_gather_planes(const void *A_planes, const uint32_t *amax_a, const void *B_planes,
                                    const uint32_t *amax_b, int64_t Kd, int32_t M, int32_t N, int32_t towers,
                                    int64_t a_stride, int64_t b_stride, int32_t splits, float *slab, float *out,
                                    const int32_t *b_rows, int32_t cfg, void *stream) {
    if (Kd > 0 && !b_rows) return fail(MERLIN_E_INVALID, "null argument");
    if (N % 64) return fail(MERLIN_E_UNSUPPORTED, "gathered rows: N must be a multiple of 64");
    return h3_gemm_tn(A_planes, amax_a, B_planes, amax_b, Kd, M, N, towers, a_stride, b_stride, splits, slab, out,
                      false, cfg, stream, b_rows, true, true);
}

int merlin_h3_gemm_tn_gather_planes_a(const void *A_planes, const uint32_t *amax_a, const float *B,
                                      const uint32_t *amax_b, int64_t Kd, int32_t M, int32_t N, int32_t towers,
                                      int64_t a_stride, int64_t b_stride, int32_t splits, float *slab, float *out,
                                      const int32_t *b_rows, int32_t cfg, void *stream) {
    if (Kd > 0 && !b_rows) return fail(MERLIN_E_INVALID, "null argument");
    if (N % 64) return fail(MERLIN_E_UNSUPPORTED, "gathered rows: N must be a multiple of 64");
    return h3_gemm_tn(A_planes, amax_a, B, amax_b, Kd, M, N, towers, a_stride, b_stride, splits, slab, out, false, cfg,
                      stream, b_rows, true);
}

int merlin_h3_gemm_tn_planes(const void *A, const uint32_t *amax_a, const void *B, const uint32_t *amax_b, int64_t Kd,
                             int32_t M, int32_t N, int32_t towers, int64_t a_stride, int64_t b_stride, int32_t splits,
                             float *slab, float *out, int32_t cfg, void *stream) {
    return h3_gemm_tn(A, amax_a, B, amax_b, Kd, M, N, towers, a_stride, b_stride, splits, slab, out, true, cfg,
                      stream);
}

int64_t merlin_clip_adam_workspace(int32_t n_tensors, const int64_t *numel) {
    if (n_tensors < 0 || n_tensors > merlin::OPT_MAX_TENSORS || (n_tensors > 0 && !numel)) return -1;
    return std::max<int64_t>(1, merlin::opt_blocks(n_tensors, numel));
}

int merlin_clip_adam(int32_t n_tensors, float *const *params, float *const *grads, float *const *exp_avg,
                     float *const *exp_avg_sq, float *const *steps, const int64_t *numel, double lr, double beta1,
                     double beta2, double eps, float max_norm, float *norm_out, double *workspace, void *stream) {
    if (n_tensors < 1 || n_tensors > merlin::OPT_MAX_TENSORS)
        return fail(MERLIN_E_INVALID, "n_tensors must be in [1, 32]");
    if (!params || !grads || !exp_avg || !exp_avg_sq || !steps || !numel || !workspace)
        return fail(MERLIN_E_INVALID, "null argument");
    int64_t blocks = 0;
    for (int i = 0; i < n_tensors; i++) {
        if (numel[i] <= 0) return fail(MERLIN_E_INVALID, "every tensor needs numel > 0");
        if (!params[i] || !grads[i] || !exp_avg[i] || !exp_avg_sq[i] || !steps[i])
            return fail(MERLIN_E_INVALID, "null tensor pointer");
    }
    blocks = merlin::opt_blocks(n_tensors, numel);
    if (blocks > INT32_MAX / 2) return fail(MERLIN_E_INVALID, "too many elements");
    HIP_TRY(merlin::launch_clip_adam(n_tensors, params, grads, exp_avg, exp_avg_sq, steps, numel, lr, beta1, beta2, eps,
                                     max_norm, norm_out, workspace, (hipStream_t)stream));
    return MERLIN_OK;
}

}  // extern "C"
