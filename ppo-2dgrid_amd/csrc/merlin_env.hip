// merlin_env.hip -- batched MiniGrid dynamics for the MERLIN envs on gfx950.
//
// One thread owns one env (the envs are independent; a wave = 64 envs).  The
// env's wall rows are staged into a per-thread LDS column (rows[r][lane]) so
// that the data-dependent row reads of the 7x7 view, the forward-cell test and
// the rejection-sampling occupancy tests are LDS reads, not scattered global
// loads; the rows reach HBM again only after a reset rewrote them.  The step
// loop keeps agent state in registers across n_steps (the env-only rollout
// runs many steps per launch).
//
// Semantics follow the reference (paths relative to its checkout):
//   step    MiniGridEnv.step via ThreeActionWrapper (three_action_wrapper.py:16-17),
//           reward 1 - 0.9*step/max_steps in f64, done = term or trunc (src/ppo.py:77),
//           StuckPenaltyWrapper.step (stuck_penalty_wrapper.py:29-57) when enabled
//   reset   MiniGridEnv.reset -> _gen_grid of easy_env.py:19-39, medium_env.py:19-33,
//           medium_hard_env.py:12-45 (+ _is_reachable :47-74), hard_env.py:11-73,
//           hardest_env.py:20-70, drawing from numpy's PCG64 with the Lemire
//           bounded-integer model (bit-exact with Generator.integers / choice)
//   view    gen_obs_grid (get_view_exts, Grid.slice, rotate_left^(dir+1),
//           process_vis with see_through_walls=False, base_env.py:39) and the
//           get_pov_render tile classes (RGBImgPartialObsWrapper, scenario_creator.py:48)
#include <algorithm>

#include <cstdlib>

#include "merlin_internal.h"

namespace merlin {
namespace {

constexpr int BLK = 64;    // reset kernels: one wave per block (map generation is long and divergent)
constexpr int SBLK = 128;  // step kernel: 2 waves per block (4096 envs: rollout 21.43 vs 21.90 ms at 256, r05ag_*)
static_assert(SBLK % BLK == 0 && SBLK >= 64, "step blocks: whole waves; one bflag each (merlin_capi.hip: n / 64)");

// ---------------------------------------------------------------------------
// numpy PCG64 + bounded integers
struct Rng {
    uint64_t slo, shi, ilo, ihi;
    uint32_t has, buf;
};

// the next output and the state after it, r unchanged
__device__ __forceinline__ uint64_t rng_peek64(const Rng &r, uint64_t &nlo, uint64_t &hi) {
    // state = state * 0x2360ed051fc65da44385df649fccf645 + inc (mod 2^128), then XSL-RR
    const uint64_t MLO = 0x4385df649fccf645ULL, MHI = 0x2360ed051fc65da4ULL;
    const uint64_t lo = r.slo * MLO;
    hi = __umul64hi(r.slo, MLO) + r.slo * MHI + r.shi * MLO;
    nlo = lo + r.ilo;
    hi += r.ihi + (nlo < lo ? 1ULL : 0ULL);
    const uint64_t x = hi ^ nlo;
    const unsigned rot = (unsigned)(hi >> 58);
    return (x >> rot) | (x << ((64u - rot) & 63u));
}
__device__ __forceinline__ uint64_t rng_next64(Rng &r) {
    uint64_t nlo, hi;
    const uint64_t v = rng_peek64(r, nlo, hi);
    r.slo = nlo;
    r.shi = hi;
    return v;
}

__device__ __forceinline__ uint32_t rng_next32(Rng &r) {
    if (r.has) {
        r.has = 0;
        return r.buf;
    }
    uint64_t v = rng_next64(r);
    r.has = 1;
    r.buf = (uint32_t)(v >> 32);
    return (uint32_t)v;
}

// buffered_bounded_lemire_uint32(rng = range - 1)
template <class R>
__device__ __forceinline__ uint32_t rng_lemire(R &r, uint32_t rng_incl) {
    const uint32_t excl = rng_incl + 1u;
    uint64_t m = (uint64_t)rng_next32(r) * excl;
    uint32_t left = (uint32_t)m;
    if (left < excl) {
        const uint32_t thresh = (0xffffffffu - rng_incl) % excl;
        while (left < thresh) {
            m = (uint64_t)rng_next32(r) * excl;
            left = (uint32_t)m;
        }
    }
    return (uint32_t)(m >> 32);
}

// Generator.integers(lo, hi)
template <class R>
__device__ __forceinline__ int rng_int(R &r, int lo, int hi) {
    uint32_t rng = (uint32_t)(hi - lo - 1);
    if (rng == 0u) return lo;
    return lo + (int)rng_lemire(r, rng);
}

// x = integers(0, S); y = integers(0, S) (place_obj over the whole grid) with ONE PCG64 step on the common path: the
// pair's 32-bit draws are the buffered half and the next output's low half (has = 1) or both halves of it (has = 0),
// so the lanes of a wave no longer diverge on which of them needs a fresh output; a pair Lemire would not accept at
// once (low product word < S, probability < 2^-27) takes the two sequential draws from the unchanged state
__device__ __forceinline__ void rng_xy(Rng &r, int S, int &x, int &y) {
    uint64_t nlo, hi;
    const uint64_t v = rng_peek64(r, nlo, hi);
    const uint32_t u1 = r.has ? r.buf : (uint32_t)v, u2 = r.has ? (uint32_t)v : (uint32_t)(v >> 32);
    const uint64_t m1 = (uint64_t)u1 * (uint32_t)S, m2 = (uint64_t)u2 * (uint32_t)S;
    if ((uint32_t)m1 >= (uint32_t)S && (uint32_t)m2 >= (uint32_t)S) {
        r.slo = nlo;
        r.shi = hi;
        r.buf = (uint32_t)(v >> 32);  // has: as it was (two halves drawn)
        x = (int)(m1 >> 32);
        y = (int)(m2 >> 32);
        return;
    }
    x = rng_int(r, 0, S);
    y = rng_int(r, 0, S);
}

__device__ __forceinline__ Rng load_rng(const EnvDev &E, int i) {
    ulonglong2 s = E.rng_s[i], c = E.rng_i[i];
    uint2 b = E.rng_b[i];
    Rng r;
    r.slo = s.x;
    r.shi = s.y;
    r.ilo = c.x;
    r.ihi = c.y;
    r.has = b.x;
    r.buf = b.y;
    return r;
}

__device__ __forceinline__ void store_rng(const EnvDev &E, int i, const Rng &r) {
    E.rng_s[i] = make_ulonglong2(r.slo, r.shi);
    E.rng_b[i] = make_uint2(r.has, r.buf);
}

// ---------------------------------------------------------------------------
// Where a grid's wall rows live while a map is generated: this thread's column of an LDS array.
template <int NB>
struct LdsRows {
    uint32_t (*p)[NB];
    int lane;
    __device__ __forceinline__ uint32_t row(int y) const { return p[y][lane]; }
    __device__ __forceinline__ void set_row(int y, uint32_t v) { p[y][lane] = v; }
};
// Grid + generator state over a row store.
template <int SP, class Rows>
struct Grid {
    Rows rows;
    int S;
    int ax, ay, dir;
    int gx, gy;
    bool goal_set;
    uint32_t err;

    __device__ __forceinline__ uint32_t row(int y) const { return rows.row(y); }
    __device__ __forceinline__ void set_row(int y, uint32_t v) { rows.set_row(y, v); }
    __device__ __forceinline__ bool wall(int x, int y) const { return (row(y) >> x) & 1u; }
    __device__ __forceinline__ void set_wall(int x, int y) { set_row(y, row(y) | (1u << x)); }
    __device__ __forceinline__ void clear_wall(int x, int y) { set_row(y, row(y) & ~(1u << x)); }
    __device__ __forceinline__ uint32_t full() const { return S >= 32 ? 0xffffffffu : ((1u << S) - 1u); }
    __device__ __forceinline__ bool occupied(int x, int y) const {
        return wall(x, y) || (goal_set && x == gx && y == gy);
    }

    // Grid(W,H) + wall_rect(0,0,W,H)
    __device__ void walled() {
        const uint32_t edge = 1u | (1u << (S - 1));
#pragma unroll
        for (int y = 0; y < SP; y++)
            if (y < S) set_row(y, (y == 0 || y == S - 1) ? full() : edge);
        goal_set = false;
    }

    // MiniGridEnv.place_obj: x then y; reject occupied cells and agent_pos.
    // kind: 0 none (agent), 1 wall, 2 goal.  max_tries < 0 = unbounded.
    template <class R>
    __device__ bool place(R &r, int kind, int tx, int ty, int sw, int sh, int max_tries, int &px, int &py) {
        const int xe = min(tx + sw, S), ye = min(ty + sh, S);
        int tries = 0;
        for (;;) {
            if (max_tries >= 0 && tries > max_tries) {
                err |= MERLIN_DEVERR_PLACE_OBJ;
                return false;
            }
            tries++;
            int x = rng_int(r, tx, xe);
            int y = rng_int(r, ty, ye);
            if (occupied(x, y)) continue;
            if (x == ax && y == ay) continue;
            if (kind == 1) set_wall(x, y);
            if (kind == 2) {
                gx = x;
                gy = y;
                goal_set = true;
            }
            px = x;
            py = y;
            return true;
        }
    }

    // MiniGridEnv.place_agent(top, size, rand_dir=True)
    template <class R>
    __device__ void place_agent(R &r, int tx, int ty, int sw, int sh) {
        int x, y;
        ax = -1;
        ay = -1;
        place(r, 0, tx, ty, sw, sh, -1, x, y);
        ax = x;
        ay = y;
        dir = rng_int(r, 0, 4);
    }

    template <class R>
    __device__ void place_goal(R &r) {
        int x, y;
        place(r, 2, 0, 0, S, S, -1, x, y);
    }

    // _is_reachable (medium_hard_env.py:47-74): the BFS's boolean equals "goal in
    // the 4-connected component of non-wall cells containing the agent"; computed
    // as a bit-parallel flood fill over row masks (Gauss-Seidel sweeps in registers).
    // A row takes in one visit every free run that holds a seed (run_fill: the carry of f + x runs from
    // the lowest seed of a run to its end, the same on the bit-reversed row for the other direction),
    // so the sweeps only have to carry the component between rows; the fixed point, hence the boolean,
    // is the same component as with one cell of horizontal spread per visit.
    __device__ static __forceinline__ uint32_t run_fill(uint32_t f, uint32_t rf, uint32_t x) {
        const uint32_t u = (f & ~(f + x)) | x;  // from the lowest seed of each run up to the run's end
        const uint32_t ru = __brev(u);
        return __brev((rf & ~(rf + ru)) | ru);  // and down to the run's start
    }
    __device__ bool reachable() const {
        uint32_t F[SP], RF[SP], R[SP];
        const uint32_t fm = full();
#pragma unroll
        for (int y = 0; y < SP; y++) {
            F[y] = (y < S) ? (~row(y) & fm) : 0u;
            RF[y] = __brev(F[y]);
            R[y] = (y == ay) ? run_fill(F[y], RF[y], 1u << ax) : 0u;
        }
        for (int it = 0; it < SP * SP; it++) {
            uint32_t changed = 0u;
#pragma unroll
            for (int y = 1; y < SP; y++) {
                const uint32_t x = (R[y - 1] | (y < SP - 1 ? R[y + 1] : 0u)) & F[y] & ~R[y];
                const uint32_t n = x ? run_fill(F[y], RF[y], x | R[y]) : R[y];
                changed |= n ^ R[y];
                R[y] = n;
            }
#pragma unroll
            for (int y = SP - 2; y >= 0; y--) {
                const uint32_t x = ((y > 0 ? R[y - 1] : 0u) | R[y + 1]) & F[y] & ~R[y];
                const uint32_t n = x ? run_fill(F[y], RF[y], x | R[y]) : R[y];
                changed |= n ^ R[y];
                R[y] = n;
            }
            uint32_t hit = 0u;
#pragma unroll
            for (int y = 0; y < SP; y++) hit |= (y == gy) ? ((R[y] >> gx) & 1u) : 0u;
            if (hit) return true;
            if (!changed) return false;
        }
        return false;
    }

    template <class R>
    __device__ void fallback(R &r, uint32_t *fallbacks) {
        atomicAdd(fallbacks, 1u);
        walled();
        place_agent(r, 0, 0, S, S);
        place_goal(r);
    }

    // EasyEnv._gen_grid (easy_env.py:19-39): put_obj(Goal, W-5, H-5) may sit on the agent
    template <class R>
    __device__ void gen_easy(R &r) {
        walled();
        place_agent(r, 0, 0, S, S);
        gx = S - 5;
        gy = S - 5;
        goal_set = true;
    }

    // MediumEnv._gen_grid (medium_env.py:19-33)
    template <class R>
    __device__ void gen_medium(R &r) {
        walled();
        place_agent(r, 0, 0, S, S);
        place_goal(r);
    }

    // MediumHardEnv._gen_grid (medium_hard_env.py:12-45); on a retry the previous
    // attempt's agent_pos still blocks wall placement (place_agent resets it later).
    template <class R>
    __device__ void gen_mediumhard(R &r, uint32_t *fallbacks) {
        const int playable = (S - 2) * (S - 2);
        const int min_obs = (playable * 10) / 100;  // int(playable * 0.10)
        const int max_obs = (playable * 20) / 100;  // int(playable * 0.20)
        for (int attempt = 0; attempt < 100; attempt++) {
            walled();
            int n = rng_int(r, max(1, min_obs), max(1, max_obs) + 1);
            // n x place(r, 1, 0, 0, S, S, 100) as one loop of draws (the same draws, checks and failure): a wave
            // runs as many iterations as its longest lane needs in all, not the sum over walls of each wall's
            // slowest lane, as nested retry loops do (refill 43 -> ~40 us, profiles/r05z_*)
            for (int k = 0, tries = 0; k < n;) {
                if (tries > 100) {
                    err |= MERLIN_DEVERR_PLACE_OBJ;
                    return;
                }
                tries++;
                int x, y;
                rng_xy(r, S, x, y);
                if (occupied(x, y) || (x == ax && y == ay)) continue;
                set_wall(x, y);
                k++;
                tries = 0;
            }
            place_agent(r, 0, 0, S, S);
            place_goal(r);
            if (reachable()) return;
        }
        fallback(r, fallbacks);
    }

    // HardEnv._gen_grid (hard_env.py:11-73), agent_start_pos None, random_goal True
    template <class R>
    __device__ void gen_hard(R &r, uint32_t *fallbacks) {
        const int mid = S / 2;
        const bool large = S > 10;
        for (int attempt = 0; attempt < 100; attempt++) {
            walled();
            const int k = large ? rng_int(r, 2, 6) : 1;
            // choice(range(1, S-1), k, replace=False): Floyd + tail shuffle (pop <= 10000)
            const int pop = S - 2;
            int idx[5] = {0, 0, 0, 0, 0};
#pragma unroll
            for (int q = 0; q < 5; q++) {
                if (q < k) {
                    const int j = pop - k + q;
                    int val = (j == 0) ? 0 : (int)rng_lemire(r, (uint32_t)j);
                    bool dup = false;
#pragma unroll
                    for (int p = 0; p < 5; p++) dup |= (p < q) && (idx[p] == val);
                    idx[q] = dup ? j : val;
                }
            }
#pragma unroll
            for (int i = 4; i >= 1; i--) {
                if (i < k) {
                    const int j = (int)rng_lemire(r, (uint32_t)i);
                    int a = 0;
#pragma unroll
                    for (int p = 0; p < 5; p++) a = (p == j) ? idx[p] : a;
                    const int b = idx[i];
#pragma unroll
                    for (int p = 0; p < 5; p++) idx[p] = (p == j) ? b : idx[p];
                    idx[i] = a;
                }
            }
            uint32_t gap_rows = 0u;  // bit i = row i is a gap
#pragma unroll
            for (int p = 0; p < 5; p++)
                if (p < k) gap_rows |= 1u << (idx[p] + 1);
            for (int i = 1; i < S - 1; i++)
                if (!((gap_rows >> i) & 1u)) set_wall(mid, i);
            if (large) {
                const int extra = rng_int(r, 6, 13);
                for (int w = 0; w < extra; w++) {
                    for (int t = 0; t < 10; t++) {
                        int x = rng_int(r, 1, S - 1);
                        int y = rng_int(r, 1, S - 1);
                        if (x != mid && !wall(x, y)) {  // no goal placed yet
                            set_wall(x, y);
                            break;
                        }
                    }
                }
            }
            int x, y;
            place(r, 2, mid + 1, 0, S - mid - 1, S, -1, x, y);
            place_agent(r, 1, 1, mid - 1, S - 2);
            if (reachable()) return;
        }
        fallback(r, fallbacks);
    }

    // HardestEnv._gen_grid (hardest_env.py:20-70)
    template <class R>
    __device__ void gen_hardest(R &r, uint32_t *fallbacks) {
        const int mx = S / 2, my = S / 2;
        for (int attempt = 0; attempt < 100; attempt++) {
            walled();
            for (int y = 1; y < S - 1; y++) set_wall(mx, y);
            set_row(my, full());  // x in [1, S-1) plus the border bits already set
            clear_wall(mx, rng_int(r, 2, my - 1));
            clear_wall(mx, rng_int(r, my + 1, S - 2));
            clear_wall(rng_int(r, 2, mx - 1), my);
            clear_wall(rng_int(r, mx + 1, S - 2), my);
            const int nobs = rng_int(r, 6, 13);
            for (int k = 0; k < nobs; k++) {
                int x = rng_int(r, 1, S - 1);
                int y = rng_int(r, 1, S - 1);
                if (!wall(x, y) && x != mx && y != my) set_wall(x, y);
            }
            place_agent(r, 0, 0, S, S);
            place_goal(r);
            if (reachable()) return;
        }
        fallback(r, fallbacks);
    }

    // MiniGridEnv.reset body: agent_pos=(-1,-1); _gen_grid(W,H)
    template <class R>
    __device__ void generate(R &r, int difficulty, uint32_t *fallbacks) {
        ax = -1;
        ay = -1;
        dir = 0;
        goal_set = false;
        switch (difficulty) {
            case MERLIN_EASY: gen_easy(r); break;
            case MERLIN_MEDIUM: gen_medium(r); break;
            case MERLIN_MEDIUMHARD: gen_mediumhard(r, fallbacks); break;
            case MERLIN_HARD: gen_hard(r, fallbacks); break;
            default: gen_hardest(r, fallbacks); break;
        }
    }
};

// Map generation runs only on reset: keep it out of line so the step loop's state stays
// in registers (the generator's Grid object lives in its own frame).
struct GenOut {
    int ax, ay, dir, gx, gy;
    uint32_t err;
};

template <int SP, int NB>
__device__ __forceinline__ void generate_map_inl(uint32_t (*rows)[NB], int lane, int S, int difficulty, Rng &r,
                                                 uint32_t *fallbacks, GenOut &o) {
    Grid<SP, LdsRows<NB>> G;
    G.rows.p = rows;
    G.rows.lane = lane;
    G.S = S;
    G.err = 0u;
    G.generate(r, difficulty, fallbacks);
    o.ax = G.ax;
    o.ay = G.ay;
    o.dir = G.dir;
    o.gx = G.gx;
    o.gy = G.gy;
    o.err = G.err;
}

// out of line for the multi-step kernel, whose step state must stay in registers across a reset
template <int SP, int NB>
__device__ __noinline__ void generate_map(uint32_t (*rows)[NB], int lane, int S, int difficulty, Rng &r,
                                          uint32_t *fallbacks, GenOut &o) {
    generate_map_inl<SP, NB>(rows, lane, S, difficulty, r, fallbacks, o);
}

__device__ __forceinline__ uint32_t bitrev7(uint32_t v) { return __brev(v) >> 25; }

// gen_obs_grid + get_pov_render tile classes -> 8 packed nibble words.
template <int SP, int NB>
__device__ __forceinline__ void view_codes(const uint32_t (*rows)[NB], int lane, int S, int ax, int ay, int dir,
                                           int goal_x, int goal_y, bool goal_set,
                                           uint32_t out[MERLIN_OBS_WORDS]) {
    // get_view_exts (top-left of the 7x7 world window)
    int tx, ty;
    if (dir == 0) {
        tx = ax;
        ty = ay - 3;
    } else if (dir == 1) {
        tx = ax - 3;
        ty = ay;
    } else if (dir == 2) {
        tx = ax - 6;
        ty = ay - 3;
    } else {
        tx = ax - 3;
        ty = ay - 6;
    }
    // Grid.slice: out-of-bounds cells read as Wall
    const uint64_t hi_ones = ~0ULL << (S + 8);
    uint32_t win[7];
#pragma unroll
    for (int r = 0; r < 7; r++) {
        const int y = ty + r;
        const bool in = (y >= 0) && (y < S);
        const uint32_t row = in ? rows[in ? y : 0][lane] : 0xffffffffu;
        const uint64_t w = ((uint64_t)row << 8) | 0xffULL | hi_ones;
        win[r] = (uint32_t)(w >> (tx + 8)) & 0x7fu;  // bit c = cell (c, r) of the slice
    }
    // rotate_left applied k = (dir+1) mod 4 times: built from transpose / row flip / bit reverse
    uint32_t tr[7];
#pragma unroll
    for (int x = 0; x < 7; x++) {
        uint32_t v = 0u;
#pragma unroll
        for (int y = 0; y < 7; y++) v |= ((win[y] >> x) & 1u) << y;
        tr[x] = v;
    }
    const int k = (dir + 1) & 3;
    const bool odd = k & 1, flip = (k == 1) || (k == 2), rev = (k >= 2);
    uint32_t V[7];  // V[j] bit i = view cell (i, j) is a wall
#pragma unroll
    for (int b = 0; b < 7; b++) {
        uint32_t m = flip ? (odd ? tr[6 - b] : win[6 - b]) : (odd ? tr[b] : win[b]);
        V[b] = rev ? bitrev7(m) : m;
    }
    // goal position in view: view(vi,vj) <- world(agent + (6-vj)*F + (vi-3)*R)
    const int Fx = (dir == 0) - (dir == 2), Fy = (dir == 1) - (dir == 3);
    const int Rx = -Fy, Ry = Fx;  // DIR_TO_VEC[(dir+1)%4]
    const int dx = goal_x - ax, dy = goal_y - ay;
    const int gvj = 6 - (dx * Fx + dy * Fy), gvi = 3 + (dx * Rx + dy * Ry);
    const bool ginv = goal_set && gvi >= 0 && gvi < 7 && gvj >= 0 && gvj < 7;
    // Grid.process_vis(agent_pos=(3,6)) as row bit-ops (walls opaque, goal/empty transparent)
    uint32_t m[7] = {0u, 0u, 0u, 0u, 0u, 0u, 1u << 3};
#pragma unroll
    for (int j = 6; j >= 0; j--) {
        const uint32_t T = ~V[j] & 0x7fu;
        uint32_t M = m[j];
#pragma unroll
        for (int s = 0; s < 6; s++) M |= (M & T & 0x3fu) << 1;  // left-to-right pass
        const uint32_t e1 = M & T & 0x3fu;
#pragma unroll
        for (int s = 0; s < 6; s++) M |= (M & T & 0x7eu) >> 1;  // right-to-left pass
        const uint32_t e2 = M & T & 0x7eu;
        m[j] = M;
        if (j > 0) m[j - 1] |= e1 | (e1 << 1) | e2 | (e2 >> 1);
    }
#pragma unroll
    for (int w = 0; w < MERLIN_OBS_WORDS; w++) out[w] = 0u;
#pragma unroll
    for (int j = 0; j < 7; j++) {
#pragma unroll
        for (int i = 0; i < 7; i++) {
            const int kk = j * 7 + i;
            uint32_t c;
            if (i == 3 && j == 6) {
                c = 4u;  // agent tile (its own cell is set to None, agent_dir=3)
            } else {
                const bool vis = (m[j] >> i) & 1u;
                const bool wl = (V[j] >> i) & 1u;
                const bool gl = ginv && gvi == i && gvj == j;
                c = !vis ? 0u : (wl ? 2u : (gl ? 3u : 1u));
            }
            out[kk >> 3] |= c << ((kk & 7) * 4);
        }
    }
}

template <int SP, int NB>
__device__ __forceinline__ void load_rows(const EnvDev &E, int i, uint32_t (*rows)[NB], int lane) {
    const uint4 *src = reinterpret_cast<const uint4 *>(E.walls + (size_t)i * SP);
#pragma unroll
    for (int q = 0; q < SP / 4; q++) {
        const uint4 v = src[q];
        rows[4 * q + 0][lane] = v.x;
        rows[4 * q + 1][lane] = v.y;
        rows[4 * q + 2][lane] = v.z;
        rows[4 * q + 3][lane] = v.w;
    }
}

template <int SP, int NB>
__device__ __forceinline__ void store_rows(const EnvDev &E, int i, const uint32_t (*rows)[NB], int lane, int S) {
    uint4 *dst = reinterpret_cast<uint4 *>(E.walls + (size_t)i * SP);
#pragma unroll
    for (int q = 0; q < SP / 4; q++) {
        const int y = 4 * q;
        dst[q] = make_uint4(y + 0 < S ? rows[y + 0][lane] : 0u, y + 1 < S ? rows[y + 1][lane] : 0u,
                            y + 2 < S ? rows[y + 2][lane] : 0u, y + 3 < S ? rows[y + 3][lane] : 0u);
    }
}

__device__ __forceinline__ void store_obs(uint32_t *obs, size_t row, const uint32_t w[8]) {
    uint4 *d = reinterpret_cast<uint4 *>(obs + row * MERLIN_OBS_WORDS);
    d[0] = make_uint4(w[0], w[1], w[2], w[3]);
    d[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

__device__ __forceinline__ uint4 pack_agent(int ax, int ay, int dir, int steps, int gx, int gy,
                                            int lx, int ly, int stay) {
    return make_uint4((uint32_t)ax | ((uint32_t)ay << 8) | ((uint32_t)dir << 16), (uint32_t)steps,
                      (uint32_t)gx | ((uint32_t)gy << 8),
                      (uint32_t)lx | ((uint32_t)ly << 8) | ((uint32_t)min(stay, 65535) << 16));
}

// Post-reset bookkeeping shared by the reset kernel and the auto-reset path.
template <int SP>
__device__ __forceinline__ void reset_visited(const EnvDev &E, int i, int ax, int ay) {
    uint32_t *vis = E.visited + (size_t)i * SP;
    for (int y = 0; y < SP; y++) vis[y] = (y == ay) ? (1u << ax) : 0u;
}

// Look-ahead maps.  An env's next map depends only on its RNG stream (MiniGridEnv.reset draws nothing
// else), so k_env_refill generates it ahead of time into the env's slot (pg_*: the rows, agent, goal
// and the RNG state after the generation) and a reset just takes the slot: the single-step kernel
// carries no map-generation code (lean registers, no wave stalled on one env's rejection sampling +
// flood fill), and the refill -- latency-bound on its slowest env -- runs once per REFILL_EVERY step
// launches instead of once per step.  A reset whose slot is empty (a second episode end before a
// refill, or a reseed) generates the same map from the env's RNG: in place in the reset and
// multi-step kernels, in k_env_fallback after a single-step launch.  In reseed mode (every reset is
// reset(seed=task_seed)) the slot is never consumed and the env's RNG never advances.
template <int SP, int NB>
__device__ __forceinline__ bool take_slot(const EnvDev &E, int i, uint32_t (*rows)[NB], int lane, GenOut &g) {
    if (!E.pg_valid[i]) return false;
    {
        const uint4 *src = reinterpret_cast<const uint4 *>(E.pg_walls + (size_t)i * SP);
#pragma unroll
        for (int q = 0; q < SP / 4; q++) {
            const uint4 v = src[q];
            rows[4 * q + 0][lane] = v.x;
            rows[4 * q + 1][lane] = v.y;
            rows[4 * q + 2][lane] = v.z;
            rows[4 * q + 3][lane] = v.w;
        }
        const uint4 a = E.pg_agent[i];
        g.ax = a.x & 0xff;
        g.ay = (a.x >> 8) & 0xff;
        g.dir = (a.x >> 16) & 3;
        g.gx = a.z & 0xff;
        g.gy = (a.z >> 8) & 0xff;
        g.err = 0u;
        if (!E.reseed) {
            E.rng_s[i] = E.pg_rng_s[i];
            E.rng_b[i] = E.pg_rng_b[i];
            E.pg_valid[i] = 0;
        }
    }
    return true;
}

template <int SP, int NB, bool INL>
__device__ __forceinline__ void take_map(const EnvDev &E, int i, uint32_t (*rows)[NB], int lane, GenOut &g) {
    if (!take_slot<SP, NB>(E, i, rows, lane, g)) {
        Rng r = load_rng(E, i);
        if (INL)
            generate_map_inl<SP, NB>(rows, lane, E.size, E.difficulty, r, E.err + 1, g);
        else
            generate_map<SP, NB>(rows, lane, E.size, E.difficulty, r, E.err + 1, g);
        if (!E.reseed) store_rng(E, i, r);
    }
}

// One env's reset (merlin_env_reset): its next map, state, episode accumulators, first observation.
template <int SP>
__device__ __forceinline__ void reset_one(const EnvDev &E, int i, uint32_t (*rows)[BLK], int lane,
                                          uint32_t *__restrict__ obs) {
    GenOut g;
    take_map<SP, BLK, true>(E, i, rows, lane, g);
    store_rows<SP, BLK>(E, i, rows, lane, E.size);
    E.agent[i] = pack_agent(g.ax, g.ay, g.dir, 0, g.gx, g.gy, g.ax, g.ay, 0);
    E.ep_ret[i] = 0.0;
    E.ep_len[i] = 0;
    if (E.explore_on) reset_visited<SP>(E, i, g.ax, g.ay);
    if (g.err) atomicOr(E.err, g.err);
    uint32_t w[MERLIN_OBS_WORDS];
    view_codes<SP, BLK>(rows, lane, E.size, g.ax, g.ay, g.dir, g.gx, g.gy, true, w);
    if (obs) store_obs(obs, (size_t)i, w);
}

template <int SP>
__global__ __launch_bounds__(BLK) void k_env_reset(EnvDev E, const uint8_t *__restrict__ mask,
                                                  uint32_t *__restrict__ obs) {
    __shared__ uint32_t rows[SP][BLK];
    const int lane = threadIdx.x;
    const int i = blockIdx.x * BLK + lane;
    if (i >= E.n) return;
    if (mask && !mask[i]) return;
    reset_one<SP>(E, i, rows, lane, obs);
}

// Fill the empty look-ahead slots: each one-wave block takes SPAN x 64 envs (SPAN 16: lane l reads the
// slot flags of envs base + 16*l .. in one 16-B load), packs the empty ones onto consecutive lanes
// (ballot + prefix count) and generates 64 at a time, one thread per env, from the env's RNG (which
// stays as it is: the slot holds the state after the generation).  SPAN 4 for the few slots a step
// uses, SPAN 1 (one wave per 64 envs, all generating at once) after a full reset used every slot.
template <int SP>
__device__ __forceinline__ void refill_one(const EnvDev &E, int i, uint32_t (*rows)[BLK], int lane) {
    Rng r = load_rng(E, i);
    GenOut g;
    generate_map_inl<SP, BLK>(rows, lane, E.size, E.difficulty, r, E.err + 1, g);
    uint4 *dst = reinterpret_cast<uint4 *>(E.pg_walls + (size_t)i * SP);
#pragma unroll
    for (int q = 0; q < SP / 4; q++) {
        const int y = 4 * q;
        dst[q] = make_uint4(y + 0 < E.size ? rows[y + 0][lane] : 0u, y + 1 < E.size ? rows[y + 1][lane] : 0u,
                            y + 2 < E.size ? rows[y + 2][lane] : 0u, y + 3 < E.size ? rows[y + 3][lane] : 0u);
    }
    E.pg_agent[i] = pack_agent(g.ax, g.ay, g.dir, 0, g.gx, g.gy, g.ax, g.ay, 0);
    E.pg_rng_s[i] = make_ulonglong2(r.slo, r.shi);
    E.pg_rng_b[i] = make_uint2(r.has, r.buf);
    E.pg_valid[i] = 1;
    if (g.err) atomicOr(E.err, g.err);
}

template <int SP, int SPAN>
__global__ __launch_bounds__(BLK) void k_env_refill(EnvDev E) {
    __shared__ uint32_t rows[SP][BLK];
    __shared__ int queue[BLK];
    const int lane = threadIdx.x;
    const unsigned long long below = (1ull << lane) - 1ull;
    static_assert(SPAN == 1 || SPAN == 4 || SPAN == 16, "refill span");
    const int64_t base = ((int64_t)blockIdx.x * BLK + lane) * SPAN;  // this lane's first env
    uint32_t fl[4] = {0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u};
    if (SPAN == 16 && base + SPAN <= E.n) {
        const uint4 v = *reinterpret_cast<const uint4 *>(E.pg_valid + base);
        fl[0] = v.x;
        fl[1] = v.y;
        fl[2] = v.z;
        fl[3] = v.w;
    } else if (SPAN == 4 && base + SPAN <= E.n) {
        fl[0] = *reinterpret_cast<const uint32_t *>(E.pg_valid + base);
    } else {
        for (int b = 0; b < SPAN; b++)
            if (base + b < E.n && !E.pg_valid[base + b]) fl[b >> 2] &= ~(0xffu << (8 * (b & 3)));
    }
    int nq = 0;  // wave-uniform
    for (int b = 0; b < SPAN; b++) {
        const bool need = !((fl[b >> 2] >> (8 * (b & 3))) & 0xffu);
        const unsigned long long m = __ballot(need);
        const int c = __popcll(m);
        if (c == 0) continue;
        if (nq + c > BLK) {  // the queue is full: run it first
            if (lane < nq) refill_one<SP>(E, queue[lane], rows, lane);
            nq = 0;
            __syncthreads();
        }
        if (need) queue[nq + __popcll(m & below)] = (int)(base + b);
        nq += c;
        __syncthreads();
    }
    if (lane < nq) refill_one<SP>(E, queue[lane], rows, lane);
}

// The resets of a single-step launch whose look-ahead slot was empty: one wave per 64 step blocks reads
// their block flags, packs the flagged envs of all flagged blocks onto lanes and regenerates them 64 at
// a time (reset_one: map, state, first observation into the step's obs row), clearing the flags.
// Generation is latency-bound on one thread, so the envs share one pass instead of one per block.
template <int SP>
__global__ __launch_bounds__(BLK) void k_env_fallback(EnvDev E, uint32_t *__restrict__ obs) {
    __shared__ uint32_t rows[SP][BLK];
    __shared__ int queue[BLK];
    const int lane = threadIdx.x;
    const unsigned long long below = (1ull << lane) - 1ull;
    const int nblocks = (E.n + SBLK - 1) / SBLK;
    const int b0 = blockIdx.x * BLK;
    const bool flagged = b0 + lane < nblocks && E.bflag[b0 + lane];
    unsigned long long bm = __ballot(flagged);
    if (flagged) E.bflag[b0 + lane] = 0;
    int nq = 0;  // wave-uniform
    while (bm) {
        const int sb = b0 + __builtin_ctzll(bm);
        bm &= bm - 1;
        for (int q = 0; q < SBLK / BLK; q++) {
            const int i = sb * SBLK + q * BLK + lane;
            const bool need = i < E.n && E.rflag[i];
            const unsigned long long m = __ballot(need);
            const int c = __popcll(m);
            if (c == 0) continue;
            if (nq + c > BLK) {  // the queue is full: run it first
                if (lane < nq) reset_one<SP>(E, queue[lane], rows, lane, obs);
                nq = 0;
                __syncthreads();
            }
            if (need) {
                E.rflag[i] = 0;
                queue[nq + __popcll(m & below)] = i;
            }
            nq += c;
            __syncthreads();
        }
    }
    if (lane < nq) reset_one<SP>(E, queue[lane], rows, lane, obs);
}

// DEFER (single-step launches): a reset takes the env's look-ahead slot; when the slot is empty the env
// is flagged (rflag, and its SBLK-env block in bflag) and k_env_fallback, launched next on the stream,
// generates its map and writes its observation, so this kernel carries no generator (lean registers).
// ACT: the action drawn from head partials (merlin_env_act_step) -- its own instantiation, so the plain step keeps its
// registers (the draw's partial loads in flight take ~40 more)
template <int SP, bool DEFER, bool ACT = false>
__global__ __launch_bounds__(SBLK) void k_env_step(EnvDev E, StepOut O) {
    __shared__ uint32_t rows[SP][SBLK];
    const int lane = threadIdx.x;
    const int i = blockIdx.x * SBLK + lane;
    if (i >= E.n) return;
    const int S = E.size;
    load_rows<SP, SBLK>(E, i, rows, lane);
    const uint4 st = E.agent[i];
    int ax = st.x & 0xff, ay = (st.x >> 8) & 0xff, dir = (st.x >> 16) & 3;
    int steps = (int)st.y;
    int gx = st.z & 0xff, gy = (st.z >> 8) & 0xff;
    int lx = st.w & 0xff, ly = (st.w >> 8) & 0xff, stay = (int)(st.w >> 16);
    double ep_ret = E.ep_ret[i];
    int ep_len = E.ep_len[i];
    uint32_t err = 0u;
    bool rows_dirty = false;
    const size_t N = (size_t)E.n;

    for (int t = 0; t < O.n_steps; t++) {
        // merlin_env_act_step: the action is drawn here from the acting GEMM's head partials (one launch instead of
        // k_act_draw + this kernel); otherwise read from the caller's actions
        int64_t a;
        if constexpr (ACT)
            a = (int64_t)act_from_parts(O.act, E.n, i);
        else
            a = O.actions[(size_t)t * O.action_stride + i];
        steps += 1;
        const int fx = ax + ((dir == 0) - (dir == 2));
        const int fy = ay + ((dir == 1) - (dir == 3));
        const bool fwall = (rows[fy][lane] >> fx) & 1u;
        const bool fgoal = (fx == gx) && (fy == gy);
        double rew = 0.0;
        bool term = false;
        if (a == 0) {
            dir = (dir + 3) & 3;
        } else if (a == 1) {
            dir = (dir + 1) & 3;
        } else if (a == 2) {
            if (!fwall) {  // None or Goal (can_overlap)
                ax = fx;
                ay = fy;
            }
            if (fgoal) {
                term = true;
                rew = 1.0 - 0.9 * ((double)steps / (double)E.max_steps);  // MiniGridEnv._reward
            }
        } else {
            err |= MERLIN_DEVERR_BAD_ACTION;
        }
        const bool trunc = steps >= E.max_steps;
        if (E.stuck_on) {  // StuckPenaltyWrapper.step
            stay = (ax == lx && ay == ly) ? stay + 1 : 0;
            if (stay >= E.max_stay) rew += E.penalty;
            lx = ax;
            ly = ay;
        }
        if (E.explore_on) {  // ExplorationBonus (MERLIN-AMD definition; absent in the reference)
            uint32_t *vrow = E.visited + (size_t)i * SP + ay;
            const uint32_t bit = 1u << ax, v = *vrow;
            if (!(v & bit)) {
                *vrow = v | bit;
                rew += E.bonus;
            }
        }
        const bool done = term || trunc;
        ep_ret += rew;
        ep_len += 1;
        const size_t row = (size_t)t * N + i;
        if (O.reward) O.reward[row] = (float)rew;
        if (O.term) O.term[row] = term;
        if (O.trunc) O.trunc[row] = trunc;
        if (O.done) O.done[row] = done ? 1.0f : 0.0f;
        if (done) {
            if (O.ep_ret_out) O.ep_ret_out[row] = ep_ret;
            if (O.ep_len_out) O.ep_len_out[row] = ep_len;
        }
        if (done && O.autoreset) {
            GenOut g;
            if constexpr (DEFER) {
                if (!take_slot<SP, SBLK>(E, i, rows, lane, g)) {
                    E.rflag[i] = 1;
                    E.bflag[blockIdx.x] = 1;
                    if (O.no_fallback) err |= MERLIN_DEVERR_SLOT_EMPTY;  // no fallback pass follows: an error
                    if (err) atomicOr(E.err, err);
                    return;
                }
            } else {
                take_map<SP, SBLK, false>(E, i, rows, lane, g);
            }
            ax = g.ax;
            ay = g.ay;
            dir = g.dir;
            gx = g.gx;
            gy = g.gy;
            err |= g.err;
            rows_dirty = true;
            steps = 0;
            stay = 0;
            lx = ax;
            ly = ay;
            ep_ret = 0.0;
            ep_len = 0;
            if (E.explore_on) reset_visited<SP>(E, i, ax, ay);
        }
        if (O.obs) {
            uint32_t w[MERLIN_OBS_WORDS];
            view_codes<SP, SBLK>(rows, lane, S, ax, ay, dir, gx, gy, true, w);
            store_obs(O.obs, row, w);
        }
    }
    E.agent[i] = pack_agent(ax, ay, dir, steps, gx, gy, lx, ly, stay);
    E.ep_ret[i] = ep_ret;
    E.ep_len[i] = ep_len;
    if (rows_dirty) store_rows<SP, SBLK>(E, i, rows, lane, S);
    if (err) atomicOr(E.err, err);
}

// The fully observable image (FullyObsWrapper + ImgObsWrapper, scenario_creator.py:45-50; minigrid 3.0.0
// wrappers.py FullyObsWrapper.observation, core/grid.py Grid.encode): out[env][x][y] = (object, color, state) of
// cell (x, y) -- empty (1, 0, 0), wall (2, grey 5, 0), goal (8, green 1, 0) -- and the agent's cell
// (agent 10, red 0, direction).  One thread per cell; the rows of walls are read as the bit rows the step keeps.
__global__ __launch_bounds__(256) void k_env_full_obs(EnvDev E, uint8_t *__restrict__ out) {
    const int S = E.size, cells = S * S;
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= (int64_t)E.n * cells) return;
    const int i = (int)(c / cells), xy = (int)(c - (int64_t)i * cells), x = xy / S, y = xy - x * S;
    const uint4 a = E.agent[i];
    const int ax = a.x & 0xff, ay = (a.x >> 8) & 0xff, dir = (a.x >> 16) & 3;
    const int gx = a.z & 0xff, gy = (a.z >> 8) & 0xff;
    uint8_t o = 1, col = 0, st = 0;
    if ((E.walls[(size_t)i * E.sp + y] >> x) & 1u) {
        o = 2;
        col = 5;
    } else if (x == gx && y == gy) {
        o = 8;
        col = 1;
    }
    if (x == ax && y == ay) {
        o = 10;
        col = 0;
        st = (uint8_t)dir;
    }
    uint8_t *p = out + c * 3;
    p[0] = o;
    p[1] = col;
    p[2] = st;
}

}  // namespace

template <int SP>
static hipError_t launch_refill_sp(const EnvDev &E, bool full, hipStream_t s) {
    // after steps: 4 envs per lane (16 one-wave blocks at 4,096 envs; 16 per lane, 4 blocks: each wave waits for the
    // slowest of more generations) -- 20.75 / 20.91 against 21.09 / 20.97 ms per rollout (profiles/r06ad_span*.log)
    if (full)
        hipLaunchKernelGGL((k_env_refill<SP, 1>), dim3((E.n + BLK - 1) / BLK), dim3(BLK), 0, s, E);
    else
        hipLaunchKernelGGL((k_env_refill<SP, 4>), dim3((E.n + BLK * 4 - 1) / (BLK * 4)), dim3(BLK), 0, s, E);
    return hipGetLastError();
}

hipError_t launch_env_refill(const EnvDev &E, bool full, hipStream_t s) {
    return E.sp == 16 ? launch_refill_sp<16>(E, full, s) : launch_refill_sp<32>(E, full, s);
}

hipError_t launch_env_reset(const EnvDev &E, const uint8_t *mask, uint32_t *obs, hipStream_t s) {
    const dim3 grid((E.n + BLK - 1) / BLK), block(BLK);
    if (E.sp == 16)
        hipLaunchKernelGGL(k_env_reset<16>, grid, block, 0, s, E, mask, obs);
    else
        hipLaunchKernelGGL(k_env_reset<32>, grid, block, 0, s, E, mask, obs);
    hipError_t e = hipGetLastError();
    return e != hipSuccess ? e : launch_env_refill(E, mask == nullptr, s);
}

template <int SP>
static hipError_t launch_step_sp(const EnvDev &E, const StepOut &O, hipStream_t s) {
    const int nb = (E.n + SBLK - 1) / SBLK;
    if (!O.autoreset) {  // no resets: the lean kernel
        hipLaunchKernelGGL((k_env_step<SP, true>), dim3(nb), dim3(SBLK), 0, s, E, O);
    } else if (O.n_steps == 1) {  // also the fused draw + step (merlin_env_act_step): the generator stays out of the
        // step kernel (k_env_step<SP, false> with it inlined takes 241 VGPRs + 92 B of scratch per lane: 15.7 against
        // 8 us per 4096-env step, profiles/r05c_kernel_stats.md)  // empty look-ahead slots reset in k_env_fallback
        if (O.act.part)
            hipLaunchKernelGGL((k_env_step<SP, true, true>), dim3(nb), dim3(SBLK), 0, s, E, O);
        else
            hipLaunchKernelGGL((k_env_step<SP, true>), dim3(nb), dim3(SBLK), 0, s, E, O);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        // (no_fallback: the caller refills every used slot after every step, before the next one -- PPO's rollout --
        // so no reset can find its slot empty; the pass and its graph node are left out)
        if (!O.no_fallback)
            hipLaunchKernelGGL(k_env_fallback<SP>, dim3((nb + BLK - 1) / BLK), dim3(BLK), 0, s, E, O.obs);
    } else {
        hipLaunchKernelGGL((k_env_step<SP, false>), dim3(nb), dim3(SBLK), 0, s, E, O);
    }
    return hipGetLastError();
}

hipError_t launch_env_step(const EnvDev &E, const StepOut &O, bool refill, hipStream_t s) {
    hipError_t e = E.sp == 16 ? launch_step_sp<16>(E, O, s) : launch_step_sp<32>(E, O, s);
    return (e != hipSuccess || !refill) ? e : launch_env_refill(E, false, s);
}

hipError_t launch_env_full_obs(const EnvDev &E, uint8_t *out, hipStream_t s) {
    const int64_t total = (int64_t)E.n * E.size * E.size;
    if (total <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_env_full_obs, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, E, out);
    return hipGetLastError();
}

}  // namespace merlin
