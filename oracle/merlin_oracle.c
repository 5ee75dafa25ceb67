/*
 * merlin_oracle.c -- TEST INFRASTRUCTURE ONLY: CPU restatement used as the
 * parity checker and as bench.py's cpu_baseline env.  See merlin_oracle.h for
 * the pinning status of each part.  Every function cites the reference
 * file:line (paths relative to the reference checkout) or, for third-party
 * code that is not vendored, the pinned package + function it restates
 * (minigrid 3.0.0 uv.lock:467-469, gymnasium 1.2.1 uv.lock:242-244,
 * numpy >=2 `Generator`/`PCG64`/`SeedSequence`).
 *
 * Build: see oracle/Makefile (gcc -O2 -ffp-contract=off).
 */
#include "merlin_oracle.h"

#include <string.h>

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------------ */
/* numpy SeedSequence (numpy/random/bit_generator.pyx: mix_entropy,
 * generate_state) -> PCG64 seeding (numpy/random/_pcg64.pyx __init__ ->
 * pcg64_set_seed -> pcg_setseq_128_srandom_r).  gymnasium seeding.np_random
 * (gymnasium 1.2.1 utils/seeding.py) = Generator(PCG64(SeedSequence(seed))). */
#define SS_INIT_A 0x43b0d7e5u
#define SS_MULT_A 0x931e8875u
#define SS_INIT_B 0x8b51f9ddu
#define SS_MULT_B 0x58f38dedu
#define SS_MIX_L 0xca01f9ddu
#define SS_MIX_R 0x4973f715u

static uint32_t ss_hashmix(uint32_t value, uint32_t *hc) {
    value ^= *hc;
    *hc *= SS_MULT_A;
    value *= *hc;
    value ^= value >> 16;
    return value;
}

static uint32_t ss_mix(uint32_t x, uint32_t y) {
    uint32_t r = SS_MIX_L * x - SS_MIX_R * y;
    r ^= r >> 16;
    return r;
}

static const u128 PCG_MULT = (((u128)0x2360ed051fc65da4ULL) << 64) | 0x4385df649fccf645ULL;

static void pcg_step(o_pcg64 *r) {
    u128 s = (((u128)r->st_hi) << 64) | r->st_lo;
    u128 inc = (((u128)r->inc_hi) << 64) | r->inc_lo;
    s = s * PCG_MULT + inc;
    r->st_hi = (uint64_t)(s >> 64);
    r->st_lo = (uint64_t)s;
}

void o_seedseq_pcg64(uint64_t seed, o_pcg64 *out) {
    uint32_t ent[2];
    int n_ent = 0;
    /* _int_to_uint32_array: little-endian 32-bit words, [0] for 0 */
    if (seed == 0) {
        ent[n_ent++] = 0;
    } else {
        uint64_t s = seed;
        while (s) {
            ent[n_ent++] = (uint32_t)(s & 0xffffffffu);
            s >>= 32;
        }
    }
    uint32_t pool[4];
    uint32_t hc = SS_INIT_A;
    for (int i = 0; i < 4; i++) pool[i] = ss_hashmix(i < n_ent ? ent[i] : 0u, &hc);
    for (int s = 0; s < 4; s++)
        for (int d = 0; d < 4; d++)
            if (s != d) pool[d] = ss_mix(pool[d], ss_hashmix(pool[s], &hc));
    /* (no remaining entropy words beyond the pool for <=2-word seeds) */
    uint32_t words[8];
    uint32_t hb = SS_INIT_B;
    for (int i = 0; i < 8; i++) {
        uint32_t v = pool[i & 3];
        v ^= hb;
        hb *= SS_MULT_B;
        v *= hb;
        v ^= v >> 16;
        words[i] = v;
    }
    uint64_t st64[4];
    for (int i = 0; i < 4; i++) st64[i] = (uint64_t)words[2 * i] | ((uint64_t)words[2 * i + 1] << 32);
    /* pcg64_set_seed(state, seed=&val[0], inc=&val[2]); PCG_128BIT_CONSTANT(high=[0], low=[1]) */
    u128 initstate = (((u128)st64[0]) << 64) | st64[1];
    u128 initseq = (((u128)st64[2]) << 64) | st64[3];
    u128 inc = (initseq << 1) | 1u;
    out->inc_hi = (uint64_t)(inc >> 64);
    out->inc_lo = (uint64_t)inc;
    out->st_hi = 0;
    out->st_lo = 0;
    pcg_step(out);
    u128 s = ((((u128)out->st_hi) << 64) | out->st_lo) + initstate;
    out->st_hi = (uint64_t)(s >> 64);
    out->st_lo = (uint64_t)s;
    pcg_step(out);
    out->has32 = 0;
    out->buf32 = 0;
}

/* pcg_setseq_128_xsl_rr_64_random_r: step, then XSL-RR output */
uint64_t o_next64(o_pcg64 *r) {
    pcg_step(r);
    uint64_t x = r->st_hi ^ r->st_lo;
    unsigned rot = (unsigned)(r->st_hi >> 58);
    return (x >> rot) | (x << ((64 - rot) & 63));
}

/* pcg64_next32: persistent low-half / high-half buffer */
uint32_t o_next32(o_pcg64 *r) {
    if (r->has32) {
        r->has32 = 0;
        return r->buf32;
    }
    uint64_t n = o_next64(r);
    r->has32 = 1;
    r->buf32 = (uint32_t)(n >> 32);
    return (uint32_t)n;
}

/* buffered_bounded_lemire_uint32 with rng = range-1 (inclusive) */
static uint32_t lemire32(o_pcg64 *r, uint32_t rng_incl) {
    const uint32_t rng_excl = rng_incl + 1u;
    uint64_t m = (uint64_t)o_next32(r) * rng_excl;
    uint32_t left = (uint32_t)m;
    if (left < rng_excl) {
        const uint32_t thresh = (uint32_t)(0xffffffffu - rng_incl) % rng_excl;
        while (left < thresh) {
            m = (uint64_t)o_next32(r) * rng_excl;
            left = (uint32_t)m;
        }
    }
    return (uint32_t)(m >> 32);
}

/* Generator.integers(lo, hi) scalar int64 path -> random_bounded_uint64_fill
 * (numpy/random/src/distributions/distributions.c); ranges here are < 2^32. */
int64_t o_integers(o_pcg64 *r, int64_t lo, int64_t hi) {
    uint64_t rng = (uint64_t)(hi - lo - 1);
    if (rng == 0) return lo;
    if (rng == 0xffffffffULL) return lo + (int64_t)o_next32(r);
    return lo + (int64_t)lemire32(r, (uint32_t)rng);
}

/* Generator.choice(pop, k, replace=False, shuffle=True), pop <= 10000:
 * Floyd's algorithm followed by _shuffle_int(k, 1) (numpy/random/_generator.pyx). */
void o_choice_noreplace(o_pcg64 *r, int64_t pop, int64_t k, int64_t *idx) {
    for (int64_t j = pop - k; j < pop; j++) {
        int64_t val = (j == 0) ? 0 : (int64_t)lemire32(r, (uint32_t)j);
        int dup = 0;
        for (int64_t q = 0; q < j - (pop - k); q++)
            if (idx[q] == val) dup = 1;
        idx[j - (pop - k)] = dup ? j : val;
    }
    for (int64_t i = k - 1; i >= 1; i--) {
        int64_t j = (int64_t)lemire32(r, (uint32_t)i);
        int64_t t = idx[j];
        idx[j] = idx[i];
        idx[i] = t;
    }
}

/* ------------------------------------------------------------------------ */
/* Env: minigrid 3.0.0 MiniGridEnv + MERLIN generators                       */

static inline uint8_t cget(const o_env *e, int x, int y) { return e->cell[y * e->size + x]; }
static inline void cset(o_env *e, int x, int y, uint8_t v) { e->cell[y * e->size + x] = v; }

void o_env_init(o_env *e, int size, int difficulty, int max_steps) {
    memset(e, 0, sizeof(*e));
    e->size = size;
    e->difficulty = difficulty;
    /* base_env.py:32-33: max_steps = 4 * size**2 when not given */
    e->max_steps = max_steps > 0 ? max_steps : 4 * size * size;
    e->ax = e->ay = -1;
    e->dir = -1;
    e->max_stay = 3;
    e->penalty = -0.1;
}

void o_env_set_stuck(o_env *e, int on, int max_stay, double penalty) {
    e->stuck_on = on;
    e->max_stay = max_stay;
    e->penalty = penalty;
}

void o_env_set_explore(o_env *e, int on, double bonus) {
    e->explore_on = on;
    e->bonus = bonus;
}

/* Grid(width,height) + wall_rect(0,0,W,H) (minigrid core/grid.py) */
static void grid_walled(o_env *e) {
    int S = e->size;
    memset(e->cell, O_EMPTY, sizeof(e->cell));
    for (int x = 0; x < S; x++) {
        cset(e, x, 0, O_WALL);
        cset(e, x, S - 1, O_WALL);
    }
    for (int y = 0; y < S; y++) {
        cset(e, 0, y, O_WALL);
        cset(e, S - 1, y, O_WALL);
    }
}

/* MiniGridEnv.place_obj(obj, top, size, max_tries) (minigrid_env.py):
 * x drawn before y; reject occupied cells and the agent's current position. */
static int place_obj(o_env *e, uint8_t obj, int tx, int ty, int sw, int sh, int max_tries, int *px,
                     int *py) {
    int S = e->size;
    if (tx < 0) tx = 0;
    if (ty < 0) ty = 0;
    long tries = 0;
    for (;;) {
        if (max_tries >= 0 && tries > max_tries) {
            e->error = 1; /* RecursionError("rejection sampling failed in place_obj") */
            return -1;
        }
        tries++;
        int x = (int)o_integers(&e->rng, tx, (tx + sw < S) ? tx + sw : S);
        int y = (int)o_integers(&e->rng, ty, (ty + sh < S) ? ty + sh : S);
        if (cget(e, x, y) != O_EMPTY) continue;
        if (x == e->ax && y == e->ay) continue;
        if (obj != O_EMPTY) cset(e, x, y, obj);
        *px = x;
        *py = y;
        return 0;
    }
}

/* MiniGridEnv.place_agent(top, size, rand_dir=True) */
static void place_agent(o_env *e, int tx, int ty, int sw, int sh) {
    int x, y;
    e->ax = -1;
    e->ay = -1;
    place_obj(e, O_EMPTY, tx, ty, sw, sh, -1, &x, &y);
    e->ax = x;
    e->ay = y;
    e->dir = (int)o_integers(&e->rng, 0, 4);
}

static void place_goal_anywhere(o_env *e) {
    int x, y;
    place_obj(e, O_GOAL, 0, 0, e->size, e->size, -1, &x, &y);
    e->gx = x;
    e->gy = y;
}

/* MediumHardEnv._is_reachable (medium_hard_env.py:47-74): 4-neighbour BFS over
 * cells that are empty or the goal.  Restated as an explicit-queue BFS. */
int o_is_reachable(const o_env *e, int sx, int sy, int gx, int gy) {
    int S = e->size;
    static const int DX[4] = {0, 1, 0, -1}, DY[4] = {1, 0, -1, 0};
    uint8_t vis[O_MAXS * O_MAXS];
    int qx[O_MAXS * O_MAXS], qy[O_MAXS * O_MAXS];
    memset(vis, 0, sizeof(vis));
    int h = 0, t = 0;
    vis[sy * S + sx] = 1;
    qx[t] = sx;
    qy[t] = sy;
    t++;
    while (h < t) {
        int cx = qx[h], cy = qy[h];
        h++;
        if (cx == gx && cy == gy) return 1;
        for (int k = 0; k < 4; k++) {
            int nx = cx + DX[k], ny = cy + DY[k];
            if (nx < 0 || ny < 0 || nx >= S || ny >= S) continue;
            if (vis[ny * S + nx]) continue;
            uint8_t c = cget(e, nx, ny);
            if (c == O_EMPTY || c == O_GOAL || (nx == gx && ny == gy)) {
                vis[ny * S + nx] = 1;
                qx[t] = nx;
                qy[t] = ny;
                t++;
            }
        }
    }
    return 0;
}

/* fallback shared by mediumhard/hard/hardest (medium_hard_env.py:40-45 etc.) */
static void gen_fallback(o_env *e) {
    e->fallbacks++;
    grid_walled(e);
    place_agent(e, 0, 0, e->size, e->size);
    place_goal_anywhere(e);
}

/* EasyEnv._gen_grid (easy_env.py:19-39) */
static void gen_easy(o_env *e) {
    int S = e->size;
    grid_walled(e);
    place_agent(e, 0, 0, S, S);
    /* put_obj(Goal(), W-5, H-5): may land on the agent (goal can_overlap) */
    cset(e, S - 5, S - 5, O_GOAL);
    e->gx = S - 5;
    e->gy = S - 5;
}

/* MediumEnv._gen_grid (medium_env.py:19-33) */
static void gen_medium(o_env *e) {
    grid_walled(e);
    place_agent(e, 0, 0, e->size, e->size);
    place_goal_anywhere(e);
}

/* MediumHardEnv._gen_grid (medium_hard_env.py:12-45) */
static void gen_mediumhard(o_env *e) {
    int S = e->size;
    for (int attempt = 0; attempt < 100; attempt++) {
        e->attempts = attempt + 1;
        grid_walled(e);
        int playable = (S - 2) * (S - 2);
        int min_obs = (int)(playable * 0.10);
        int max_obs = (int)(playable * 0.20);
        int lo = min_obs > 1 ? min_obs : 1;
        int hi = (max_obs > 1 ? max_obs : 1) + 1;
        int n = (int)o_integers(&e->rng, lo, hi);
        for (int i = 0; i < n; i++) {
            int x, y;
            /* agent_pos still holds the previous attempt's position */
            if (place_obj(e, O_WALL, 0, 0, S, S, 100, &x, &y) != 0) return;
        }
        place_agent(e, 0, 0, S, S);
        place_goal_anywhere(e);
        if (o_is_reachable(e, e->ax, e->ay, e->gx, e->gy)) return;
    }
    gen_fallback(e);
}

/* HardEnv._gen_grid (hard_env.py:11-73), agent_start_pos None, random_goal True */
static void gen_hard(o_env *e) {
    int S = e->size;
    for (int attempt = 0; attempt < 100; attempt++) {
        e->attempts = attempt + 1;
        grid_walled(e);
        int mid = S / 2;
        int large = S > 10;
        int num_gaps = large ? (int)o_integers(&e->rng, 2, 6) : 1;
        int64_t gi[32];
        /* choice(list(range(1, S-1)), size=num_gaps, replace=False) */
        o_choice_noreplace(&e->rng, S - 2, num_gaps, gi);
        for (int i = 1; i < S - 1; i++) {
            int is_gap = 0;
            for (int q = 0; q < num_gaps; q++)
                if (gi[q] + 1 == i) is_gap = 1;
            if (!is_gap) cset(e, mid, i, O_WALL);
        }
        if (large) {
            int extra = (int)o_integers(&e->rng, 6, 13);
            for (int w = 0; w < extra; w++) {
                for (int k = 0; k < 10; k++) {
                    int x = (int)o_integers(&e->rng, 1, S - 1);
                    int y = (int)o_integers(&e->rng, 1, S - 1);
                    if (x != mid && cget(e, x, y) == O_EMPTY) {
                        cset(e, x, y, O_WALL);
                        break;
                    }
                }
            }
        }
        int x, y;
        place_obj(e, O_GOAL, mid + 1, 0, S - mid - 1, S, -1, &x, &y);
        e->gx = x;
        e->gy = y;
        place_agent(e, 1, 1, mid - 1, S - 2);
        if (o_is_reachable(e, e->ax, e->ay, e->gx, e->gy)) return;
    }
    gen_fallback(e);
}

/* HardestEnv._gen_grid (hardest_env.py:20-70) */
static void gen_hardest(o_env *e) {
    int S = e->size;
    for (int attempt = 0; attempt < 100; attempt++) {
        e->attempts = attempt + 1;
        grid_walled(e);
        int mx = S / 2, my = S / 2;
        for (int y = 1; y < S - 1; y++) cset(e, mx, y, O_WALL);
        for (int x = 1; x < S - 1; x++) cset(e, x, my, O_WALL);
        int oyt = (int)o_integers(&e->rng, 2, my - 1);
        cset(e, mx, oyt, O_EMPTY);
        int oyb = (int)o_integers(&e->rng, my + 1, S - 2);
        cset(e, mx, oyb, O_EMPTY);
        int oxl = (int)o_integers(&e->rng, 2, mx - 1);
        cset(e, oxl, my, O_EMPTY);
        int oxr = (int)o_integers(&e->rng, mx + 1, S - 2);
        cset(e, oxr, my, O_EMPTY);
        int nobs = (int)o_integers(&e->rng, 6, 13);
        for (int i = 0; i < nobs; i++) {
            int x = (int)o_integers(&e->rng, 1, S - 1);
            int y = (int)o_integers(&e->rng, 1, S - 1);
            if (cget(e, x, y) == O_EMPTY && x != mx && y != my) cset(e, x, y, O_WALL);
        }
        place_agent(e, 0, 0, S, S);
        place_goal_anywhere(e);
        if (o_is_reachable(e, e->ax, e->ay, e->gx, e->gy)) return;
    }
    gen_fallback(e);
}

/* gymnasium Env.reset(seed) + MiniGridEnv.reset (minigrid_env.py) */
void o_env_reset(o_env *e, int has_seed, uint64_t seed) {
    if (has_seed) {
        o_seedseq_pcg64(seed, &e->rng);
        e->rng_ready = 1;
    }
    e->ax = -1;
    e->ay = -1;
    e->dir = -1;
    e->attempts = 1;
    switch (e->difficulty) {
        case O_EASY: gen_easy(e); break;
        case O_MEDIUM: gen_medium(e); break;
        case O_MEDIUMHARD: gen_mediumhard(e); break;
        case O_HARD: gen_hard(e); break;
        default: gen_hardest(e); break;
    }
    e->step_count = 0;
    /* StuckPenaltyWrapper.reset (stuck_penalty_wrapper.py:19-27) */
    e->stay = 0;
    e->last_x = e->ax;
    e->last_y = e->ay;
    /* ExplorationBonus: start cell counts as visited */
    memset(e->visited, 0, sizeof(e->visited));
    e->visited[e->ay] |= 1u << e->ax;
}

static const int DIRX[4] = {1, 0, -1, 0};
static const int DIRY[4] = {0, 1, 0, -1};

/* MiniGridEnv.step (minigrid_env.py) via ThreeActionWrapper (identity map
 * {0:left,1:right,2:forward}, three_action_wrapper.py:16-17), then
 * StuckPenaltyWrapper.step (stuck_penalty_wrapper.py:29-57) if enabled. */
void o_env_step(o_env *e, int64_t action, double *reward, int *terminated, int *truncated) {
    double rew = 0.0;
    int term = 0, trunc = 0;
    e->step_count += 1;
    int fx = e->ax + DIRX[e->dir], fy = e->ay + DIRY[e->dir];
    uint8_t fc = cget(e, fx, fy);
    if (action == 0) {
        e->dir -= 1;
        if (e->dir < 0) e->dir += 4;
    } else if (action == 1) {
        e->dir = (e->dir + 1) % 4;
    } else if (action == 2) {
        if (fc == O_EMPTY || fc == O_GOAL) {
            e->ax = fx;
            e->ay = fy;
        }
        if (fc == O_GOAL) {
            term = 1;
            /* MiniGridEnv._reward: 1 - 0.9 * (step_count / max_steps), float64 */
            rew = 1.0 - 0.9 * ((double)e->step_count / (double)e->max_steps);
        }
    } else {
        e->error = 2; /* IndexError in ThreeActionWrapper._action_map */
    }
    if (e->step_count >= e->max_steps) trunc = 1;
    if (e->stuck_on) {
        if (e->ax == e->last_x && e->ay == e->last_y)
            e->stay += 1;
        else
            e->stay = 0;
        if (e->stay >= e->max_stay) rew += e->penalty;
        e->last_x = e->ax;
        e->last_y = e->ay;
    }
    if (e->explore_on) {
        uint32_t bit = 1u << e->ax;
        if (!(e->visited[e->ay] & bit)) {
            e->visited[e->ay] |= bit;
            rew += e->bonus;
        }
    }
    *reward = rew;
    *terminated = term;
    *truncated = trunc;
}

/* MiniGridEnv.gen_obs_grid -> get_view_exts / Grid.slice / rotate_left^(dir+1)
 * / Grid.process_vis, then Grid.render tile selection as in get_pov_render
 * (agent tile at view (3,6), highlight = vis mask).  Uses the closed form
 * view(vi,vj) <- world(agent + (6-vj)*F + (vi-3)*R), cross-checked against the
 * literal slice+rotate restatement in oracle/minigrid_literal.py. */
void o_env_view_codes(const o_env *e, uint8_t codes[49]) {
    int S = e->size;
    int F0 = DIRX[e->dir], F1 = DIRY[e->dir];
    int R0 = DIRX[(e->dir + 1) & 3], R1 = DIRY[(e->dir + 1) & 3];
    uint8_t v[7][7]; /* v[i][j]: i = view x, j = view y */
    for (int j = 0; j < 7; j++)
        for (int i = 0; i < 7; i++) {
            int wx = e->ax + (6 - j) * F0 + (i - 3) * R0;
            int wy = e->ay + (6 - j) * F1 + (i - 3) * R1;
            v[i][j] = (wx < 0 || wy < 0 || wx >= S || wy >= S) ? O_WALL : cget(e, wx, wy);
        }
    uint8_t m[7][7];
    memset(m, 0, sizeof(m));
    m[3][6] = 1;
    for (int j = 6; j >= 0; j--) {
        for (int i = 0; i < 6; i++) {
            if (!m[i][j]) continue;
            if (v[i][j] == O_WALL) continue; /* Wall.see_behind() == False */
            m[i + 1][j] = 1;
            if (j > 0) {
                m[i + 1][j - 1] = 1;
                m[i][j - 1] = 1;
            }
        }
        for (int i = 6; i >= 1; i--) {
            if (!m[i][j]) continue;
            if (v[i][j] == O_WALL) continue;
            m[i - 1][j] = 1;
            if (j > 0) {
                m[i - 1][j - 1] = 1;
                m[i][j - 1] = 1;
            }
        }
    }
    for (int j = 0; j < 7; j++)
        for (int i = 0; i < 7; i++) {
            uint8_t c;
            if (i == 3 && j == 6)
                c = O_T_AGENT;
            else if (!m[i][j])
                c = O_T_DARK;
            else if (v[i][j] == O_WALL)
                c = O_T_WALL;
            else if (v[i][j] == O_GOAL)
                c = O_T_GOAL;
            else
                c = O_T_EMPTY;
            codes[j * 7 + i] = c;
        }
}

/* ------------------------------------------------------------------------ */
void o_batch_rollout(int n, int size, int difficulty, int max_steps, const uint64_t *seeds, int steps,
                     const int64_t *actions, int stuck_on, int explore_on, double explore_bonus,
                     uint8_t *codes_out, float *reward_out, uint8_t *term_out, uint8_t *trunc_out,
                     int32_t *agent_out) {
    for (int i = 0; i < n; i++) {
        o_env e;
        o_env_init(&e, size, difficulty, max_steps);
        o_env_set_stuck(&e, stuck_on, 3, -0.1);
        o_env_set_explore(&e, explore_on, explore_bonus);
        o_env_reset(&e, 1, seeds[i]);
        if (codes_out) o_env_view_codes(&e, codes_out + (size_t)i * 49);
        if (agent_out) {
            int32_t *a = agent_out + (size_t)i * 4;
            a[0] = e.ax; a[1] = e.ay; a[2] = e.dir; a[3] = e.step_count;
        }
        for (int t = 0; t < steps; t++) {
            double r;
            int te, tr;
            o_env_step(&e, actions[(size_t)t * n + i], &r, &te, &tr);
            size_t k = (size_t)t * n + i;
            reward_out[k] = (float)r;
            term_out[k] = (uint8_t)te;
            trunc_out[k] = (uint8_t)tr;
            if (te || tr) o_env_reset(&e, 0, 0);
            size_t k1 = (size_t)(t + 1) * n + i;
            if (codes_out) o_env_view_codes(&e, codes_out + k1 * 49);
            if (agent_out) {
                int32_t *a = agent_out + k1 * 4;
                a[0] = e.ax; a[1] = e.ay; a[2] = e.dir; a[3] = e.step_count;
            }
        }
    }
}

void o_gen_map(int size, int difficulty, uint64_t seed, uint8_t *cells, int32_t *meta5) {
    o_env e;
    o_env_init(&e, size, difficulty, 0);
    o_env_reset(&e, 1, seed);
    for (int y = 0; y < size; y++)
        for (int x = 0; x < size; x++) cells[y * size + x] = cget(&e, x, y);
    meta5[0] = e.ax;
    meta5[1] = e.ay;
    meta5[2] = e.dir;
    meta5[3] = e.gx;
    meta5[4] = e.gy;
    meta5[5] = e.attempts;
}

/* Grid.render placement: tile (i,j) -> img[8j:8j+8, 8i:8i+8] */
void o_render(const uint8_t *codes, int n, const uint8_t *atlas, uint8_t *out) {
    for (int s = 0; s < n; s++)
        for (int y = 0; y < 56; y++)
            for (int x = 0; x < 56; x++) {
                int c = codes[(size_t)s * 49 + (y / 8) * 7 + (x / 8)];
                for (int ch = 0; ch < 3; ch++)
                    out[(((size_t)s * 56 + y) * 56 + x) * 3 + ch] =
                        atlas[((c * 8 + (y & 7)) * 8 + (x & 7)) * 3 + ch];
            }
}

/* PPO.compute_gae (src/ppo.py:107-120), fp32 tensor op order:
 *   mask  = 1 - d[t]
 *   delta = (r[t] + (gamma*next_val)*mask) - v[t]
 *       t == T-1: gamma*last_value is a Python float product, cast to f32
 *       else    : f32(gamma) * v[t+1]
 *   gae   = delta + (f32(gamma*lam)*mask)*gae
 *   returns = values + adv (un-normalised advantages) */
void o_gae_f32(const float *r, const float *v, const float *d, float last_value, int T, double gamma,
               double lam, float *adv, float *ret) {
    o_gae_f32_tn(r, v, d, &last_value, T, 1, gamma, lam, adv, ret);
}

void o_gae_f32_tn(const float *r, const float *v, const float *d, const float *last_value, int T,
                  int N, double gamma, double lam, float *adv, float *ret) {
    const float gf = (float)gamma;
    const float gl = (float)(gamma * lam);
    for (int i = 0; i < N; i++) {
        float gae = 0.0f;
        for (int t = T - 1; t >= 0; t--) {
            size_t k = (size_t)t * N + i;
            float mask = 1.0f - d[k];
            float gn = (t == T - 1) ? (float)(gamma * (double)last_value[i]) : gf * v[k + N];
            float delta = (r[k] + gn * mask) - v[k];
            gae = delta + (gl * mask) * gae;
            adv[k] = gae;
        }
        for (int t = 0; t < T; t++) {
            size_t k = (size_t)t * N + i;
            ret[k] = v[k] + adv[k];
        }
    }
}

/* ------------------------------------------------------------------------ */
#include <stdlib.h>

o_env *o_env_new(int size, int difficulty, int max_steps) {
    o_env *e = (o_env *)malloc(sizeof(o_env));
    o_env_init(e, size, difficulty, max_steps);
    return e;
}

void o_env_free(o_env *e) { free(e); }

void o_env_reset_codes(o_env *e, int has_seed, uint64_t seed, uint8_t codes[49]) {
    o_env_reset(e, has_seed, seed);
    o_env_view_codes(e, codes);
}

double o_env_step_codes(o_env *e, int64_t action, uint8_t codes[49], int *terminated, int *truncated) {
    double r;
    o_env_step(e, action, &r, terminated, truncated);
    o_env_view_codes(e, codes);
    return r;
}
