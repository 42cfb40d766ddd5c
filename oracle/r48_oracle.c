/*
 * oracle/r48_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * Plain-C restatement of the reference 2048 environment (nevertiree/Rein48,
 * game/GameClient.py) over the build's board layout, used by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg. Nothing in
 * rein48_amd/ links, loads or calls this file.
 *
 * Board layout (shared with the HIP kernel): int8 e[16], row-major, cell (r,c) at 4*r+c,
 * e = 0 empty, e > 0 means tile value 2^e.  The reference stores raw values in a
 * list[list[int]]; doubling a value (merge) is e+1 here.
 *
 * Pinned by tests/golden/ (generated from the reference itself): the 40 line KATs,
 * the filled / game-over KATs, the SHA-256 of the exhaustive 18^4-line table, and
 * 64 seeded reference trajectories replayed bit-for-bit through the CPython-compatible
 * MT19937 below.
 */
#include <stdint.h>
#include <string.h>

#define ORC_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------------------------
 * Line move: the reference's two-pointer slide/merge, GameClient.py:141-179 (UP form;
 * DOWN :183-203, LEFT :207-227, RIGHT :231-251 are the same loop over a differently
 * ordered line).  `line[0]` is the cell the tiles move toward.  i trails, j scans ahead:
 *   - j skips empties (:147-148); j past the end ends the line (:150-152)
 *   - line[i] empty        -> line[i] takes line[j]                     (:156-160)
 *   - line[i] == line[j]   -> merge into line[i] (value doubles = e+1), i advances (:162-167)
 *   - line[i] != line[j]   -> line[j] moves to i+1 (if it is not already there), i advances
 *                                                                          (:169-176)
 *   - j advances (:179)
 * Returns the merge reward in raw tile values (sum of the merged tiles' new values); the
 * reference always reports reward 0 (GameClient.py:138), that figure is the opt-in mode.
 * ---------------------------------------------------------------------------------- */
static int64_t move_line(int8_t *const *cell, int n)
{
    int64_t reward = 0;
    int i = 0, j = 1;
    while (j < n) {
        while (j < n && *cell[j] == 0)
            j++;
        if (j == n)
            break;
        if (*cell[i] == 0) {
            *cell[i] = *cell[j];
            *cell[j] = 0;
        } else if (*cell[i] == *cell[j]) {
            *cell[i] = (int8_t)(*cell[i] + 1);
            *cell[j] = 0;
            reward += (int64_t)1 << *cell[i];
            i++;
        } else {
            if (i + 1 != j) {
                *cell[i + 1] = *cell[j];
                *cell[j] = 0;
            }
            i++;
        }
        j++;
    }
    return reward;
}

/* Pointers to the 4 lines of a 4x4 board in move order for action a:
 * 0 UP (column, top first), 1 DOWN (column, bottom first), 2 LEFT (row, left first),
 * 3 RIGHT (row, right first) -- the action codes of GameClient.py:140,182,206,230. */
static void line_ptrs(int8_t *b, int a, int line, int8_t *p[4])
{
    for (int k = 0; k < 4; k++) {
        int r, c;
        switch (a) {
        case 0: r = k;     c = line; break;
        case 1: r = 3 - k; c = line; break;
        case 2: r = line;  c = k;    break;
        default: r = line; c = 3 - k; break;
        }
        p[k] = &b[4 * r + c];
    }
}

/* update_matrix (GameClient.py:129-254) on one board: returns 1 if the board changed
 * (the reference's `origin_matrix != matrix`, :137/:180), -1 on a bad action (the
 * reference raises ValueError, :254; here the board is left as it was). */
ORC_API int orc_move(int8_t *b, int a, int64_t *reward)
{
    if (a < 0 || a > 3)
        return -1;
    int8_t orig[16];
    memcpy(orig, b, 16);
    int64_t rw = 0;
    for (int line = 0; line < 4; line++) {
        int8_t *p[4];
        line_ptrs(b, a, line, p);
        rw += move_line(p, 4);
    }
    if (reward)
        *reward = rw;
    return memcmp(orig, b, 16) != 0;
}

/* Generic line form used for the exhaustive table: `n`-cell line already in move order. */
ORC_API int orc_move_line(int8_t *line, int n)
{
    int8_t orig[64];
    int8_t *p[64];
    if (n < 1 || n > 64)
        return -1;
    memcpy(orig, line, (size_t)n);
    for (int k = 0; k < n; k++)
        p[k] = &line[k];
    move_line(p, n);
    return memcmp(orig, line, (size_t)n) != 0;
}

/* Exhaustive 18^4 x 4 table, the layout tests/golden/line_table.json hashes:
 * out int8[4][18^4][4], chg uint8[4][18^4]. For UP/LEFT the line's cell 0 is the
 * matrix's first cell; for DOWN/RIGHT the reference walks the line from the far end, so
 * the line is reversed before and after the move. */
ORC_API void orc_line_table(int8_t *out, uint8_t *chg)
{
    const int n = 18 * 18 * 18 * 18;
    for (int d = 0; d < 4; d++) {
        for (int idx = 0; idx < n; idx++) {
            int8_t cells[4];
            int t = idx;
            for (int k = 3; k >= 0; k--) {
                cells[k] = (int8_t)(t % 18);
                t /= 18;
            }
            int8_t line[4];
            int rev = (d == 1 || d == 3);
            for (int k = 0; k < 4; k++)
                line[k] = rev ? cells[3 - k] : cells[k];
            int c = orc_move_line(line, 4);
            int8_t *o = out + ((size_t)d * n + idx) * 4;
            for (int k = 0; k < 4; k++)
                o[k] = rev ? line[3 - k] : line[k];
            chg[(size_t)d * n + idx] = (uint8_t)c;
        }
    }
}

/* has_table_filled (GameClient.py:96-100) and has_game_over (:65-94): over iff the
 * board has no empty cell and no two orthogonal neighbours are equal. */
ORC_API int orc_filled(const int8_t *b)
{
    for (int k = 0; k < 16; k++)
        if (b[k] == 0)
            return 0;
    return 1;
}

ORC_API int orc_game_over(const int8_t *b)
{
    if (!orc_filled(b))
        return 0;
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) {
            if (r + 1 < 4 && b[4 * r + c] == b[4 * (r + 1) + c])
                return 0;
            if (c + 1 < 4 && b[4 * r + c] == b[4 * r + c + 1])
                return 0;
        }
    return 1;
}

ORC_API int orc_blank_count(const int8_t *b)
{
    int n = 0;
    for (int k = 0; k < 16; k++)
        n += (b[k] == 0);
    return n;
}

/* random_fill_grid (GameClient.py:102-127) given its two draws: the blanks are listed in
 * row-major order (:109-114), `rank` picks one (:121-122), the tile is 4 (e=2) when
 * `four`, else 2 (e=1) (:125). No blank -> unchanged (:117-118). Returns the cell or -1. */
ORC_API int orc_spawn(int8_t *b, int rank, int four)
{
    int seen = 0;
    for (int k = 0; k < 16; k++) {
        if (b[k] == 0) {
            if (seen == rank) {
                b[k] = four ? 2 : 1;
                return k;
            }
            seen++;
        }
    }
    return -1;
}

/* The build's Philox-mode spawn: the same uniform choice among the
 * blanks, counted in LINE order for action a instead of row-major: k = 0..3 cells from the
 * wall the tiles moved toward, then line l = 0..3 -- cell (k, l) is (row k, col l) for UP,
 * (row 3-k, col l) DOWN, (row l, col k) LEFT, (row l, col 3-k) RIGHT. */
ORC_API int orc_spawn_lines(int8_t *b, int a, int rank, int four)
{
    int seen = 0;
    for (int k = 0; k < 4; k++)
        for (int l = 0; l < 4; l++) {
            int r = a == 0 ? k : a == 1 ? 3 - k : l;
            int c = a < 2 ? l : a == 2 ? k : 3 - k;
            int cell = 4 * r + c;
            if (b[cell] == 0) {
                if (seen == rank) {
                    b[cell] = four ? 2 : 1;
                    return cell;
                }
                seen++;
            }
        }
    return -1;
}

/* ------------------------------------------------------------------------------------
 * CPython `random` (Python 3.10, Modules/_randommodule.c + Lib/random.py semantics):
 * MT19937 seeded by init_by_array over the 32-bit words of abs(seed), getrandbits(k<=32) =
 * genrand >> (32-k), _randbelow(n) = rejection on getrandbits(n.bit_length()),
 * random() = (a>>5 * 2^26 + b>>6) / 2^53.  The reference draws with
 * random.randint (GameClient.py:121; control/rand.py:11) and random.uniform (:125).
 * ---------------------------------------------------------------------------------- */
#define MT_N 624
#define MT_M 397

typedef struct {
    uint32_t mt[MT_N];
    int idx;
} orc_mt;

ORC_API int orc_mt_state_size(void) { return (int)sizeof(orc_mt); }

static void mt_init_genrand(orc_mt *s, uint32_t seed)
{
    s->mt[0] = seed;
    for (int i = 1; i < MT_N; i++)
        s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
    s->idx = MT_N;
}

static void mt_init_by_array(orc_mt *s, const uint32_t *key, int len)
{
    mt_init_genrand(s, 19650218u);
    int i = 1, j = 0;
    for (int k = (MT_N > len ? MT_N : len); k; k--) {
        s->mt[i] = (s->mt[i] ^ ((s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        i++;
        j++;
        if (i >= MT_N) {
            s->mt[0] = s->mt[MT_N - 1];
            i = 1;
        }
        if (j >= len)
            j = 0;
    }
    for (int k = MT_N - 1; k; k--) {
        s->mt[i] = (s->mt[i] ^ ((s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
        i++;
        if (i >= MT_N) {
            s->mt[0] = s->mt[MT_N - 1];
            i = 1;
        }
    }
    s->mt[0] = 0x80000000u;
    s->idx = MT_N;
}

static uint32_t mt_next(orc_mt *s)
{
    if (s->idx >= MT_N) {
        for (int k = 0; k < MT_N; k++) {
            uint32_t y = (s->mt[k] & 0x80000000u) | (s->mt[(k + 1) % MT_N] & 0x7fffffffu);
            s->mt[k] = s->mt[(k + MT_M) % MT_N] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        s->idx = 0;
    }
    uint32_t y = s->mt[s->idx++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

/* random.seed(n) for a non-negative integer n < 2^64 */
ORC_API void orc_mt_seed(orc_mt *s, uint64_t seed)
{
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    mt_init_by_array(s, key, key[1] ? 2 : 1);
}

ORC_API uint32_t orc_mt_getrandbits(orc_mt *s, int k)
{
    return mt_next(s) >> (32 - k);
}

ORC_API uint32_t orc_mt_randbelow(orc_mt *s, uint32_t n)
{
    int k = 0;
    for (uint32_t t = n; t; t >>= 1)
        k++;
    uint32_t r = orc_mt_getrandbits(s, k);
    while (r >= n)
        r = orc_mt_getrandbits(s, k);
    return r;
}

ORC_API double orc_mt_random(orc_mt *s)
{
    uint32_t a = mt_next(s) >> 5, b = mt_next(s) >> 6;
    return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
}

/* random_fill_grid with the reference's own draws: randint(0, n_blank-1) then
 * uniform(0,1) > 0.1 -> 2 else 4 (GameClient.py:121,125). No blank: no draw (:117-118). */
static void pyrand_fill(orc_mt *s, int8_t *b, int32_t *rank, int32_t *four)
{
    int nb = orc_blank_count(b);
    *rank = -1;
    *four = -1;
    if (!nb)
        return;
    int r = (int)orc_mt_randbelow(s, (uint32_t)nb);
    double u = orc_mt_random(s);
    int f = !(u > 0.1);
    orc_spawn(b, r, f);
    *rank = r;
    *four = f;
}

/* One reference episode driven exactly like main.py:36-42 with control/rand.py's policy,
 * continuing the given MT stream: Game() -> reset (one spawn, :33-38), then
 * Rand.random_action (randint(0,3), rand.py:11) -> step (:40-51) until done or max_steps.
 * Writes start board + per-step (before, action, after, done, changed, rank, four).
 * Returns the number of steps. */
ORC_API int orc_pyrand_episode(orc_mt *s, int max_steps, int8_t *start, int32_t *start_draw,
                               int8_t *before, int32_t *action, int8_t *after, uint8_t *done,
                               uint8_t *changed, int32_t *rank, int32_t *four)
{
    int8_t b[16] = {0};
    pyrand_fill(s, b, &start_draw[0], &start_draw[1]);
    memcpy(start, b, 16);
    int t = 0;
    for (; t < max_steps; t++) {
        memcpy(before + 16 * t, b, 16);
        int a = (int)orc_mt_randbelow(s, 4);
        action[t] = a;
        int c = orc_move(b, a, 0);
        changed[t] = (uint8_t)c;
        rank[t] = -1;
        four[t] = -1;
        if (c)
            pyrand_fill(s, b, &rank[t], &four[t]);
        memcpy(after + 16 * t, b, 16);
        done[t] = (uint8_t)orc_game_over(b);
        if (done[t]) {
            t++;
            break;
        }
    }
    return t;
}

/* ------------------------------------------------------------------------------------
 * Philox4x32 (Salmon et al., SC'11) -- the production RNG of the HIP kernel. Only the
 * build defines how its words are used (the reference has no counter-based RNG); this is
 * the specification the kernel must match bit-for-bit (contract version 3
 * = R48_DRAW_CONTRACT in include/rein48.h):
 *   key = {seed lo, seed hi}
 *   step:  Philox4x32-7; boards with global ids 2q and 2q+1 share ctr = {q lo, q hi, step, 0x2048}; the even
 *          board takes (x, y) = (w0, w1), the odd one (w2, w3). Per board: action x >> 30 in
 *          random-policy mode; spawn a 4 iff (x & 0x3FFFFFFF) < 0x06666666; spawn rank
 *          mulhi(y, n_blank) with the blanks counted in LINE order of the action
 *          (orc_spawn_lines); auto-reset tile: cell y >> 28 (row-major), a 4 iff
 *          (y & 0x0FFFFFFF) < 0x0199999A (y is free then: a step that ends done spawned into
 *          its last blank, mulhi(y, 1) = 0, or spawned nothing).
 *          Contract version 1 (round 1) counted the spawn rank in row-major order, version 2
 *          (rounds 2-3) drew the step words from Philox4x32-10: seeds saved under either do not
 *          replay under version 3.
 *   reset: Philox4x32-10, ctr = {gid lo, gid hi, reset_ctr, 0x5E7} -> cell w0 >> 28, four iff w1 < 0x1999999A
 * ---------------------------------------------------------------------------------- */
/* Philox4x32 with `rounds` rounds (Salmon et al., SC'11): 10 is Random123's default (pinned by its
 * KAT vectors, tests/test_oracle_pinned.py), the env step's draws use 7 (contract version 3) */
ORC_API void orc_philox4x32_r(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4], int rounds)
{
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < rounds; r++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

ORC_API void orc_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4])
{
    orc_philox4x32_r(ctr_in, key_in, out, 10);
}

#define ORC_FLAG_AUTO_RESET 1u
#define ORC_FLAG_RANDOM_POLICY 2u
#define ORC_FLAG_MERGE_REWARD 4u

static inline uint32_t mulhi32(uint32_t a, uint32_t b)
{
    return (uint32_t)(((uint64_t)a * b) >> 32);
}

/* Batched step in the kernel's Philox mode (r48_env_step; draw contract in DESIGN.md section 7):
 * boards with global ids 2q and 2q+1 share Philox4x32-7({q lo, q hi, step, 0x2048}); the even
 * board takes (x, y) = (w0, w1), the odd one (w2, w3). action = x >> 30, spawn a 4 iff
 * (x & 0x3FFFFFFF) < 0x06666666, blank rank = mulhi(y, n_blank) with the blanks in line order
 * (orc_spawn_lines), auto-reset cell = y >> 28 (row-major) with
 * a 4 iff (y & 0x0FFFFFFF) < 0x0199999A. actions are read, or written in random-policy mode.
 * Outputs may be NULL. Returns the number of boards with a bad action. */
ORC_API int64_t orc_step_philox(int8_t *boards, int64_t n, uint64_t seed, int64_t board_offset,
                                uint32_t step, uint32_t flags, int8_t *actions, uint8_t *done,
                                uint8_t *changed, int32_t *reward, int32_t *score)
{
    int64_t bad = 0;
    const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (int64_t i = 0; i < n; i++) {
        int8_t *b = boards + 16 * i;
        /* boards 2q and 2q+1 share one Philox call; the even one takes (w0, w1), the odd one (w2, w3) */
        uint64_t gid = (uint64_t)(board_offset + i), q = gid >> 1;
        uint32_t ctr[4] = {(uint32_t)q, (uint32_t)(q >> 32), step, 0x2048u}, w[4];
        orc_philox4x32_r(ctr, key, w, 7);
        const uint32_t x = w[2 * (gid & 1)], y = w[2 * (gid & 1) + 1];
        int a;
        if (flags & ORC_FLAG_RANDOM_POLICY) {
            a = (int)(x >> 30);
            if (actions)
                actions[i] = (int8_t)a;
        } else {
            a = actions[i];
        }
        int64_t rw = 0;
        int c = orc_move(b, a, &rw);
        if (c < 0) {
            bad++;
            c = 0;
        }
        if (c) {   /* c > 0 implies 0 <= a < 4 */
            int nb = orc_blank_count(b);
            orc_spawn_lines(b, a, (int)mulhi32(y, (uint32_t)nb), (x & 0x3FFFFFFFu) < 0x06666666u);
        }
        int d = orc_game_over(b);
        if (score) {
            int32_t sc = 0;
            for (int k = 0; k < 16; k++)
                sc += b[k] ? (1 << b[k]) : 0;
            score[i] = sc;
        }
        if (d && (flags & ORC_FLAG_AUTO_RESET)) {   /* y is unused by a step that ends done */
            memset(b, 0, 16);
            b[y >> 28] = ((y & 0x0FFFFFFFu) < 0x0199999Au) ? 2 : 1;
        }
        if (done)
            done[i] = (uint8_t)d;
        if (changed)
            changed[i] = (uint8_t)c;
        if (reward)
            reward[i] = (flags & ORC_FLAG_MERGE_REWARD) ? (int32_t)rw : 0;
    }
    return bad;
}

/* Batched step with injected draws (r48_env_step_with_draws): spawn rank taken modulo the
 * blank count, as the kernel does. */
ORC_API int64_t orc_step_draws(int8_t *boards, int64_t n, const int8_t *actions, const uint8_t *rank,
                               const uint8_t *four, uint8_t *done, uint8_t *changed, int32_t *reward,
                               uint32_t flags)
{
    int64_t bad = 0;
    for (int64_t i = 0; i < n; i++) {
        int8_t *b = boards + 16 * i;
        int64_t rw = 0;
        int c = orc_move(b, actions[i], &rw);
        if (c < 0) {
            bad++;
            c = 0;
        }
        if (c) {
            int nb = orc_blank_count(b);
            orc_spawn(b, rank[i] % nb, four[i] != 0);
        }
        if (done)
            done[i] = (uint8_t)orc_game_over(b);
        if (changed)
            changed[i] = (uint8_t)c;
        if (reward)
            reward[i] = (flags & ORC_FLAG_MERGE_REWARD) ? (int32_t)rw : 0;
    }
    return bad;
}

/* reset (GameClient.py:33-38) in Philox mode for masked boards (mask NULL = all). */
ORC_API void orc_reset_philox(int8_t *boards, int64_t n, uint64_t seed, int64_t board_offset,
                              uint32_t reset_ctr, const uint8_t *mask)
{
    const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (int64_t i = 0; i < n; i++) {
        if (mask && !mask[i])
            continue;
        uint64_t gid = (uint64_t)(board_offset + i);
        uint32_t ctr[4] = {(uint32_t)gid, (uint32_t)(gid >> 32), reset_ctr, 0x5E7u}, w[4];
        orc_philox4x32_10(ctr, key, w);
        int8_t *b = boards + 16 * i;
        memset(b, 0, 16);
        b[w[0] >> 28] = (w[1] < 0x1999999Au) ? 2 : 1;
    }
}

/* Synthetic start boards (r48_env_fill_random; SURVEY.md 8(d) bench input, no reference
 * counterpart): two Philox blocks {gid lo, gid hi, j, 0xF111}, j = 0, 1, give 16 half-words,
 * cell c takes half-word c in (block, word, low-then-high) order; odd -> tile
 * 1 + ((h >> 1) * max_exp >> 15), even -> empty. */
ORC_API void orc_fill_random(int8_t *boards, int64_t n, uint64_t seed, int64_t board_offset, uint32_t max_exp)
{
    const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (int64_t i = 0; i < n; i++) {
        uint64_t gid = (uint64_t)(board_offset + i);
        uint32_t w[8];
        for (uint32_t j = 0; j < 2; j++) {
            uint32_t ctr[4] = {(uint32_t)gid, (uint32_t)(gid >> 32), j, 0xF111u};
            orc_philox4x32_10(ctr, key, w + 4 * j);
        }
        for (int c = 0; c < 16; c++) {
            uint32_t h = (c & 1) ? (w[c >> 1] >> 16) : (w[c >> 1] & 0xFFFFu);
            boards[16 * i + c] = (h & 1u) ? (int8_t)(1u + (((h >> 1) * max_exp) >> 15)) : 0;
        }
    }
}

/* Replay sampling draws (rein48_amd/csrc/r48_replay.hip). Ring: uniform with replacement,
 * index = mulhi64(w0 | w1 << 32, size), counter {i lo, i hi, sample_ctr, 0x5A4}. */
ORC_API void orc_replay_ring_index(uint64_t seed, uint32_t sample_ctr, int64_t size, int64_t n, int64_t *out)
{
    const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (int64_t i = 0; i < n; i++) {
        uint32_t ctr[4] = {(uint32_t)i, (uint32_t)((uint64_t)i >> 32), sample_ctr, 0x5A4u}, w[4];
        orc_philox4x32_10(ctr, key, w);
        const uint64_t u = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
        out[i] = (int64_t)(((unsigned __int128)u * (uint64_t)size) >> 64);
    }
}

/* Fill-drain sampling without replacement (replay.py:34's random.sample, restated with a keyed
 * permutation): a 4-round balanced Feistel network on 2h bits (h = ceil(ceil(log2 size) / 2),
 * h >= 1), round j: (L, R) -> (R, L ^ (Philox({R, sample_ctr, j, 0x5A3}).w0 & (2^h - 1))),
 * cycle-walked until the value is < size. Row i < n (n <= size) takes slot perm(i). */
static uint64_t orc_feistel(uint64_t x, uint32_t h, uint32_t ctr, const uint32_t key[2])
{
    const uint64_t mask = (1ull << h) - 1ull;
    uint64_t L = x >> h, R = x & mask;
    for (uint32_t j = 0; j < 4; j++) {
        uint32_t c[4] = {(uint32_t)R, ctr, j, 0x5A3u}, w[4];
        orc_philox4x32_10(c, key, w);
        const uint64_t nl = R;
        R = L ^ ((uint64_t)w[0] & mask);
        L = nl;
    }
    return (L << h) | R;
}

ORC_API void orc_replay_perm_index(uint64_t seed, uint32_t sample_ctr, int64_t size, int64_t n, int64_t *out)
{
    const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t k = 1;
    while (k < 63 && ((int64_t)1 << k) < size)
        k++;
    const uint32_t h = (k + 1) / 2;
    for (int64_t i = 0; i < n; i++) {
        uint64_t x = (uint64_t)i;
        do
            x = orc_feistel(x, h, sample_ctr, key);
        while (x >= (uint64_t)size);
        out[i] = (int64_t)x;
    }
}

/* Tile-value sum per board: main.py:48's np.sum(state_matrix). */
ORC_API void orc_score(const int8_t *boards, int64_t n, int32_t *out)
{
    for (int64_t i = 0; i < n; i++) {
        int32_t s = 0;
        for (int k = 0; k < 16; k++)
            s += boards[16 * i + k] ? (1 << boards[16 * i + k]) : 0;
        out[i] = s;
    }
}

/* CPU "strong baseline": one board, reference semantics, random policy with the CPython
 * RNG, auto-reset on done, for `steps` steps. Returns the number of episodes finished. */
ORC_API int64_t orc_bench_pyrand(uint64_t seed, int64_t steps)
{
    orc_mt s;
    orc_mt_seed(&s, seed);
    int8_t b[16] = {0};
    int32_t r, f;
    int64_t episodes = 0;
    pyrand_fill(&s, b, &r, &f);
    for (int64_t t = 0; t < steps; t++) {
        int a = (int)orc_mt_randbelow(&s, 4);
        if (orc_move(b, a, 0))
            pyrand_fill(&s, b, &r, &f);
        if (orc_game_over(b)) {
            episodes++;
            memset(b, 0, 16);
            pyrand_fill(&s, b, &r, &f);
        }
    }
    return episodes;
}
