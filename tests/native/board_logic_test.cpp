// Host build of the kernel's per-lane board logic (rein48_amd/csrc/r48_board.h) checked
// against the C oracle (oracle/r48_oracle.c) -- a CPU test harness, never shipped.
// Build+run: tests/test_board_logic_host.py (g++ -O2, links the oracle object).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

#include "../../rein48_amd/csrc/r48_board.h"

extern "C" {
int orc_move(int8_t *b, int a, int64_t *reward);
void orc_line_table(int8_t *out, uint8_t *chg);
int orc_game_over(const int8_t *b);
int64_t orc_step_philox(int8_t *boards, int64_t n, uint64_t seed, int64_t board_offset, uint32_t step,
                        uint32_t flags, int8_t *actions, uint8_t *done, uint8_t *changed, int32_t *reward,
                        int32_t *score);
int64_t orc_step_draws(int8_t *boards, int64_t n, const int8_t *actions, const uint8_t *rank,
                       const uint8_t *four, uint8_t *done, uint8_t *changed, int32_t *reward, uint32_t flags);
}

using r48::Board;

static Board load(const int8_t *b)
{
    Board r;
    memcpy(&r, b, 16);
    return r;
}
static void store(int8_t *b, const Board &r) { memcpy(b, &r, 16); }

static int fails = 0;
#define CHECK(cond, ...)                                  \
    do {                                                  \
        if (!(cond)) {                                    \
            if (fails < 20) {                             \
                fprintf(stderr, "FAIL %s:%d ", __FILE__, __LINE__); \
                fprintf(stderr, __VA_ARGS__);             \
                fprintf(stderr, "\n");                    \
            }                                             \
            fails++;                                      \
        }                                                 \
    } while (0)

int main()
{
    // 1. transpose is an involution and a transpose
    {
        int8_t b[16];
        for (int k = 0; k < 16; k++) b[k] = (int8_t)k;
        Board t = r48::transpose(load(b));
        int8_t o[16];
        store(o, t);
        for (int r = 0; r < 4; r++)
            for (int c = 0; c < 4; c++) CHECK(o[4 * r + c] == b[4 * c + r], "transpose %d %d", r, c);
    }
    // 2. exhaustive line table: every 18^4 line in every direction, embedded as line 0..3 of a board
    {
        const int n = 18 * 18 * 18 * 18;
        int8_t *tab = new int8_t[4 * (size_t)n * 4];
        uint8_t *chg = new uint8_t[4 * (size_t)n];
        orc_line_table(tab, chg);
        for (int d = 0; d < 4; d++)
            for (int idx = 0; idx < n; idx++) {
                int8_t cells[4];
                int t = idx;
                for (int k = 3; k >= 0; k--) { cells[k] = (int8_t)(t % 18); t /= 18; }
                const int slot = idx & 3;  // which row/column of the board carries the line
                int8_t b[16] = {0};
                for (int k = 0; k < 4; k++) {
                    if (d < 2) b[4 * k + slot] = cells[k]; else b[4 * slot + k] = cells[k];
                }
                Board L = r48::to_lines(load(b), (uint32_t)d);
                const Board L0 = L;
                r48::move_lines<false>(L);
                Board r = r48::from_lines(L, (uint32_t)d);
                int8_t o[16];
                store(o, r);
                const int8_t *want = tab + ((size_t)d * n + idx) * 4;
                for (int k = 0; k < 4; k++) {
                    int8_t got = d < 2 ? o[4 * k + slot] : o[4 * slot + k];
                    CHECK(got == want[k], "table d=%d idx=%d k=%d got %d want %d", d, idx, k, got, want[k]);
                }
                const bool c = memcmp(&L, &L0, 16) != 0;
                CHECK(c == (chg[(size_t)d * n + idx] != 0), "changed d=%d idx=%d", d, idx);
            }
        delete[] tab;
        delete[] chg;
    }
    // 3. random full boards: move + reward vs oracle, game over vs oracle
    std::mt19937_64 rng(12345);
    {
        for (int it = 0; it < 400000; it++) {
            int8_t b[16];
            const int emax = 1 + (int)(rng() % 17);
            for (int k = 0; k < 16; k++) b[k] = (rng() % 3 == 0) ? 0 : (int8_t)(1 + rng() % emax);
            const int a = (int)(rng() & 3);
            int8_t ob[16];
            memcpy(ob, b, 16);
            int64_t orw = 0;
            const int oc = orc_move(ob, a, &orw);
            Board L = r48::to_lines(load(b), (uint32_t)a);
            const uint32_t rw = r48::move_lines<true>(L);
            int8_t o[16];
            store(o, r48::from_lines(L, (uint32_t)a));
            CHECK(memcmp(o, ob, 16) == 0, "move it=%d a=%d", it, a);
            CHECK((int64_t)rw == orw, "reward it=%d %u vs %lld", it, rw, (long long)orw);
            (void)oc;
            Board rb = load(ob);
            const r48::Blanks bl = r48::blanks(rb);
            CHECK((bool)r48::game_over(rb, bl.n) == (bool)orc_game_over(ob), "over it=%d", it);
        }
    }
    // 4. full step, injected draws and Philox mode, vs the oracle's batched steps
    {
        const int n = 200000;
        int8_t *boards = new int8_t[16 * (size_t)n];
        int8_t *ob = new int8_t[16 * (size_t)n];
        int8_t *act = new int8_t[n];
        uint8_t *rank = new uint8_t[n], *four = new uint8_t[n], *done = new uint8_t[n], *chg = new uint8_t[n];
        int32_t *rw = new int32_t[n], *sc = new int32_t[n];
        for (int i = 0; i < 16 * n; i++) boards[i] = (rng() % 2) ? 0 : (int8_t)(1 + rng() % 8);
        for (int i = 0; i < n; i++) {
            act[i] = (int8_t)(rng() % 5 == 4 ? (int)(rng() % 256) - 128 : (int)(rng() & 3));
            rank[i] = (uint8_t)(rng() % 256);
            four[i] = (uint8_t)(rng() % 2);
        }
        memcpy(ob, boards, 16 * (size_t)n);
        orc_step_draws(ob, n, act, rank, four, done, chg, rw, 4u);
        for (int i = 0; i < n; i++) {
            Board r = load(boards + 16 * i);
            r48::StepOut s = r48::step_board<true, true>(r, (uint32_t)(uint8_t)act[i], rank[i], four[i] != 0);
            int8_t o[16];
            store(o, r);
            CHECK(memcmp(o, ob + 16 * i, 16) == 0, "draws board i=%d a=%d", i, act[i]);
            CHECK(s.done == done[i] && s.changed == chg[i], "draws flags i=%d", i);
            CHECK((int32_t)s.reward == rw[i], "draws reward i=%d", i);
        }
        // Philox random-policy + auto-reset, 3 consecutive steps
        memcpy(ob, boards, 16 * (size_t)n);
        const uint64_t seed = 0x2048'5EEDull;
        const int64_t off = 1000;
        for (uint32_t step = 7; step < 10; step++) {
            orc_step_philox(ob, n, seed, off, step, 1u | 2u, act, done, chg, rw, sc);
            for (int i = 0; i < n; i++) {
                // pair contract (r48::step_draw): boards 2q, 2q+1 share one Philox4x32-7 call; even
                // takes (w0, w1), odd (w2, w3)
                const uint64_t gid = (uint64_t)(off + i);
                uint32_t x, y;
                r48::step_draw(gid, step, (uint32_t)seed, (uint32_t)(seed >> 32), x, y);
                const uint32_t a = x >> 30;
                CHECK((int8_t)a == act[i], "philox action i=%d", i);
                Board r = load(boards + 16 * i);
                r48::StepOut s = r48::step_board<false, false>(r, a, y, (x & 0x3FFFFFFFu) < r48::kFourThresh30);
                CHECK((int32_t)r48::tile_sum(r) == sc[i], "score i=%d", i);
                if (s.done) r48::reset_board(r, y >> 28, (y & 0x0FFFFFFFu) < r48::kFourThresh28);
                store(boards + 16 * i, r);
                CHECK(memcmp(boards + 16 * i, ob + 16 * i, 16) == 0, "philox board i=%d step=%u", i, step);
                CHECK(s.done == done[i] && s.changed == chg[i], "philox flags i=%d", i);
            }
        }
        delete[] boards; delete[] ob; delete[] act; delete[] rank; delete[] four; delete[] done; delete[] chg;
        delete[] rw; delete[] sc;
    }
    // 6. orientation table: from the line form of o, kOrient[4o + a] gives the line form of a
    //    (every (o, a), random boards with distinct cells so any misplaced byte shows)
    {
        std::mt19937 g(7);
        for (int it = 0; it < 2000; it++) {
            int8_t b[16];
            for (int k = 0; k < 16; k++) b[k] = (int8_t)(g() & 0x3f);
            const Board R = load(b);
            for (uint32_t o = 0; o < 4; o++)
                for (uint32_t a = 0; a < 4; a++) {
                    const Board got = r48::reorient(r48::to_lines(R, o), r48::kOrient[4 * o + a]);
                    const Board want = r48::to_lines(R, a);
                    CHECK(memcmp(&got, &want, 16) == 0, "kOrient o=%u a=%u", o, a);
                }
            // back to rows from any line form: kOrient[4o + UP]
            for (uint32_t o = 0; o < 4; o++) {
                const Board got = r48::reorient(r48::to_lines(R, o), r48::kOrient[4 * o]);
                CHECK(memcmp(&got, &R, 16) == 0, "kOrient back to rows o=%u", o);
            }
        }
    }
    // 7. k_step_n's orientation-tracked loop (step_lane_lines in r48_env.hip, restated here on
    //    the host): boards stay in the line form of their last action for many steps, back to
    //    rows at the end == orc_step_philox repeated, random policy + auto-reset
    {
        const int n = 4096, steps = 300;
        int8_t *boards = new int8_t[16 * (size_t)n], *ob = new int8_t[16 * (size_t)n];
        std::mt19937 g(11);
        for (int i = 0; i < n; i++)
            for (int k = 0; k < 16; k++) boards[16 * i + k] = (g() & 1) ? (int8_t)(1 + g() % 7) : 0;
        memcpy(ob, boards, 16 * (size_t)n);
        const uint64_t seed = 0x5EED'2048ull;
        const int64_t off = 2;
        for (uint32_t step = 0; step < (uint32_t)steps; step++)
            orc_step_philox(ob, n, seed, off, 100 + step, 1u | 2u, nullptr, nullptr, nullptr, nullptr, nullptr);
        for (int i = 0; i < n; i++) {
            Board L = load(boards + 16 * i);
            uint32_t o = 0;
            const uint64_t gid = (uint64_t)(off + i);
            for (uint32_t step = 0; step < (uint32_t)steps; step++) {
                uint32_t x, y;
                r48::step_draw(gid, 100 + step, (uint32_t)seed, (uint32_t)(seed >> 32), x, y);
                const uint32_t a = x >> 30;
                L = r48::reorient(L, r48::kOrient[4 * o + a]);
                o = a;
                const r48::StepOut s = r48::step_lines<false, true>(L, a, y, (x & 0x3FFFFFFFu) < r48::kFourThresh30);
                if (s.done) {
                    r48::reset_board(L, y >> 28, (y & 0x0FFFFFFFu) < r48::kFourThresh28);
                    o = 0;
                }
            }
            L = r48::reorient(L, r48::kOrient[4 * o]);
            CHECK(memcmp(&L, ob + 16 * i, 16) == 0, "orientation-tracked board i=%d", i);
        }
        delete[] boards; delete[] ob;
    }
    printf("board_logic_test: %s (%d failures)\n", fails ? "FAIL" : "OK", fails);
    return fails ? 1 : 0;
}
