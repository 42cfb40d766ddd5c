// r48_env.hip -- gfx950 kernels + C-ABI (include/rein48.h) of the vectorized 2048 env.
//
// Hot path: Game.step (nevertiree/Rein48 game/GameClient.py:40-51) over millions of
// int8[16] boards in lockstep. One board per lane: a 16-B global_load_dwordx4 per lane
// (1 KiB contiguous per wave), the step on four VGPRs (r48_board.h), a 16-B store back.
// Spawn draws come from a per-lane Philox4x32-10 keyed by (seed, global board id) with
// the step counter -- no RNG state lives in HBM. HBM traffic per board-step (random policy):
// 16 B board in + 16 B board out + 1 B action out + 1 B done out = 34 B.
#include <hip/hip_runtime.h>

#include <atomic>
#include <map>
#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/rein48.h"
#include "r48_board.h"

using r48::Board;

namespace {

constexpr int kBlock = 256;
// r48_env_step_n splits an env of >= kChainMin boards into kMaxChains contiguous shards, each
// replaying its own graph on its own stream: the two dependent-launch chains overlap one
// shard's load latency / store drain with the other's compute (1M boards: 10.3 -> 7.2 us).
#ifndef R48_MAX_CHAINS
#define R48_MAX_CHAINS 2
#endif
constexpr int kMaxChains = R48_MAX_CHAINS;
constexpr int64_t kChainMin = (int64_t)1 << 18;
// 2^24 boards = 256 MiB, the Infinity Cache: above it both patterns stream from HBM and
// ping-pong wins (2^26: 384 vs 425 us per step, tools/pingpong_bw.hip); at 2^24 the in-place
// array still fits the cache and in-place wins (85 vs 101 us)
constexpr int64_t kPingPongMin = ((int64_t)1 << 24) + 1;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#ifndef R48_NT_BOARDS
#define R48_NT_BOARDS 0   // experiments: 1 = nontemporal board loads, 2 = stores, 3 = both
#endif

__device__ __forceinline__ Board load_board(const int8_t *boards, int64_t i)
{
    const u32x4 *p = reinterpret_cast<const u32x4 *>(boards + 16 * i);
    const u32x4 v = (R48_NT_BOARDS & 1) ? __builtin_nontemporal_load(p) : *p;
    return Board{v.x, v.y, v.z, v.w};
}

__device__ __forceinline__ void store_board(int8_t *boards, int64_t i, const Board &b)
{
    u32x4 *p = reinterpret_cast<u32x4 *>(boards + 16 * i);
    const u32x4 v = {b.w0, b.w1, b.w2, b.w3};
    if (R48_NT_BOARDS & 2)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

__device__ __forceinline__ void philox_words(uint32_t w[4], uint64_t gid, uint32_t ctr, uint32_t tag,
                                             uint32_t k0, uint32_t k1)
{
    w[0] = (uint32_t)gid;
    w[1] = (uint32_t)(gid >> 32);
    w[2] = ctr;
    w[3] = tag;
    r48::philox4x32_10(w, k0, k1);
}

// one wave-level atomic per wave that saw a bad action byte
__device__ __forceinline__ void count_bad(bool bad, unsigned long long *err)
{
    const unsigned long long m = __ballot(bad);
    if (m && (threadIdx.x & 63) == __builtin_ctzll(m))
        atomicAdd(err, (unsigned long long)__builtin_popcountll(m));
}

// ---------------------------------------------------------------- Philox-mode step
// Draw contract (oracle/r48_oracle.c orc_step_philox): boards 2q and 2q+1
// (global ids) share one Philox4x32-10(key = seed, counter = {q lo, q hi, step, kStepTag});
// board 2q takes (x, y) = (w0, w1), board 2q+1 takes (w2, w3). Per board: action = x >> 30
// (random policy), spawn tile 4 iff (x & 0x3FFFFFFF) < kFourThresh30, blank rank =
// mulhi(y, n_blank); auto-reset cell = y >> 28, 4 iff (y & 0x0FFFFFFF) < kFourThresh28. A board
// is only done when its spawn had at most one blank (mulhi(y, n) = 0 for n <= 1) or no spawn,
// so y carried no information into that step and its bits are free for the reset.
struct Draw {
    uint32_t x, y;
};

__device__ __forceinline__ void pair_draws(uint64_t q, uint32_t step, uint32_t k0, uint32_t k1, Draw &even,
                                           Draw &odd)
{
    uint32_t w[4];
    philox_words(w, q, step, r48::kStepTag, k0, k1);
    even = Draw{w[0], w[1]};
    odd = Draw{w[2], w[3]};
}

__device__ __forceinline__ Draw board_draw(uint64_t gid, uint32_t step, uint32_t k0, uint32_t k1)
{
    Draw e, o;
    pair_draws(gid >> 1, step, k0, k1, e, o);
    return (gid & 1u) ? o : e;
}

struct LaneOut {
    Board b;
    uint32_t a, done, changed, reward, score;
};

template <bool RANDOM, bool AUTO_RESET, bool REWARD, bool RESET_BRANCH = true>
__device__ __forceinline__ LaneOut step_lane(Board b, int64_t i, Draw d, const int8_t *actions, bool want_score,
                                             unsigned long long *err)
{
    LaneOut r;
    if (RANDOM) {
        r.a = d.x >> 30;  // uniform over {UP, DOWN, LEFT, RIGHT} (control/rand.py:9-11)
    } else {
        r.a = (uint32_t)(uint8_t)actions[i];
        count_bad(r.a > 3u, err);
    }
    const r48::StepOut o =
        r48::step_board<REWARD, false, RANDOM>(b, r.a, d.y, (d.x & 0x3FFFFFFFu) < r48::kFourThresh30);
    r.score = want_score ? r48::tile_sum(b) : 0u;
    // auto-reset: ~1 board-step in 140 is done, so most waves skip it (wave-uniform branch).
    // Inside a multi-board tile (RESET_BRANCH = false) the branch would split the straight-line
    // load/compute pipeline, so there it is a select.
    if (AUTO_RESET && (RESET_BRANCH ? __ballot(o.done) != 0 : true)) {
        Board z;
        r48::reset_board(z, d.y >> 28, (d.y & 0x0FFFFFFFu) < r48::kFourThresh28);
        b = Board{r48::sel(o.done, z.w0, b.w0), r48::sel(o.done, z.w1, b.w1), r48::sel(o.done, z.w2, b.w2),
                  r48::sel(o.done, z.w3, b.w3)};
    }
    r.b = b;
    r.done = o.done;
    r.changed = o.changed;
    r.reward = o.reward;
    return r;
}

template <bool RANDOM, bool REWARD>
__device__ __forceinline__ void emit(const LaneOut &r, int64_t i, int8_t *boards, int8_t *actions, uint8_t *done,
                                     uint8_t *changed, int32_t *reward, int32_t *score)
{
    store_board(boards, i, r.b);
    if (RANDOM && actions)
        actions[i] = (int8_t)r.a;
    if (done)
        done[i] = (uint8_t)r.done;
    if (changed)
        changed[i] = (uint8_t)r.changed;
    if (reward)
        reward[i] = REWARD ? (int32_t)r.reward : 0;
    if (score)
        score[i] = (int32_t)r.score;
}

// both boards of a pair (i even): one 2-byte store per byte plane, so a wave's action / done /
// changed stores are each one contiguous 128-byte run
template <bool RANDOM, bool REWARD>
__device__ __forceinline__ void emit_pair(const LaneOut &e, const LaneOut &o, int64_t i, int8_t *boards,
                                          int8_t *actions, uint8_t *done, uint8_t *changed, int32_t *reward,
                                          int32_t *score)
{
    store_board(boards, i, e.b);
    store_board(boards, i + 1, o.b);
    if (RANDOM && actions)
        *reinterpret_cast<uint16_t *>(actions + i) = (uint16_t)((e.a & 0xffu) | (o.a << 8));
    if (done)
        *reinterpret_cast<uint16_t *>(done + i) = (uint16_t)(e.done | (o.done << 8));
    if (changed)
        *reinterpret_cast<uint16_t *>(changed + i) = (uint16_t)(e.changed | (o.changed << 8));
    if (reward)
        *reinterpret_cast<uint2 *>(reward + i) =
            make_uint2(REWARD ? e.reward : 0u, REWARD ? o.reward : 0u);
    if (score)
        *reinterpret_cast<uint2 *>(score + i) = make_uint2(e.score, o.score);
}

// Boards are read from `src` and written to `boards` (the same array for an in-place step; two
// arrays when r48_env_step_n ping-pongs a large env through its scratch copy, see launch_step).
// The Philox step counter is `step_arg` (eager launches) or `*d_ctr + step_arg` (graph
// replays: node k of a captured chunk carries step_arg = k and the launch function sets
// *d_ctr to the env's counter with a memset before each replay).
//
// NP board pairs per lane: a block owns a tile of 2 * NP * kBlock boards, lane t's pair j is
// boards tile + 2 * kBlock * j + 2t and +1 (each pair = 32 contiguous bytes, a wave's pair slot
// one contiguous 2 KiB), and ONE Philox call serves both boards of a pair. Full, pair-aligned
// tiles take a straight-line path -- all loads issued back to back, each pair computed as soon
// as its loads have landed, all stores at the end. The grid's partial last tile and envs whose
// global board ids start odd (pairs straddling the tile) take the guarded per-board path.
template <bool RANDOM, bool AUTO_RESET, bool REWARD, int NP>
__global__ __launch_bounds__(kBlock) void k_step(const int8_t *src, int8_t *boards, int64_t n, int64_t gid0,
                                                 uint32_t k0, uint32_t k1, const uint32_t *__restrict__ d_ctr,
                                                 uint32_t step_arg, int8_t *__restrict__ actions,
                                                 uint8_t *__restrict__ done, uint8_t *__restrict__ changed,
                                                 int32_t *__restrict__ reward, int32_t *__restrict__ score,
                                                 unsigned long long *err)
{
    constexpr int64_t kTile = (int64_t)kBlock * 2 * NP;
    const int64_t base = (int64_t)blockIdx.x * kTile + 2 * (int64_t)threadIdx.x;
    const uint32_t step = (d_ctr ? *d_ctr : 0u) + step_arg;
    const bool want_score = score != nullptr;
    // the pair path stores 2-byte / 8-byte pairs: caller planes must be aligned for that
    const bool aligned = ((((uintptr_t)actions | (uintptr_t)done | (uintptr_t)changed) & 1u) |
                          (((uintptr_t)reward | (uintptr_t)score) & 7u)) == 0;
    if ((int64_t)(blockIdx.x + 1) * kTile <= n && (gid0 & 1) == 0 && aligned) {
        Board b[2 * NP];
#pragma unroll
        for (int j = 0; j < NP; j++) {
            b[2 * j] = load_board(src, base + 2 * kBlock * j);
            b[2 * j + 1] = load_board(src, base + 2 * kBlock * j + 1);
        }
        LaneOut r[2 * NP];
#pragma unroll
        for (int j = 0; j < NP; j++) {
            const int64_t i = base + 2 * kBlock * j;
            Draw de, dd;
#if defined(R48_ABLATE_STEP_COPY)
            // timing floor only (tools/exp_step_variants.py): same launches and I/O, no compute
            r[2 * j] = LaneOut{Board{b[2 * j].w0 ^ step, b[2 * j].w1, b[2 * j].w2, b[2 * j].w3}, step & 3u, 0u, 0u, 0u, 0u};
            r[2 * j + 1] = LaneOut{Board{b[2 * j + 1].w0 ^ step, b[2 * j + 1].w1, b[2 * j + 1].w2, b[2 * j + 1].w3},
                                   step & 3u, 0u, 0u, 0u, 0u};
            continue;
#endif
            pair_draws((uint64_t)(gid0 + i) >> 1, step, k0, k1, de, dd);
            r[2 * j] = step_lane<RANDOM, AUTO_RESET, REWARD, NP == 1>(b[2 * j], i, de, actions, want_score, err);
            r[2 * j + 1] =
                step_lane<RANDOM, AUTO_RESET, REWARD, NP == 1>(b[2 * j + 1], i + 1, dd, actions, want_score, err);
        }
#pragma unroll
        for (int j = 0; j < NP; j++)
            emit_pair<RANDOM, REWARD>(r[2 * j], r[2 * j + 1], base + 2 * kBlock * j, boards, actions, done, changed,
                                      reward, score);
    } else {
        for (int j = 0; j < 2 * NP; j++) {
            const int64_t i = base + 2 * kBlock * (j >> 1) + (j & 1);
            if (i < n) {
                const Draw d = board_draw((uint64_t)(gid0 + i), step, k0, k1);
                const LaneOut r = step_lane<RANDOM, AUTO_RESET, REWARD, false>(load_board(src, i), i, d, actions,
                                                                               want_score, err);
                emit<RANDOM, REWARD>(r, i, boards, actions, done, changed, reward, score);
            }
        }
    }
}

// ---------------------------------------------------------------- injected-draw step
template <bool REWARD>
__global__ __launch_bounds__(kBlock) void k_step_draws(int8_t *__restrict__ boards, int64_t n,
                                                       const int8_t *__restrict__ actions,
                                                       const uint8_t *__restrict__ rank,
                                                       const uint8_t *__restrict__ four,
                                                       uint8_t *__restrict__ done, uint8_t *__restrict__ changed,
                                                       int32_t *__restrict__ reward, unsigned long long *err)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    Board b = load_board(boards, i);
    const uint32_t a = (uint32_t)(uint8_t)actions[i];
    count_bad(a > 3u, err);
    const r48::StepOut o = r48::step_board<REWARD, true>(b, a, rank[i], four[i] != 0);
    store_board(boards, i, b);
    if (done)
        done[i] = (uint8_t)o.done;
    if (changed)
        changed[i] = (uint8_t)o.changed;
    if (reward)
        reward[i] = REWARD ? (int32_t)o.reward : 0;
}

// ---------------------------------------------------------------- move / spawn halves
template <bool REWARD>
__global__ __launch_bounds__(kBlock) void k_move(int8_t *__restrict__ boards, int64_t n,
                                                 const int8_t *__restrict__ actions,
                                                 uint8_t *__restrict__ changed, uint8_t *__restrict__ n_blank,
                                                 int32_t *__restrict__ reward, unsigned long long *err)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    Board b = load_board(boards, i);
    const uint32_t a = (uint32_t)(uint8_t)actions[i];
    const bool valid = a < 4u;
    count_bad(!valid, err);
    Board L = r48::to_lines(b, a & 3u);
    const Board L0 = L;
    uint32_t rw = r48::move_lines<REWARD>(L);
    const uint32_t diff = (L.w0 ^ L0.w0) | (L.w1 ^ L0.w1) | (L.w2 ^ L0.w2) | (L.w3 ^ L0.w3);
    const bool c = valid && diff != 0u;
    const Board m = r48::from_lines(L, a & 3u);
    b = Board{r48::sel(c, m.w0, b.w0), r48::sel(c, m.w1, b.w1), r48::sel(c, m.w2, b.w2), r48::sel(c, m.w3, b.w3)};
    store_board(boards, i, b);
    if (changed)
        changed[i] = (uint8_t)c;
    if (n_blank)
        n_blank[i] = (uint8_t)r48::blanks(b).n;
    if (reward)
        reward[i] = (REWARD && c) ? (int32_t)rw : 0;
}

__global__ __launch_bounds__(kBlock) void k_spawn(int8_t *__restrict__ boards, int64_t n,
                                                  const uint8_t *__restrict__ mask, const uint8_t *__restrict__ rank,
                                                  const uint8_t *__restrict__ four, uint8_t *__restrict__ done)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    Board b = load_board(boards, i);
    const r48::Blanks bl = r48::blanks(b);
    const bool on = (mask == nullptr || mask[i] != 0) && bl.n != 0u;
    const uint32_t cell = r48::select_blank(bl, on ? rank[i] % bl.n : 0u);
    r48::place(b, cell, (on && four[i]) ? 2u : 1u, on);
    if (on)
        store_board(boards, i, b);
    if (done)
        done[i] = (uint8_t)r48::game_over(b, bl.n - (on ? 1u : 0u));
}

// ---------------------------------------------------------------- reset
__global__ __launch_bounds__(kBlock) void k_reset(int8_t *__restrict__ boards, int64_t n, int64_t gid0,
                                                  uint32_t k0, uint32_t k1, uint32_t ctr,
                                                  const uint8_t *__restrict__ mask)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n || (mask && !mask[i]))
        return;
    uint32_t w[4];
    philox_words(w, (uint64_t)(gid0 + i), ctr, r48::kResetTag, k0, k1);
    Board b;
    r48::reset_board(b, w[0] >> 28, w[1] < r48::kFourThresh);
    store_board(boards, i, b);
}

__global__ __launch_bounds__(kBlock) void k_reset_draws(int8_t *__restrict__ boards, int64_t n,
                                                        const uint8_t *__restrict__ mask,
                                                        const uint8_t *__restrict__ rank,
                                                        const uint8_t *__restrict__ four)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n || (mask && !mask[i]))
        return;
    Board b;
    r48::reset_board(b, rank[i] & 15u, four[i] != 0);
    store_board(boards, i, b);
}

// ---------------------------------------------------------------- synthetic start boards
// SURVEY.md 8(d) bench input: each cell empty w.p. 1/2, else e ~ U{1..max_exp}. Two Philox
// blocks per board (counter {gid lo, gid hi, j, kFillTag}, j = 0, 1) give 16 half-words; cell c
// reads half-word h = block c>>3, word (c>>1)&3, half c&1 (low first): empty iff !(h & 1), else
// e = 1 + (((h >> 1) * max_exp) >> 15).
__global__ __launch_bounds__(kBlock) void k_fill_random(int8_t *__restrict__ boards, int64_t n, int64_t gid0,
                                                        uint32_t k0, uint32_t k1, uint32_t max_exp)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    uint32_t w[8];
    philox_words(w, (uint64_t)(gid0 + i), 0u, r48::kFillTag, k0, k1);
    philox_words(w + 4, (uint64_t)(gid0 + i), 1u, r48::kFillTag, k0, k1);
    uint32_t row[4];
    R48_UNROLL
    for (int r = 0; r < 4; ++r) {
        uint32_t word = 0;
        R48_UNROLL
        for (int k = 0; k < 4; ++k) {
            const int c = 4 * r + k;
            const uint32_t h = (w[4 * (c >> 3) + ((c >> 1) & 3)] >> (16 * (c & 1))) & 0xFFFFu;
            const uint32_t e = (h & 1u) ? 1u + (((h >> 1) * max_exp) >> 15) : 0u;
            word |= e << (8 * k);
        }
        row[r] = word;
    }
    store_board(boards, i, Board{row[0], row[1], row[2], row[3]});
}

// ---------------------------------------------------------------- rollout (K steps in registers)
__global__ __launch_bounds__(kBlock) void k_rollout(int8_t *__restrict__ boards, int64_t n, int64_t gid0,
                                                    uint32_t k0, uint32_t k1, uint32_t step0, int32_t n_steps,
                                                    int8_t *__restrict__ actions, uint8_t *__restrict__ done)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    Board b = load_board(boards, i);
    const uint64_t gid = (uint64_t)(gid0 + i);
    for (int32_t t = 0; t < n_steps; t++) {
        const Draw d = board_draw(gid, step0 + (uint32_t)t, k0, k1);   // the k_step contract
        const uint32_t a = d.x >> 30;
        const r48::StepOut o = r48::step_board<false, false, true>(b, a, d.y, (d.x & 0x3FFFFFFFu) < r48::kFourThresh30);
        if (o.done)
            r48::reset_board(b, d.y >> 28, (d.y & 0x0FFFFFFFu) < r48::kFourThresh28);
        if (actions)
            actions[(int64_t)t * n + i] = (int8_t)a;
        if (done)
            done[(int64_t)t * n + i] = (uint8_t)o.done;
    }
    store_board(boards, i, b);
}

// ---------------------------------------------------------------- score
__global__ __launch_bounds__(kBlock) void k_score(const int8_t *__restrict__ boards, int64_t n,
                                                  int32_t *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    out[i] = (int32_t)r48::tile_sum(load_board(boards, i));
}

// ---------------------------------------------------------------- value-domain helpers
// Raw integer tiles (the reference's static methods accept any ints, GameClientTest.py
// uses 1s): the reference's two-pointer line walk (GameClient.py:141-179), equal tiles sum.
__device__ int64_t value_line(int32_t *c[4])
{
    int64_t rw = 0;
    int i = 0, j = 1;
    while (j < 4) {
        while (j < 4 && *c[j] == 0)
            j++;
        if (j == 4)
            break;
        if (*c[i] == 0) {
            *c[i] = *c[j];
            *c[j] = 0;
        } else if (*c[i] == *c[j]) {
            *c[i] += *c[j];
            *c[j] = 0;
            rw += *c[i];
            i++;
        } else {
            if (i + 1 != j) {
                *c[i + 1] = *c[j];
                *c[j] = 0;
            }
            i++;
        }
        j++;
    }
    return rw;
}

__global__ __launch_bounds__(kBlock) void k_values_move(int32_t *__restrict__ boards,
                                                        const int8_t *__restrict__ actions, int64_t n,
                                                        uint8_t *__restrict__ changed, int64_t *__restrict__ reward)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    int32_t v[16], o[16];
    for (int k = 0; k < 16; k++)
        o[k] = v[k] = boards[16 * i + k];
    const int a = actions[i];
    int64_t rw = 0;
    if (a >= 0 && a <= 3) {
        for (int line = 0; line < 4; line++) {
            int32_t *p[4];
            for (int k = 0; k < 4; k++) {
                const int r = a == 0 ? k : a == 1 ? 3 - k : line;
                const int cc = a == 0 || a == 1 ? line : a == 2 ? k : 3 - k;
                p[k] = &v[4 * r + cc];
            }
            rw += value_line(p);
        }
    }
    bool c = false;
    for (int k = 0; k < 16; k++) {
        c |= v[k] != o[k];
        boards[16 * i + k] = v[k];
    }
    if (changed)
        changed[i] = (uint8_t)c;
    if (reward)
        reward[i] = rw;
}

__global__ __launch_bounds__(kBlock) void k_values_check(const int32_t *__restrict__ boards, int64_t n,
                                                         int32_t rows, int32_t cols, uint8_t *__restrict__ filled,
                                                         uint8_t *__restrict__ over)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    const int32_t *m = boards + 16 * i;
    bool full = true, eq = false;
    for (int r = 0; r < rows; r++)
        for (int c = 0; c < cols; c++) {
            const int32_t v = m[4 * r + c];
            full &= v != 0;
            if (r + 1 < rows)
                eq |= v == m[4 * (r + 1) + c];
            if (c + 1 < cols)
                eq |= v == m[4 * r + c + 1];
        }
    if (filled)
        filled[i] = (uint8_t)full;
    if (over)
        over[i] = (uint8_t)(full && !eq);
}

}  // namespace

// =============================================================================== C-ABI
struct GraphKey {
    int32_t chain;
    int32_t n_steps;
    uint32_t flags;
    const void *p[6];
    bool operator<(const GraphKey &o) const
    {
        if (chain != o.chain)
            return chain < o.chain;
        if (n_steps != o.n_steps)
            return n_steps < o.n_steps;
        if (flags != o.flags)
            return flags < o.flags;
        for (int k = 0; k < 6; k++)
            if (p[k] != o.p[k])
                return p[k] < o.p[k];
        return false;
    }
};

struct r48_env {
    int device;
    int64_t n;
    uint64_t seed;
    int64_t gid0;
    uint32_t step_ctr;
    uint32_t reset_ctr;
    int8_t *boards;
    unsigned long long *err;  // device counter of bad action bytes
    uint32_t *d_ctr;          // step counter read by graph-replayed step kernels
    hipStream_t chain[kMaxChains];  // private streams: one per shard chain of r48_env_step_n
    hipEvent_t fork, join[kMaxChains];
    std::map<GraphKey, hipGraphExec_t> graphs;
    // r48_env_step_n on envs of >= pingpong_min boards alternates the boards between the bound
    // array and this env-owned copy (read one, write the other): past the Infinity Cache an
    // in-place read-modify-write sweep moves ~10 % fewer bytes per second than read-A/write-B
    int8_t *scratch = nullptr;
    int64_t pingpong_min = kPingPongMin;
};

namespace {

thread_local std::string g_last_error;

}  // namespace

namespace r48 {
void set_last_error(const std::string &msg) { g_last_error = msg; }
}  // namespace r48

namespace {

int fail(int code, const std::string &msg)
{
    g_last_error = msg;
    return code;
}

struct DeviceGuard {
    int prev = -1;
    bool ok = true;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess)
            prev = -1;
        if (prev != dev)
            ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard()
    {
        if (prev >= 0)
            (void)hipSetDevice(prev);
    }
};

int check_env(const r48_env *env, bool need_boards = true)
{
    if (!env)
        return fail(R48_EINVAL, "env is NULL");
    if (need_boards && !env->boards)
        return fail(R48_EINVAL, "no boards bound (call r48_env_bind_boards)");
    return R48_OK;
}

int launched(const char *what)
{
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(R48_EHIP, std::string(what) + ": " + hipGetErrorString(e));
    return R48_OK;
}

inline dim3 grid_for(int64_t n) { return dim3((unsigned)((n + kBlock - 1) / kBlock)); }

}  // namespace

extern "C" {

const char *r48_last_error(void) { return g_last_error.c_str(); }

const char *r48_version(void) { return "rein48 0.1.0 gfx950"; }

int r48_env_create(r48_env **out, int device, int64_t n_boards, uint64_t seed, int64_t board_offset)
{
    if (!out)
        return fail(R48_EINVAL, "out is NULL");
    *out = nullptr;
    if (n_boards <= 0 || n_boards > ((int64_t)1 << 40))
        return fail(R48_EINVAL, "n_boards out of range");
    if (board_offset < 0)
        return fail(R48_EINVAL, "board_offset < 0");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return fail(R48_EINVAL, "no such HIP device " + std::to_string(device));
    DeviceGuard g(device);
    if (!g.ok)
        return fail(R48_EHIP, "hipSetDevice failed");
    r48_env *env = new r48_env{device, n_boards, seed, board_offset, 0u, 0u, nullptr, nullptr, nullptr, {}, nullptr, {},
                               {}};
    if (hipMalloc(&env->err, sizeof(unsigned long long)) != hipSuccess) {
        delete env;
        return fail(R48_ENOMEM, "hipMalloc(error counter) failed");
    }
    if (hipMalloc(&env->d_ctr, sizeof(uint32_t)) != hipSuccess) {
        (void)hipFree(env->err);
        delete env;
        return fail(R48_ENOMEM, "hipMalloc(step counter) failed");
    }
    if (hipMemset(env->err, 0, sizeof(unsigned long long)) != hipSuccess) {
        (void)hipFree(env->err);
        delete env;
        return fail(R48_EHIP, "hipMemset failed");
    }
    *out = env;
    return R48_OK;
}

int r48_env_destroy(r48_env *env)
{
    if (!env)
        return R48_OK;
    DeviceGuard g(env->device);
    for (auto &kv : env->graphs)
        (void)hipGraphExecDestroy(kv.second);
    for (int c = 0; c < kMaxChains; c++) {
        if (env->chain[c])
            (void)hipStreamDestroy(env->chain[c]);
        if (env->join[c])
            (void)hipEventDestroy(env->join[c]);
    }
    if (env->fork)
        (void)hipEventDestroy(env->fork);
    (void)hipFree(env->d_ctr);
    (void)hipFree(env->err);
    if (env->scratch)
        (void)hipFree(env->scratch);
    delete env;
    return R48_OK;
}

int r48_env_bind_boards(r48_env *env, int8_t *boards)
{
    if (int s = check_env(env, false))
        return s;
    if (!boards || (reinterpret_cast<uintptr_t>(boards) & 15u))
        return fail(R48_EINVAL, "boards must be a non-NULL 16-byte aligned device pointer");
    if (env->boards != boards) {
        for (auto &kv : env->graphs)
            (void)hipGraphExecDestroy(kv.second);
        env->graphs.clear();
    }
    env->boards = boards;
    return R48_OK;
}

int8_t *r48_env_boards(const r48_env *env) { return env ? env->boards : nullptr; }

int r48_env_set_pingpong_min(r48_env *env, int64_t min_boards)
{
    if (int s = check_env(env, false))
        return s;
    if (min_boards < 0)
        return fail(R48_EINVAL, "min_boards < 0");
    env->pingpong_min = min_boards == 0 ? INT64_MAX : min_boards;
    if (env->n < env->pingpong_min && env->scratch) {
        for (auto &kv : env->graphs)
            (void)hipGraphExecDestroy(kv.second);
        env->graphs.clear();
        (void)hipFree(env->scratch);
        env->scratch = nullptr;
    }
    return R48_OK;
}

int64_t r48_env_size(const r48_env *env) { return env ? env->n : 0; }

int r48_env_get_counters(const r48_env *env, uint32_t *step, uint32_t *reset)
{
    if (int s = check_env(env, false))
        return s;
    if (step)
        *step = env->step_ctr;
    if (reset)
        *reset = env->reset_ctr;
    return R48_OK;
}

int r48_env_set_counters(r48_env *env, uint32_t step, uint32_t reset)
{
    if (int s = check_env(env, false))
        return s;
    env->step_ctr = step;
    env->reset_ctr = reset;
    return R48_OK;
}

int r48_env_reset(r48_env *env, const uint8_t *mask, void *stream)
{
    if (int s = check_env(env))
        return s;
    DeviceGuard g(env->device);
    hipLaunchKernelGGL(k_reset, grid_for(env->n), dim3(kBlock), 0, (hipStream_t)stream, env->boards, env->n,
                       env->gid0, (uint32_t)env->seed, (uint32_t)(env->seed >> 32), env->reset_ctr, mask);
    env->reset_ctr++;
    return launched("k_reset");
}

int r48_env_fill_random(r48_env *env, uint32_t max_exp, void *stream)
{
    if (int s = check_env(env))
        return s;
    if (max_exp < 1 || max_exp > 17)
        return fail(R48_EINVAL, "max_exp must be in 1..17");
    DeviceGuard g(env->device);
    hipLaunchKernelGGL(k_fill_random, grid_for(env->n), dim3(kBlock), 0, (hipStream_t)stream, env->boards,
                       env->n, env->gid0, (uint32_t)env->seed, (uint32_t)(env->seed >> 32), max_exp);
    return launched("k_fill_random");
}

int r48_env_reset_with_draws(r48_env *env, const uint8_t *mask, const uint8_t *rank, const uint8_t *four,
                             void *stream)
{
    if (int s = check_env(env))
        return s;
    if (!rank || !four)
        return fail(R48_EINVAL, "rank and four are required");
    DeviceGuard g(env->device);
    hipLaunchKernelGGL(k_reset_draws, grid_for(env->n), dim3(kBlock), 0, (hipStream_t)stream, env->boards,
                       env->n, mask, rank, four);
    return launched("k_reset_draws");
}

}  // extern "C"

namespace {

int validate_step(const r48_env *env, const int8_t *actions, uint32_t flags)
{
    if (int s = check_env(env))
        return s;
    if (flags & ~(R48_AUTO_RESET | R48_RANDOM_POLICY | R48_MERGE_REWARD))
        return fail(R48_EINVAL, "unknown flag bits");
    if (!(flags & R48_RANDOM_POLICY) && !actions)
        return fail(R48_EINVAL, "actions required unless R48_RANDOM_POLICY");
    return R48_OK;
}

// one k_step launch over boards [off, off+cnt) of the env; step counter =
// (d_ctr ? *d_ctr : 0) + step_arg. A lane takes one board pair (one Philox call per two boards)
// at every size: two pairs per lane measured slower even on the HBM-bound 2^26-board sweep
// (437 vs 428-432 us per step), so only NP = 1 is instantiated.
void launch_step(r48_env *env, int64_t off, int64_t cnt, const uint32_t *d_ctr, uint32_t step_arg,
                 int8_t *actions, uint32_t flags, uint8_t *done, uint8_t *changed, int32_t *reward, int32_t *score,
                 hipStream_t stream, const int8_t *src = nullptr, int8_t *dst = nullptr)
{
    if (!src)
        src = env->boards;
    if (!dst)
        dst = env->boards;
    const bool rnd = flags & R48_RANDOM_POLICY, ar = flags & R48_AUTO_RESET, rw = flags & R48_MERGE_REWARD;
    const uint32_t k0 = (uint32_t)env->seed, k1 = (uint32_t)(env->seed >> 32);
    auto at = [off](auto *p) { return p ? p + off : p; };
    auto go = [&](auto kern, int NP) {
        const int64_t tile = (int64_t)kBlock * 2 * NP;
        const dim3 grid((unsigned)((cnt + tile - 1) / tile));
        hipLaunchKernelGGL(kern, grid, dim3(kBlock), 0, stream, src + 16 * off, dst + 16 * off, cnt, env->gid0 + off, k0,
                           k1, d_ctr, step_arg, at(actions), at(done), at(changed), at(reward), at(score), env->err);
    };
#define R48_GO(RN, AR, RW) go(k_step<RN, AR, RW, 1>, 1)
    // 8 instantiations: policy source x auto-reset x reward mode
    if (rnd) {
        if (ar) rw ? R48_GO(true, true, true) : R48_GO(true, true, false);
        else rw ? R48_GO(true, false, true) : R48_GO(true, false, false);
    } else {
        if (ar) rw ? R48_GO(false, true, true) : R48_GO(false, true, false);
        else rw ? R48_GO(false, false, true) : R48_GO(false, false, false);
    }
#undef R48_GO
}

}  // namespace

extern "C" {

int r48_env_step(r48_env *env, int8_t *actions, uint32_t flags, uint8_t *done, uint8_t *changed, int32_t *reward,
                 int32_t *score, void *stream)
{
    if (int s = validate_step(env, actions, flags))
        return s;
    DeviceGuard g(env->device);
    launch_step(env, 0, env->n, nullptr, env->step_ctr, actions, flags, done, changed, reward, score,
                (hipStream_t)stream);
    env->step_ctr++;
    return launched("k_step");
}

}  // extern "C"

namespace {

// Find or capture+instantiate the per-chain graphs of n_steps step kernels.
int chain_graphs(r48_env *env, int32_t n_steps, int8_t *actions, uint32_t flags, uint8_t *done, uint8_t *changed,
                 int32_t *reward, int32_t *score, int chains, hipGraphExec_t *exec)
{
    if (env->n >= env->pingpong_min && !env->scratch) {
        // one allocation per env; without it (out of memory) the chains simply step in place
        if (hipMalloc(&env->scratch, (size_t)env->n * 16) != hipSuccess) {
            (void)hipGetLastError();
            env->scratch = nullptr;
        } else {
            for (auto &kv : env->graphs)   // graphs captured in place are stale now
                (void)hipGraphExecDestroy(kv.second);
            env->graphs.clear();
        }
    }
    if (!env->fork) {
        for (int c = 0; c < kMaxChains; c++)
            if (hipStreamCreateWithFlags(&env->chain[c], hipStreamNonBlocking) != hipSuccess ||
                hipEventCreateWithFlags(&env->join[c], hipEventDisableTiming) != hipSuccess)
                return fail(R48_EHIP, "creating chain streams/events failed");
        if (hipEventCreateWithFlags(&env->fork, hipEventDisableTiming) != hipSuccess)
            return fail(R48_EHIP, "hipEventCreate failed");
    }
    for (int c = 0; c < chains; c++) {
        // shard boundaries on even board ids: every board pair stays inside one shard
        const int64_t off = (env->n * c / chains) & ~(int64_t)1;
        const int64_t end = c + 1 == chains ? env->n : (env->n * (c + 1) / chains) & ~(int64_t)1;
        const int64_t cnt = end - off;
        const GraphKey key{c, n_steps, flags, {env->boards, actions, done, changed, reward, score}};
        auto it = env->graphs.find(key);
        if (it == env->graphs.end()) {
            // capture this shard's n_steps dependent step kernels once; replays read the
            // step counter from d_ctr
            if (hipStreamBeginCapture(env->chain[c], hipStreamCaptureModeThreadLocal) != hipSuccess)
                return fail(R48_EHIP, "hipStreamBeginCapture failed");
            // ping-pong: step k writes the bound array when n_steps - 1 - k is even, else the
            // scratch copy, and reads what step k - 1 wrote -- the last step always lands in the
            // bound array (an odd count starts with one in-place step)
            const int8_t *src = env->boards;
            for (int32_t k = 0; k < n_steps; k++) {
                int8_t *dst = (!env->scratch || ((n_steps - 1 - k) & 1) == 0) ? env->boards : env->scratch;
                launch_step(env, off, cnt, env->d_ctr, (uint32_t)k, actions, flags, done, changed, reward, score,
                            env->chain[c], src, dst);
                src = dst;
            }
            hipGraph_t graph = nullptr;
            const hipError_t ce = hipStreamEndCapture(env->chain[c], &graph);
            if (ce != hipSuccess || !graph)
                return fail(R48_EHIP, std::string("stream capture failed: ") + hipGetErrorString(ce));
            hipGraphExec_t x = nullptr;
            const hipError_t ie = hipGraphInstantiate(&x, graph, nullptr, nullptr, 0);
            (void)hipGraphDestroy(graph);
            if (ie != hipSuccess)
                return fail(R48_EHIP, std::string("hipGraphInstantiate failed: ") + hipGetErrorString(ie));
            // move the one-time upload of the executable graph off the first replay
            if (hipGraphUpload(x, env->chain[c]) != hipSuccess || hipStreamSynchronize(env->chain[c]) != hipSuccess)
                return fail(R48_EHIP, "hipGraphUpload failed");
            it = env->graphs.emplace(key, x).first;
        }
        exec[c] = it->second;
    }
    return R48_OK;
}

int check_step_n(const r48_env *env, const int8_t *actions, uint32_t flags, int32_t n_steps)
{
    if (int s = validate_step(env, actions, flags))
        return s;
    if (n_steps < 0 || n_steps > 4096)
        return fail(R48_EINVAL, "n_steps must be in 0..4096");
    return R48_OK;
}

}  // namespace

extern "C" {

int r48_env_prepare_step_n(r48_env *env, int32_t n_steps, int8_t *actions, uint32_t flags, uint8_t *done,
                           uint8_t *changed, int32_t *reward, int32_t *score)
{
    if (int s = check_step_n(env, actions, flags, n_steps))
        return s;
    if (n_steps == 0)
        return R48_OK;
    DeviceGuard g(env->device);
    hipGraphExec_t exec[kMaxChains] = {};
    return chain_graphs(env, n_steps, actions, flags, done, changed, reward, score,
                        env->n >= kChainMin ? kMaxChains : 1, exec);
}

int r48_env_step_n(r48_env *env, int32_t n_steps, int8_t *actions, uint32_t flags, uint8_t *done, uint8_t *changed,
                   int32_t *reward, int32_t *score, void *stream)
{
    if (int s = check_step_n(env, actions, flags, n_steps))
        return s;
    if (n_steps == 0)
        return R48_OK;
    DeviceGuard g(env->device);
    const hipStream_t user = (hipStream_t)stream;
    const int chains = env->n >= kChainMin ? kMaxChains : 1;
    hipGraphExec_t exec[kMaxChains] = {};
    if (int s = chain_graphs(env, n_steps, actions, flags, done, changed, reward, score, chains, exec))
        return s;
    // caller's stream: counter memset -> [fork] -> shard 0's graph; shard 1's graph replays on
    // the env's own stream between one fork and one join (a cross-stream wait costs tens of
    // microseconds, so there is exactly one of each per call)
    if (hipMemsetD32Async((hipDeviceptr_t)env->d_ctr, (int)env->step_ctr, 1, user) != hipSuccess)
        return fail(R48_EHIP, "hipMemsetD32Async(step counter) failed");
    if (chains > 1 && hipEventRecord(env->fork, user) != hipSuccess)
        return fail(R48_EHIP, "recording the fork event failed");
    for (int c = 1; c < chains; c++)
        if (hipStreamWaitEvent(env->chain[c], env->fork, 0) != hipSuccess)
            return fail(R48_EHIP, "forking a shard chain failed");
    for (int c = 0; c < chains; c++) {
        const hipError_t le = hipGraphLaunch(exec[c], c == 0 ? user : env->chain[c]);
        if (le != hipSuccess)
            return fail(R48_EHIP, std::string("hipGraphLaunch failed: ") + hipGetErrorString(le));
    }
    for (int c = 1; c < chains; c++)
        if (hipEventRecord(env->join[c], env->chain[c]) != hipSuccess ||
            hipStreamWaitEvent(user, env->join[c], 0) != hipSuccess)
            return fail(R48_EHIP, "joining a shard chain failed");
    env->step_ctr += (uint32_t)n_steps;
    return R48_OK;
}

int r48_env_step_with_draws(r48_env *env, const int8_t *actions, const uint8_t *rank, const uint8_t *four,
                            uint32_t flags, uint8_t *done, uint8_t *changed, int32_t *reward, void *stream)
{
    if (int s = check_env(env))
        return s;
    if (!actions || !rank || !four)
        return fail(R48_EINVAL, "actions, rank and four are required");
    if (flags & ~R48_MERGE_REWARD)
        return fail(R48_EINVAL, "only R48_MERGE_REWARD is valid with injected draws");
    DeviceGuard g(env->device);
    if (flags & R48_MERGE_REWARD)
        hipLaunchKernelGGL(k_step_draws<true>, grid_for(env->n), dim3(kBlock), 0, (hipStream_t)stream,
                           env->boards, env->n, actions, rank, four, done, changed, reward, env->err);
    else
        hipLaunchKernelGGL(k_step_draws<false>, grid_for(env->n), dim3(kBlock), 0, (hipStream_t)stream,
                           env->boards, env->n, actions, rank, four, done, changed, reward, env->err);
    return launched("k_step_draws");
}

int r48_env_move(r48_env *env, const int8_t *actions, uint32_t flags, uint8_t *changed, uint8_t *n_blank,
                 int32_t *reward, void *stream)
{
    if (int s = check_env(env))
        return s;
    if (!actions)
        return fail(R48_EINVAL, "actions required");
    if (flags & ~R48_MERGE_REWARD)
        return fail(R48_EINVAL, "only R48_MERGE_REWARD is valid for r48_env_move");
    DeviceGuard g(env->device);
    if (flags & R48_MERGE_REWARD)
        hipLaunchKernelGGL(k_move<true>, grid_for(env->n), dim3(kBlock), 0, (hipStream_t)stream, env->boards,
                           env->n, actions, changed, n_blank, reward, env->err);
    else
        hipLaunchKernelGGL(k_move<false>, grid_for(env->n), dim3(kBlock), 0, (hipStream_t)stream, env->boards,
                           env->n, actions, changed, n_blank, reward, env->err);
    return launched("k_move");
}

int r48_env_spawn(r48_env *env, const uint8_t *mask, const uint8_t *rank, const uint8_t *four, uint8_t *done,
                  void *stream)
{
    if (int s = check_env(env))
        return s;
    if (!rank || !four)
        return fail(R48_EINVAL, "rank and four are required");
    DeviceGuard g(env->device);
    hipLaunchKernelGGL(k_spawn, grid_for(env->n), dim3(kBlock), 0, (hipStream_t)stream, env->boards, env->n,
                       mask, rank, four, done);
    return launched("k_spawn");
}

int r48_env_rollout(r48_env *env, int32_t n_steps, int8_t *actions, uint8_t *done, void *stream)
{
    if (int s = check_env(env))
        return s;
    if (n_steps < 0)
        return fail(R48_EINVAL, "n_steps < 0");
    if (n_steps == 0)
        return R48_OK;
    DeviceGuard g(env->device);
    hipLaunchKernelGGL(k_rollout, grid_for(env->n), dim3(kBlock), 0, (hipStream_t)stream, env->boards, env->n,
                       env->gid0, (uint32_t)env->seed, (uint32_t)(env->seed >> 32), env->step_ctr, n_steps,
                       actions, done);
    env->step_ctr += (uint32_t)n_steps;
    return launched("k_rollout");
}

int r48_env_score(r48_env *env, int32_t *out, void *stream)
{
    if (int s = check_env(env))
        return s;
    if (!out)
        return fail(R48_EINVAL, "out is NULL");
    DeviceGuard g(env->device);
    hipLaunchKernelGGL(k_score, grid_for(env->n), dim3(kBlock), 0, (hipStream_t)stream, env->boards, env->n, out);
    return launched("k_score");
}

int r48_env_error_count(r48_env *env, int64_t *out, void *stream)
{
    if (int s = check_env(env, false))
        return s;
    if (!out)
        return fail(R48_EINVAL, "out is NULL");
    DeviceGuard g(env->device);
    unsigned long long v = 0;
    if (hipMemcpyAsync(&v, env->err, sizeof v, hipMemcpyDeviceToHost, (hipStream_t)stream) != hipSuccess ||
        hipStreamSynchronize((hipStream_t)stream) != hipSuccess)
        return fail(R48_EHIP, "reading the error counter failed");
    *out = (int64_t)v;
    return R48_OK;
}

int r48_env_clear_errors(r48_env *env, void *stream)
{
    if (int s = check_env(env, false))
        return s;
    DeviceGuard g(env->device);
    if (hipMemsetAsync(env->err, 0, sizeof(unsigned long long), (hipStream_t)stream) != hipSuccess)
        return fail(R48_EHIP, "hipMemsetAsync failed");
    return R48_OK;
}

int r48_values_move(int32_t *boards, const int8_t *actions, int64_t n, uint8_t *changed, int64_t *reward,
                    void *stream)
{
    if (!boards || !actions || n < 0)
        return fail(R48_EINVAL, "boards/actions NULL or n < 0");
    if (n == 0)
        return R48_OK;
    hipLaunchKernelGGL(k_values_move, grid_for(n), dim3(kBlock), 0, (hipStream_t)stream, boards, actions, n,
                       changed, reward);
    return launched("k_values_move");
}

int r48_values_check(const int32_t *boards, int64_t n, int32_t rows, int32_t cols, uint8_t *filled, uint8_t *over,
                     void *stream)
{
    if (!boards || n < 0 || rows < 1 || rows > 4 || cols < 1 || cols > 4)
        return fail(R48_EINVAL, "boards NULL, n < 0 or rows/cols outside 1..4");
    if (n == 0)
        return R48_OK;
    hipLaunchKernelGGL(k_values_check, grid_for(n), dim3(kBlock), 0, (hipStream_t)stream, boards, n, rows, cols,
                       filled, over);
    return launched("k_values_check");
}

}  // extern "C"
