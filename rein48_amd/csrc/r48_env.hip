// r48_env.hip -- gfx950 kernels + C-ABI (include/rein48.h) of the vectorized 2048 env.
//
// Hot path: Game.step (nevertiree/Rein48 game/GameClient.py:40-51) over millions of
// int8[16] boards in lockstep. One board per lane: a 16-B global_load_dwordx4 per lane
// (1 KiB contiguous per wave), the step on four VGPRs (r48_board.h), a 16-B store back.
// Spawn draws come from a per-lane Philox4x32-7 keyed by (seed, global board id) with
// the step counter -- no RNG state lives in HBM. HBM traffic per board-step (random policy):
// 16 B board in + 16 B board out + 1 B action out + 1 B done out = 34 B.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <utility>

#include "../../include/rein48.h"
#include "r48_board.h"
#include "r48_host.h"

using r48::Board;

namespace {

constexpr int kBlock = 256;
#ifndef R48_STEPN_NP
#define R48_STEPN_NP 1
#endif
constexpr int kStepNP = R48_STEPN_NP;   // board pairs per lane in k_step_n (A/B builds: -DR48_STEPN_NP=2)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ Board load_board(const int8_t *boards, int64_t i)
{
    const u32x4 *p = reinterpret_cast<const u32x4 *>(boards + 16 * i);
    const u32x4 v = *p;
    return Board{v.x, v.y, v.z, v.w};
}

__device__ __forceinline__ void store_board(int8_t *boards, int64_t i, const Board &b)
{
    u32x4 *p = reinterpret_cast<u32x4 *>(boards + 16 * i);
    *p = u32x4{b.w0, b.w1, b.w2, b.w3};
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
__device__ __forceinline__ void count_bad(bool bad, unsigned long long *err, unsigned times = 1)
{
    const unsigned long long m = __ballot(bad);
    if (m && (threadIdx.x & 63) == __builtin_ctzll(m))
        atomicAdd(err, (unsigned long long)__builtin_popcountll(m) * times);
}

// ---------------------------------------------------------------- Philox-mode step
// Draw contract (oracle/r48_oracle.c orc_step_philox): boards 2q and 2q+1
// (global ids) share one Philox4x32-7(key = seed, counter = {q lo, q hi, step, kStepTag});
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
    uint32_t w[4] = {(uint32_t)q, (uint32_t)(q >> 32), step, r48::kStepTag};
    r48::philox4x32_r<r48::kStepRounds>(w, k0, k1);
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

// One Philox-mode step of one board held in registers. `a_given` is the caller's action byte
// (ignored under RANDOM); bad bytes (> 3) leave the board unchanged -- the caller counts them.
// want_score: tile sum of the stepped board before any auto-reset (main.py:48).
template <bool RANDOM, bool AUTO_RESET, bool REWARD, bool RESET_BRANCH = true>
__device__ __forceinline__ LaneOut step_lane(Board b, uint32_t a_given, Draw d, bool want_score)
{
    LaneOut r;
    r.a = RANDOM ? d.x >> 30 : a_given;  // uniform over {UP, DOWN, LEFT, RIGHT} (control/rand.py:9-11)
    const r48::StepOut o =
        r48::step_board<REWARD, false, RANDOM>(b, r.a, d.y, (d.x & 0x3FFFFFFFu) < r48::kFourThresh30);
    r.score = 0u;
    if (want_score) {
        // wave-uniform branch; the empty asm keeps the compiler from if-converting the ~40-VALU
        // tile sum into every step
        asm volatile("" ::: "memory");
        r.score = r48::tile_sum(b);
    }
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

// ---------------------------------------------------------------- orientation-tracked step
// k_step_n keeps each board in the line form of its last action (r48_board.h "Orientations"):
// `ob` = 64 x that action (0 = rows, after a load or a reset), so the selector record taking the
// board to the line form of action a sits at byte ob + 16a of the 256-byte LDS table. A step is
// then one reorient (8 v_perm) + step_lines -- no to_lines / from_lines round trip, no per-lane
// selects on the action -- and the boards go back to rows once, when the call ends.
__device__ __forceinline__ r48::Orient orient_at(const r48::Orient *tab, uint32_t off)
{
    // one ds_read_b128 (the table is 16-byte aligned, off a multiple of 16)
    const u32x4 v = *reinterpret_cast<const u32x4 *>(
        __builtin_assume_aligned(reinterpret_cast<const char *>(tab) + off, 16));
    return r48::Orient{v.x, v.y, v.z, v.w};
}

__device__ __forceinline__ void load_orient_table(r48::Orient *tab)
{
    if (threadIdx.x < 16)
        tab[threadIdx.x] = r48::kOrient[threadIdx.x];
    __syncthreads();
}

template <bool RANDOM, bool AUTO_RESET, bool REWARD>
__device__ __forceinline__ LaneOut step_lane_lines(Board &L, uint32_t &ob, const r48::Orient *tab, uint32_t a_given,
                                                   Draw d, bool want_score)
{
    LaneOut r;
    r.a = RANDOM ? d.x >> 30 : a_given;  // uniform over {UP, DOWN, LEFT, RIGHT} (control/rand.py:9-11)
    const uint32_t a16 = RANDOM ? (d.x >> 26) & 0x30u : (a_given & 3u) << 4;
    L = r48::reorient(L, orient_at(tab, ob + a16));
    ob = a16 << 2;
    const r48::StepOut o =
        r48::step_lines<REWARD, RANDOM>(L, r.a, d.y, (d.x & 0x3FFFFFFFu) < r48::kFourThresh30);
    r.score = 0u;
    if (want_score) {
        asm volatile("" ::: "memory");   // keep the tile sum out of the other steps (see step_lane)
        r.score = r48::tile_sum(L);      // order-free: any orientation
    }
    if (AUTO_RESET && __ballot(o.done) != 0) {
        Board z;
        r48::reset_board(z, d.y >> 28, (d.y & 0x0FFFFFFFu) < r48::kFourThresh28);   // rows
        L = Board{r48::sel(o.done, z.w0, L.w0), r48::sel(o.done, z.w1, L.w1), r48::sel(o.done, z.w2, L.w2),
                  r48::sel(o.done, z.w3, L.w3)};
        ob = o.done ? 0u : ob;
    }
    r.done = o.done;
    r.changed = o.changed;
    r.reward = o.reward;
    return r;
}

// k_step_n's random-policy step on a board ALREADY reoriented to the line form of this step's
// action (d.x >> 30). `s_next` holds the caller's read-ahead of the next step's selector record,
// taken from the line form of this action; boards this step resets are back in rows, so theirs is
// re-read from the rows entry (offset a16n).
template <bool AUTO_RESET, bool REWARD>
__device__ __forceinline__ LaneOut step_lane_pre(Board &L, r48::Orient &s_next, uint32_t a16n, const r48::Orient *tab,
                                                 Draw d, bool want_score)
{
    LaneOut r;
    r.a = d.x >> 30;
    const r48::StepOut o = r48::step_lines<REWARD, true>(L, r.a, d.y, (d.x & 0x3FFFFFFFu) < r48::kFourThresh30);
    r.score = 0u;
    if (want_score) {
        asm volatile("" ::: "memory");
        r.score = r48::tile_sum(L);
    }
    if (AUTO_RESET && __ballot(o.done) != 0) {
        Board z;
        r48::reset_board(z, d.y >> 28, (d.y & 0x0FFFFFFFu) < r48::kFourThresh28);   // rows
        L = Board{r48::sel(o.done, z.w0, L.w0), r48::sel(o.done, z.w1, L.w1), r48::sel(o.done, z.w2, L.w2),
                  r48::sel(o.done, z.w3, L.w3)};
        const r48::Orient z0 = orient_at(tab, a16n);
        s_next = r48::Orient{r48::sel(o.done, z0.x0, s_next.x0), r48::sel(o.done, z0.x1, s_next.x1),
                             r48::sel(o.done, z0.te, s_next.te), r48::sel(o.done, z0.to, s_next.to)};
    }
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

// the pair path stores 2-byte / 8-byte pairs: caller planes must be aligned for that
__device__ __forceinline__ bool planes_aligned(const void *actions, const void *done, const void *changed,
                                               const void *reward, const void *score)
{
    return ((((uintptr_t)actions | (uintptr_t)done | (uintptr_t)changed) & 1u) |
            (((uintptr_t)reward | (uintptr_t)score) & 7u)) == 0;
}

// ---------------------------------------------------------------- one step (r48_env_step)
// One launch = one step of every board, boards read from and written back to HBM: 34 B per
// board-step under the random policy, the HBM-roofline kernel.
// A lane takes one board PAIR: boards tile + 2t and + 1 of its block's tile (32 contiguous
// bytes; a wave's pairs are one contiguous 2 KiB) and ONE Philox call serves both boards. Full,
// pair-aligned tiles take a straight-line path; the grid's partial last tile and envs whose
// global board ids start odd (pairs straddling the tile) take the guarded per-board path.
template <bool RANDOM, bool AUTO_RESET, bool REWARD>
__global__ __launch_bounds__(kBlock) void k_step(int8_t *boards, int64_t n, int64_t gid0, uint32_t k0, uint32_t k1,
                                                 uint32_t step, int8_t *__restrict__ actions,
                                                 uint8_t *__restrict__ done, uint8_t *__restrict__ changed,
                                                 int32_t *__restrict__ reward, int32_t *__restrict__ score,
                                                 unsigned long long *err)
{
    constexpr int64_t kTile = (int64_t)kBlock * 2;
    const int64_t i = (int64_t)blockIdx.x * kTile + 2 * (int64_t)threadIdx.x;
    const bool want_score = score != nullptr;
    __shared__ __attribute__((aligned(16))) r48::Orient tab[16];
    load_orient_table(tab);
    if ((int64_t)(blockIdx.x + 1) * kTile <= n && (gid0 & 1) == 0 &&
        planes_aligned(actions, done, changed, reward, score)) {
        Board be = load_board(boards, i), bo = load_board(boards, i + 1);
        uint32_t ae = 0, ao = 0;
        if (!RANDOM) {
            const uint16_t a2 = *reinterpret_cast<const uint16_t *>(actions + i);
            ae = a2 & 0xffu;
            ao = a2 >> 8;
            count_bad(ae > 3u, err);
            count_bad(ao > 3u, err);
        }
        Draw de, dd;
        pair_draws((uint64_t)(gid0 + i) >> 1, step, k0, k1, de, dd);
        // rows -> line form of the action and back through the LDS selector table (k_step_n's
        // orientation machinery with o = rows on entry and exit)
        uint32_t obe = 0, obo = 0;
        LaneOut re = step_lane_lines<RANDOM, AUTO_RESET, REWARD>(be, obe, tab, ae, de, want_score);
        LaneOut ro = step_lane_lines<RANDOM, AUTO_RESET, REWARD>(bo, obo, tab, ao, dd, want_score);
        re.b = r48::reorient(be, orient_at(tab, obe));
        ro.b = r48::reorient(bo, orient_at(tab, obo));
        emit_pair<RANDOM, REWARD>(re, ro, i, boards, actions, done, changed, reward, score);
    } else {
        for (int j = 0; j < 2; j++) {
            if (i + j < n) {
                const uint32_t a = RANDOM ? 0u : (uint32_t)(uint8_t)actions[i + j];
                if (!RANDOM)
                    count_bad(a > 3u, err);
                const Draw d = board_draw((uint64_t)(gid0 + i + j), step, k0, k1);
                const LaneOut r =
                    step_lane<RANDOM, AUTO_RESET, REWARD, false>(load_board(boards, i + j), a, d, want_score);
                emit<RANDOM, REWARD>(r, i + j, boards, actions, done, changed, reward, score);
            }
        }
    }
}


// ---------------------------------------------------------------- K steps in one launch
// r48_env_step_n: n_steps consecutive steps of every board in ONE launch. Boards are independent,
// so a lane keeps its NP board pairs in VGPRs for all n_steps steps (no grid barrier, no board
// round trip through HBM between steps) and writes the boards and the last step's output planes
// once at the end -- exactly what n_steps k_step launches leave in memory (the per-step planes
// are overwritten by every step). Same draw contract as k_step, step counter step0 + t. Bound:
// VALU issue (~200 VALU per board-step); HBM traffic is 34 B per board per
// call, not per step.
// TRAJ (r48_env_rollout): also every step's action and done into row t of traj_actions /
// traj_done ([n_steps][n], each nullable) -- one 2-byte store per plane per pair and step.
template <bool RANDOM, bool AUTO_RESET, bool REWARD, int NP, bool TRAJ = false>
// The read-ahead below needs ~62 VGPRs; waves_per_eu(8) holds the allocator to the 64 that keep the
// 8 waves per SIMD the VALU issue bound needs. The merge-reward variants need more than 64 (they
// spilled 28-48 B per lane to scratch under the cap), so they keep the plain launch bounds.
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(REWARD ? 1 : 8 / NP, 8 / NP))) void k_step_n(int8_t *boards, int64_t n, int64_t gid0, uint32_t k0, uint32_t k1,
                                                   uint32_t step0, int32_t n_steps, int8_t *__restrict__ actions,
                                                   uint8_t *__restrict__ done, uint8_t *__restrict__ changed,
                                                   int32_t *__restrict__ reward, int32_t *__restrict__ score,
                                                   unsigned long long *err, int8_t *__restrict__ traj_actions = nullptr,
                                                   uint8_t *__restrict__ traj_done = nullptr)
{
    constexpr int64_t kTile = (int64_t)kBlock * 2 * NP;
    const int64_t base = (int64_t)blockIdx.x * kTile + 2 * (int64_t)threadIdx.x;
    const bool want_score = score != nullptr;
    const int32_t last = n_steps - 1;
    __shared__ __attribute__((aligned(16))) r48::Orient tab[16];
    load_orient_table(tab);
    // trajectory rows whose pair addresses are not all 2-byte aligned (odd n or odd row pointers)
    // take byte stores inside the fast path, instead of sending the whole grid down the guarded one
    const bool traj_bytes = TRAJ && ((n | (int64_t)((uintptr_t)traj_actions | (uintptr_t)traj_done)) & 1) != 0;
    if ((int64_t)(blockIdx.x + 1) * kTile <= n && (gid0 & 1) == 0 &&
        planes_aligned(actions, done, changed, reward, score)) {
        Board b[2 * NP];
        uint32_t a[2 * NP], ob[2 * NP];
        uint64_t q[NP];
#pragma unroll
        for (int j = 0; j < NP; j++) {
            const int64_t i = base + 2 * kBlock * j;
            b[2 * j] = load_board(boards, i);
            b[2 * j + 1] = load_board(boards, i + 1);
            q[j] = (uint64_t)(gid0 + i) >> 1;
            a[2 * j] = a[2 * j + 1] = 0u;
            ob[2 * j] = ob[2 * j + 1] = 0u;   // rows
            if (!RANDOM) {
                const uint16_t a2 = *reinterpret_cast<const uint16_t *>(actions + i);
                a[2 * j] = a2 & 0xffu;
                a[2 * j + 1] = a2 >> 8;
                // every step re-reads the same bad byte: n_steps errors per board, like k_step
                count_bad(a[2 * j] > 3u, err, (unsigned)n_steps);
                count_bad(a[2 * j + 1] > 3u, err, (unsigned)n_steps);
            }
        }
        LaneOut r[2 * NP];
        // Progress-ordered issue priority. The SIMD's VALU is the bound and its arbiter prefers
        // the oldest wave: left alone, the 8 waves of a SIMD finish one after another and the
        // last ones run with too few partners to fill the VALU. Dropping a wave's priority as it
        // passes 1/8, 3/8 and 3/4 of the call lets the laggards catch up at each boundary, so all
        // 8 stay to the end (boundaries measured on three boxes: profiles/r02/exp_stepn_priority*).
        // The call runs as four phases at priority 3, 2, 1, 0, the boundaries at {1, 3, 6}/8 of the
        // call ({1, 3, 5}/8 for calls of at most 64 steps, where the last phase needs the longer
        // run-in): an outer loop over the phases around the step loop, so the priority change is
        // one scalar branch per phase and no per-step counter compares. Boundary sweeps at 2^20
        // boards (profiles/r03/stepn_priority_sweep_r03.txt): K = 20 81.3 -> 80.2 us with the last
        // boundary at 5/8, K = 1000 best at 6/8 (3.47 vs 3.50 us per step).
        const int32_t q3 = n_steps <= 64 ? 5 : 6;
        const int32_t ends[4] = {n_steps >> 3, (n_steps * 3) >> 3, (n_steps * q3) >> 3, n_steps};
        // Read-ahead (random policy): the draws depend on (pair, step) only, so step t + 1's Philox
        // runs under step t's board chain -- two independent dependency chains per wave -- and
        // step t + 1's selector record (last action -> next action, both known from the draws)
        // is read from LDS while step t moves. Measured on the 2^20-board A/B
        // (profiles/r03/stepn_readahead_ab.txt, with the phase loop below): K = 20 82.0 -> 81.3 us,
        // K = 1000 3.597 -> 3.46 us per step; bit-identical boards.
        Draw de[NP], dd[NP];
#pragma unroll
        for (int j = 0; j < NP; j++)
            pair_draws(q[j], step0, k0, k1, de[j], dd[j]);
        r48::Orient se[NP], sd[NP];   // this step's selector records (from rows on entry)
#pragma unroll
        for (int j = 0; j < NP; j++) {
            se[j] = orient_at(tab, (de[j].x >> 26) & 0x30u);
            sd[j] = orient_at(tab, (dd[j].x >> 26) & 0x30u);
        }
        int32_t t = 0;
#pragma nounroll
        for (int ph = 0; ph < 4; ph++) {
            switch (ph) {   // s_setprio takes an immediate
            case 0: __builtin_amdgcn_s_setprio(3); break;
            case 1: __builtin_amdgcn_s_setprio(2); break;
            case 2: __builtin_amdgcn_s_setprio(1); break;
            default: __builtin_amdgcn_s_setprio(0); break;
            }
            for (const int32_t end = ends[ph]; t < end; t++) {
                const uint32_t step = step0 + (uint32_t)t;
                const bool sc = want_score && t == last;
#pragma unroll
                for (int j = 0; j < NP; j++) {
                    Draw ne, nd;
                    pair_draws(q[j], step + 1u, k0, k1, ne, nd);
                    if (RANDOM) {
                        const uint32_t ane = (ne.x >> 26) & 0x30u, and_ = (nd.x >> 26) & 0x30u;
                        // this step's reorient first, then the next step's selector reads into the
                        // same registers: their LDS latency runs under this step's move
                        r48::Orient xe = orient_at(tab, ((de[j].x >> 24) & 0xC0u) + ane);
                        r48::Orient xd = orient_at(tab, ((dd[j].x >> 24) & 0xC0u) + and_);
                        b[2 * j] = r48::reorient(b[2 * j], se[j]);
                        b[2 * j + 1] = r48::reorient(b[2 * j + 1], sd[j]);
                        r[2 * j] = step_lane_pre<AUTO_RESET, REWARD>(b[2 * j], xe, ane, tab, de[j], sc);
                        r[2 * j + 1] = step_lane_pre<AUTO_RESET, REWARD>(b[2 * j + 1], xd, and_, tab, dd[j], sc);
                        se[j] = xe;
                        sd[j] = xd;
                    } else {
                        r[2 * j] = step_lane_lines<RANDOM, AUTO_RESET, REWARD>(b[2 * j], ob[2 * j], tab, a[2 * j], de[j], sc);
                        r[2 * j + 1] = step_lane_lines<RANDOM, AUTO_RESET, REWARD>(b[2 * j + 1], ob[2 * j + 1], tab,
                                                                                   a[2 * j + 1], dd[j], sc);
                    }
                    de[j] = ne;
                    dd[j] = nd;
                    if (TRAJ) {
                        const int64_t at = (int64_t)t * n + base + 2 * kBlock * j;
                        if (traj_bytes) {   // wave-uniform
                            if (traj_actions) {
                                traj_actions[at] = (int8_t)r[2 * j].a;
                                traj_actions[at + 1] = (int8_t)r[2 * j + 1].a;
                            }
                            if (traj_done) {
                                traj_done[at] = (uint8_t)r[2 * j].done;
                                traj_done[at + 1] = (uint8_t)r[2 * j + 1].done;
                            }
                        } else {
                            if (traj_actions)
                                *reinterpret_cast<uint16_t *>(traj_actions + at) =
                                    (uint16_t)(r[2 * j].a | (r[2 * j + 1].a << 8));
                            if (traj_done)
                                *reinterpret_cast<uint16_t *>(traj_done + at) =
                                    (uint16_t)(r[2 * j].done | (r[2 * j + 1].done << 8));
                        }
                    }
                }
            }
        }
        if (RANDOM) {   // the line form of the last action, or rows after a reset in the last step
            // (without AUTO_RESET a done board is not reset: it stays in the line form of its action)
#pragma unroll
            for (int j = 0; j < 2 * NP; j++)
                ob[j] = (AUTO_RESET && r[j].done) ? 0u : r[j].a << 6;
        }
#pragma unroll
        for (int j = 0; j < NP; j++) {
            r[2 * j].b = r48::reorient(b[2 * j], orient_at(tab, ob[2 * j]));   // back to rows
            r[2 * j + 1].b = r48::reorient(b[2 * j + 1], orient_at(tab, ob[2 * j + 1]));
            emit_pair<RANDOM, REWARD>(r[2 * j], r[2 * j + 1], base + 2 * kBlock * j, boards, actions, done, changed,
                                      reward, score);
        }
    } else {
        for (int j = 0; j < 2 * NP; j++) {
            const int64_t i = base + 2 * kBlock * (j >> 1) + (j & 1);
            if (i < n) {
                const uint32_t a = RANDOM ? 0u : (uint32_t)(uint8_t)actions[i];
                if (!RANDOM)
                    count_bad(a > 3u, err, (unsigned)n_steps);
                Board b = load_board(boards, i);
                LaneOut r;
                for (int32_t t = 0; t < n_steps; t++) {
                    const Draw d = board_draw((uint64_t)(gid0 + i), step0 + (uint32_t)t, k0, k1);
                    r = step_lane<RANDOM, AUTO_RESET, REWARD, false>(b, a, d, want_score && t == last);
                    b = r.b;
                    if (TRAJ && traj_actions)
                        traj_actions[(int64_t)t * n + i] = (int8_t)r.a;
                    if (TRAJ && traj_done)
                        traj_done[(int64_t)t * n + i] = (uint8_t)r.done;
                }
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

// Any rows x cols (Game(n) for n > 4, GameClient.py:19-27): boards int32[n][rows][cols] of raw
// values, one thread per (board, line) -- the lines of a move are independent. The reference's
// two-pointer walk (GameClient.py:141-179) along the line's cells from the wall; `changed`
// (zeroed by the caller) gets 1 from any line that moved a tile.
__global__ __launch_bounds__(kBlock) void k_values_move_grid(int32_t *__restrict__ boards, int64_t n, int32_t rows,
                                                             int32_t cols, const int8_t *__restrict__ actions,
                                                             uint8_t *__restrict__ changed)
{
    const int32_t lines = rows > cols ? rows : cols;
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t i = t / lines;
    const int32_t line = (int32_t)(t % lines);
    if (i >= n)
        return;
    const int a = actions[i];
    if (a < 0 || a > 3)
        return;
    const bool vert = a < 2, rev = (a & 1) != 0;
    const int32_t len = vert ? rows : cols;
    if (line >= (vert ? cols : rows))
        return;
    int32_t *m = boards + i * (int64_t)rows * cols;
    // element offset of cell k of this line counted from the wall
    const int64_t step = vert ? (rev ? -(int64_t)cols : cols) : (rev ? -1 : 1);
    const int64_t first = vert ? (rev ? (int64_t)(rows - 1) * cols + line : line)
                               : (int64_t)line * cols + (rev ? cols - 1 : 0);
    int32_t *p = m + first;
    bool moved = false;
    int32_t ii = 0, j = 1;
    while (j < len) {
        while (j < len && p[j * step] == 0)
            j++;
        if (j == len)
            break;
        const int32_t vj = p[j * step];
        const int32_t vi = p[ii * step];
        if (vi == 0) {                 // switch: the tile slides into the empty cell
            p[ii * step] = vj;
            p[j * step] = 0;
            moved = true;
        } else if (vi == vj) {         // merge
            p[ii * step] = vi + vj;
            p[j * step] = 0;
            ii++;
            moved = true;
        } else {                       // move behind i (a no-op when it already is there)
            if (ii + 1 != j) {
                p[(ii + 1) * step] = vj;
                p[j * step] = 0;
                moved = true;
            }
            ii++;
        }
        j++;
    }
    if (moved && changed)
        changed[i] = 1;
}

// has_table_filled / has_game_over (GameClient.py:65-100) on any rows x cols, one thread per board
__global__ __launch_bounds__(kBlock) void k_values_check_grid(const int32_t *__restrict__ boards, int64_t n,
                                                              int32_t rows, int32_t cols,
                                                              uint8_t *__restrict__ filled, uint8_t *__restrict__ over)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    const int32_t *m = boards + i * (int64_t)rows * cols;
    bool full = true, eq = false;
    for (int32_t r = 0; r < rows; r++)
        for (int32_t c = 0; c < cols; c++) {
            const int32_t v = m[(int64_t)r * cols + c];
            full &= v != 0;
            if (r + 1 < rows)
                eq |= v == m[(int64_t)(r + 1) * cols + c];
            if (c + 1 < cols)
                eq |= v == m[(int64_t)r * cols + c + 1];
        }
    if (filled)
        filled[i] = (uint8_t)full;
    if (over)
        over[i] = (uint8_t)(full && !eq);
}

}  // namespace

// =============================================================================== C-ABI
struct r48_env {
    int device;
    int64_t n;
    uint64_t seed;
    int64_t gid0;
    uint32_t step_ctr;
    uint32_t reset_ctr;
    int8_t *boards;
    unsigned long long *err;  // device counter of bad action bytes
};

namespace {

thread_local std::string g_last_error;

}  // namespace

namespace r48 {
void set_last_error(const std::string &msg) { g_last_error = msg; }

int stream_device(hipStream_t stream)
{
    int dev = 0;
    if (stream != nullptr && hipStreamGetDevice(stream, &dev) == hipSuccess)
        return dev;
    return hipGetDevice(&dev) == hipSuccess ? dev : 0;
}

int device_cus(int device)
{
    static std::mutex mu;
    static std::map<int, int> cache;
    std::lock_guard<std::mutex> lock(mu);
    auto it = cache.find(device);
    if (it != cache.end())
        return it->second;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0)
        cus = 256;
    cache[device] = cus;
    return cus;
}

bool ensure_dynamic_lds(const void *kernel, int bytes, int device)
{
    static std::mutex mu;
    static std::set<std::pair<const void *, int>> done;
    std::lock_guard<std::mutex> lock(mu);
    if (done.count({kernel, device}))
        return true;
    int prev = -1;
    const bool switched = hipGetDevice(&prev) == hipSuccess && prev != device && hipSetDevice(device) == hipSuccess;
    const hipError_t e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (switched)
        (void)hipSetDevice(prev);
    if (e != hipSuccess) {   // not recorded: the next launch tries the opt-in again
        set_last_error("hipFuncSetAttribute(MaxDynamicSharedMemorySize = " + std::to_string(bytes) +
                       ", device " + std::to_string(device) + "): " + hipGetErrorString(e));
        return false;
    }
    done.insert({kernel, device});
    return true;
}
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
    r48_env *env = new r48_env{device, n_boards, seed, board_offset, 0u, 0u, nullptr, nullptr};
    if (hipMalloc(&env->err, sizeof(unsigned long long)) != hipSuccess) {
        delete env;
        return fail(R48_ENOMEM, "hipMalloc(error counter) failed");
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
    (void)hipFree(env->err);
    delete env;
    return R48_OK;
}

int r48_env_bind_boards(r48_env *env, int8_t *boards)
{
    if (int s = check_env(env, false))
        return s;
    if (!boards || (reinterpret_cast<uintptr_t>(boards) & 15u))
        return fail(R48_EINVAL, "boards must be a non-NULL 16-byte aligned device pointer");
    env->boards = boards;
    return R48_OK;
}

int8_t *r48_env_boards(const r48_env *env) { return env ? env->boards : nullptr; }

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

// one launch over all boards: n_steps == 1 -> k_step (boards through HBM), else k_step_n
// (boards in VGPRs for all n_steps). 8 instantiations each: policy source x auto-reset x reward.
void launch_steps(r48_env *env, int32_t n_steps, int8_t *actions, uint32_t flags, uint8_t *done, uint8_t *changed,
                  int32_t *reward, int32_t *score, hipStream_t stream)
{
    const bool rnd = flags & R48_RANDOM_POLICY, ar = flags & R48_AUTO_RESET, rw = flags & R48_MERGE_REWARD;
    const uint32_t k0 = (uint32_t)env->seed, k1 = (uint32_t)(env->seed >> 32);
    auto one = [&](auto kern) {
        const int64_t tile = (int64_t)kBlock * 2;
        hipLaunchKernelGGL(kern, dim3((unsigned)((env->n + tile - 1) / tile)), dim3(kBlock), 0, stream, env->boards,
                           env->n, env->gid0, k0, k1, env->step_ctr, actions, done, changed, reward, score,
                           env->err);
    };
    auto many = [&](auto kern) {
        const int64_t tile = (int64_t)kBlock * 2 * kStepNP;
        hipLaunchKernelGGL(kern, dim3((unsigned)((env->n + tile - 1) / tile)), dim3(kBlock), 0, stream, env->boards,
                           env->n, env->gid0, k0, k1, env->step_ctr, n_steps, actions, done, changed, reward, score,
                           env->err, (int8_t *)nullptr, (uint8_t *)nullptr);
    };
#define R48_GO(RN, AR, RW) \
    (n_steps == 1 ? one(k_step<RN, AR, RW>) : many(k_step_n<RN, AR, RW, kStepNP>))
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
    launch_steps(env, 1, actions, flags, done, changed, reward, score, (hipStream_t)stream);
    env->step_ctr++;
    return launched("k_step");
}

int r48_env_step_n(r48_env *env, int32_t n_steps, int8_t *actions, uint32_t flags, uint8_t *done, uint8_t *changed,
                   int32_t *reward, int32_t *score, void *stream)
{
    if (int s = validate_step(env, actions, flags))
        return s;
    if (n_steps < 0)
        return fail(R48_EINVAL, "n_steps < 0");
    if (n_steps == 0)
        return R48_OK;
    DeviceGuard g(env->device);
    launch_steps(env, n_steps, actions, flags, done, changed, reward, score, (hipStream_t)stream);
    env->step_ctr += (uint32_t)n_steps;
    return launched("k_step_n");
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
    // = r48_env_step_n(random policy, auto-reset) that also writes every step's action and done
    const int64_t tile = (int64_t)kBlock * 2 * kStepNP;
    hipLaunchKernelGGL((k_step_n<true, true, false, kStepNP, true>), dim3((unsigned)((env->n + tile - 1) / tile)),
                       dim3(kBlock), 0, (hipStream_t)stream, env->boards, env->n, env->gid0, (uint32_t)env->seed,
                       (uint32_t)(env->seed >> 32), env->step_ctr, n_steps, (int8_t *)nullptr, (uint8_t *)nullptr,
                       (uint8_t *)nullptr, (int32_t *)nullptr, (int32_t *)nullptr, env->err, actions, done);
    env->step_ctr += (uint32_t)n_steps;
    return launched("k_step_n (rollout)");
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

int r48_values_move_grid(int32_t *boards, int64_t n, int32_t rows, int32_t cols, const int8_t *actions,
                         uint8_t *changed, void *stream)
{
    if (!boards || !actions || n < 0 || rows < 1 || cols < 1 || rows > R48_GRID_MAX || cols > R48_GRID_MAX)
        return fail(R48_EINVAL, "boards/actions NULL, n < 0 or rows/cols outside 1..R48_GRID_MAX");
    if (n == 0)
        return R48_OK;
    if (changed && hipMemsetAsync(changed, 0, (size_t)n, (hipStream_t)stream) != hipSuccess)
        return fail(R48_EHIP, "hipMemsetAsync failed");
    const int64_t threads = n * (int64_t)(rows > cols ? rows : cols);
    hipLaunchKernelGGL(k_values_move_grid, grid_for(threads), dim3(kBlock), 0, (hipStream_t)stream, boards, n, rows,
                       cols, actions, changed);
    return launched("k_values_move_grid");
}

int r48_values_check_grid(const int32_t *boards, int64_t n, int32_t rows, int32_t cols, uint8_t *filled,
                          uint8_t *over, void *stream)
{
    if (!boards || n < 0 || rows < 1 || cols < 1 || rows > R48_GRID_MAX || cols > R48_GRID_MAX)
        return fail(R48_EINVAL, "boards NULL, n < 0 or rows/cols outside 1..R48_GRID_MAX");
    if (n == 0)
        return R48_OK;
    hipLaunchKernelGGL(k_values_check_grid, grid_for(n), dim3(kBlock), 0, (hipStream_t)stream, boards, n, rows,
                       cols, filled, over);
    return launched("k_values_check_grid");
}

}  // extern "C"
