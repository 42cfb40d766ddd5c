// r48_board.h -- per-lane 2048 board logic for the gfx950 env kernels (r48_env.hip).
//
// One board per lane, held in four 32-bit VGPRs: row word R[r] holds cells (r,0..3) in
// bytes 0..3 (cell value = exponent e, 0 = empty, tile = 2^e). Everything here is
// branch-free integer work on those registers: no MFMA (this is a byte shuffle, not a
// contraction), no LDS, no divergence by action.
//
// Move = the reference's update_matrix (nevertiree/Rein48 game/GameClient.py:129-254).
// Instead of walking one line at a time with two pointers, all four lines of the board
// are moved at once, SWAR-style: the board is first re-expressed as "line-parallel"
// words L[k] whose byte l is the k-th cell of line l counted from the side the tiles
// move toward. In that form a move is the same word-wide byte-select sequence for every
// direction:
//     UP    L[k] = R[k]          DOWN  L[k] = R[3-k]
//     LEFT  L[k] = T(R)[k]       RIGHT L[k] = T(R)[3-k]        (T = 4x4 byte transpose)
// then (1) compaction -- bytes shift toward L[0] over empty cells -- and (2) one merge
// pass over adjacent equal pairs (each tile merges at most once, pairs nearest L[0]
// first), which is exactly the reference's two-pointer result (checked exhaustively in
// tests against the 18^4-line table produced by the reference itself).
//
// The same functions compile for the host (R48_HD empty, v_perm emulated) so the CPU
// test harness tests/native/board_logic_test.cpp can check this logic against the oracle
// without a GPU; the product library only ever runs the device build.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define R48_HD __host__ __device__ __forceinline__
#define R48_UNROLL _Pragma("unroll")
#else
#define R48_HD static inline
#define R48_UNROLL
#endif

namespace r48 {

// v_perm_b32: byte k of the result = byte sel[k] of the 8-byte pool {hi:lo}
// (0-3 = lo bytes, 4-7 = hi bytes, 12 = 0x00).
R48_HD uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(hi, lo, sel);
#else
    const uint64_t pool = ((uint64_t)hi << 32) | lo;
    uint32_t out = 0;
    for (int k = 0; k < 4; k++) {
        const uint32_t s = (sel >> (8 * k)) & 0xffu;
        uint32_t b;
        if (s >= 13)
            b = 0xffu;
        else if (s == 12)
            b = 0u;
        else if (s >= 8)
            b = ((pool >> (16 * (s - 8) + 15)) & 1u) ? 0xffu : 0u;
        else
            b = (uint32_t)(pool >> (8 * s)) & 0xffu;
        out |= b << (8 * k);
    }
    return out;
#endif
}

R48_HD uint32_t popc(uint32_t x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)__builtin_popcount(x);
#else
    return (uint32_t)__builtin_popcount(x);
#endif
}

R48_HD uint32_t mulhi(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

// Byte-lane predicates, valid while every byte is <= 0x80 (cell exponents are 0..30):
// 0x80 in each byte that is nonzero / zero.
R48_HD uint32_t nz80(uint32_t x) { return (x + 0x7F7F7F7Fu) & 0x80808080u; }
R48_HD uint32_t z80(uint32_t x) { return ~(x + 0x7F7F7F7Fu) & 0x80808080u; }
// Bit 7 of each byte -> 0xFF/0x00 byte mask (other bits ignored): v_perm_b32's selectors
// 8..11 replicate the sign bit of pool bytes 1, 3, 5, 7; with pool {f<<8 : f} those are
// f's bytes 1, 3, 0, 2.  Two instructions (shift + perm).
R48_HD uint32_t ff(uint32_t f) { return perm(f << 8, f, 0x090B080Au); }
// 0xFF in each nonzero byte of x (bytes <= 0x80): add + shift + perm
R48_HD uint32_t nzff(uint32_t x) { return ff(x + 0x7F7F7F7Fu); }
// bytewise select: m ? x : y   (v_bfi_b32)
R48_HD uint32_t bsel(uint32_t m, uint32_t x, uint32_t y) { return (x & m) | (y & ~m); }

// Four row words as named scalars (no arrays: a selected array index would be lowered to
// a dynamically indexed private array, which hipcc promotes to LDS).
struct Board {
    uint32_t w0, w1, w2, w3;
};

R48_HD uint32_t sel(bool c, uint32_t x, uint32_t y) { return c ? x : y; }

// 4x4 byte transpose in 8 v_perm_b32: out.w<c> byte k = in.w<k> byte c. An involution.
R48_HD Board transpose(const Board &r)
{
    const uint32_t a0 = perm(r.w1, r.w0, 0x05010400u);  // r0.b0 r1.b0 r0.b1 r1.b1
    const uint32_t a1 = perm(r.w1, r.w0, 0x07030602u);  // r0.b2 r1.b2 r0.b3 r1.b3
    const uint32_t b0 = perm(r.w3, r.w2, 0x05010400u);
    const uint32_t b1 = perm(r.w3, r.w2, 0x07030602u);
    return Board{perm(b0, a0, 0x05040100u), perm(b0, a0, 0x07060302u), perm(b1, a1, 0x05040100u),
                 perm(b1, a1, 0x07060302u)};
}

// rows -> line-parallel words for action a (0 UP, 1 DOWN, 2 LEFT, 3 RIGHT)
R48_HD Board to_lines(const Board &r, uint32_t a)
{
    const bool vert = a < 2u, rev = (a & 1u) != 0;
    const Board t = transpose(r);
    const uint32_t s0 = sel(vert, r.w0, t.w0), s1 = sel(vert, r.w1, t.w1);
    const uint32_t s2 = sel(vert, r.w2, t.w2), s3 = sel(vert, r.w3, t.w3);
    return Board{sel(rev, s3, s0), sel(rev, s2, s1), sel(rev, s1, s2), sel(rev, s0, s3)};
}

// inverse of to_lines
R48_HD Board from_lines(const Board &l, uint32_t a)
{
    const bool vert = a < 2u, rev = (a & 1u) != 0;
    const Board s{sel(rev, l.w3, l.w0), sel(rev, l.w2, l.w1), sel(rev, l.w1, l.w2), sel(rev, l.w0, l.w3)};
    const Board t = transpose(s);
    return Board{sel(vert, s.w0, t.w0), sel(vert, s.w1, t.w1), sel(vert, s.w2, t.w2), sel(vert, s.w3, t.w3)};
}

// Slide + merge all four lines toward L[0]. Returns the merge reward (sum of merged tile
// values) when REWARD, else 0.
template <bool REWARD>
R48_HD uint32_t move_lines(Board &L)
{
    uint32_t l0 = L.w0, l1 = L.w1, l2 = L.w2, l3 = L.w3;
    // (1) compaction, from the far side in: where line cell i is empty, the cells behind it
    //     shift one place toward L[0] (GameClient.py:147-160: j skips empties, i takes j).
    uint32_t k = nzff(l2);
    l2 = bsel(k, l2, l3);
    l3 &= k;
    k = nzff(l1);
    l1 = bsel(k, l1, l2);
    l2 = bsel(k, l2, l3);
    l3 &= k;
    k = nzff(l0);
    l0 = bsel(k, l0, l1);
    l1 = bsel(k, l1, l2);
    l2 = bsel(k, l2, l3);
    l3 &= k;
    // (2) merge adjacent equal tiles once, nearest the wall first (GameClient.py:162-167):
    //     (0,1) always wins, (1,2) only if (0,1) did not, (2,3) unless (1,2) merged.
    //     Flags live in bit 7 of each byte: equal = bit 7 of (a^b)+0x7F clear, nonzero =
    //     bit 7 of b+0x7F set.
    const uint32_t e01 = ~((l0 ^ l1) + 0x7F7F7F7Fu) & (l1 + 0x7F7F7F7Fu);
    const uint32_t e12 = ~((l1 ^ l2) + 0x7F7F7F7Fu) & (l2 + 0x7F7F7F7Fu);
    const uint32_t e23 = ~((l2 ^ l3) + 0x7F7F7F7Fu) & (l3 + 0x7F7F7F7Fu);
    const uint32_t f01 = ff(e01);
    const uint32_t f12 = ff(e12 & ~e01);
    const uint32_t f23 = ff(e23 & (e01 | ~e12));
    uint32_t reward = 0;
    // apply the far pair first so the nearer pairs' shifts carry its result along
    l2 += f23 & 0x01010101u;
    if (REWARD) {
        for (int b = 0; b < 4; b++)
            reward += ((f23 >> (8 * b)) & 1u) << ((l2 >> (8 * b)) & 31u);
    }
    l3 &= ~f23;
    l1 += f12 & 0x01010101u;
    if (REWARD) {
        for (int b = 0; b < 4; b++)
            reward += ((f12 >> (8 * b)) & 1u) << ((l1 >> (8 * b)) & 31u);
    }
    l2 = bsel(f12, l3, l2);
    l3 &= ~f12;
    l0 += f01 & 0x01010101u;
    if (REWARD) {
        for (int b = 0; b < 4; b++)
            reward += ((f01 >> (8 * b)) & 1u) << ((l0 >> (8 * b)) & 31u);
    }
    l1 = bsel(f01, l2, l1);
    l2 = bsel(f01, l3, l2);
    l3 &= ~f01;
    L = Board{l0, l1, l2, l3};
    return reward;
}

// Blank cells in row-major order (GameClient.py:109-114), as per-row zero flags.
struct Blanks {
    uint32_t z0, z1, z2, z3;  // 0x80 in each empty byte of row r
    uint32_t p1, p2, p3, n;   // prefix counts of rows 0..2 and the total
};

R48_HD Blanks blanks(const Board &r)
{
    Blanks b;
    b.z0 = z80(r.w0);
    b.z1 = z80(r.w1);
    b.z2 = z80(r.w2);
    b.z3 = z80(r.w3);
    b.p1 = popc(b.z0);
    b.p2 = b.p1 + popc(b.z1);
    b.p3 = b.p2 + popc(b.z2);
    b.n = b.p3 + popc(b.z3);
    return b;
}

// Cell index (4*r + c) of the rank-th blank, rank < b.n (random_fill_grid's
// blank_grid_index_list[random_grid_index], GameClient.py:121-122).
R48_HD uint32_t select_blank(const Blanks &b, uint32_t rank)
{
    const bool s1 = rank >= b.p1, s2 = rank >= b.p2, s3 = rank >= b.p3;
    const uint32_t row = (uint32_t)s1 + (uint32_t)s2 + (uint32_t)s3;
    const uint32_t base = sel(s3, b.p3, sel(s2, b.p2, sel(s1, b.p1, 0u)));
    uint32_t z = sel(s3, b.z3, sel(s2, b.z2, sel(s1, b.z1, b.z0)));
    uint32_t j = rank - base;
    const uint32_t lo = popc(z & 0x8080u);
    const bool hi = j >= lo;
    j -= hi ? lo : 0u;
    z = hi ? (z >> 16) : z;
    const uint32_t col = (hi ? 2u : 0u) + ((j >= ((z >> 7) & 1u)) ? 1u : 0u);
    return 4u * row + col;
}

// select_blank + place in one: the row of the rank-th blank is where the prefix counts
// cross `rank`; the three comparisons are lane masks, so the row-hit masks are SGPR logic
// and each row word takes one v_cndmask + v_or (no row index, no per-row compares).
R48_HD void spawn_at_rank(Board &r, const Blanks &b, uint32_t rank, uint32_t e, bool on)
{
    const bool s1 = rank >= b.p1, s2 = rank >= b.p2, s3 = rank >= b.p3;
    const uint32_t base = sel(s3, b.p3, sel(s2, b.p2, sel(s1, b.p1, 0u)));
    uint32_t z = sel(s3, b.z3, sel(s2, b.z2, sel(s1, b.z1, b.z0)));
    uint32_t j = rank - base;
    const uint32_t lo = popc(z & 0x8080u);
    const bool hi = j >= lo;
    j -= hi ? lo : 0u;
    z = hi ? (z >> 16) : z;
    const uint32_t col = (hi ? 2u : 0u) + ((j >= ((z >> 7) & 1u)) ? 1u : 0u);
    const uint32_t v = (e & (0u - (uint32_t)on)) << (8u * col);   // arithmetic, not a select: no branch
    r.w0 |= sel(!s1, v, 0u);
    r.w1 |= sel(s1 && !s2, v, 0u);
    r.w2 |= sel(s2 && !s3, v, 0u);
    r.w3 |= sel(s3, v, 0u);
}

// Put exponent e (1 = tile 2, 2 = tile 4) into cell `cell` when `on` (GameClient.py:125).
R48_HD void place(Board &r, uint32_t cell, uint32_t e, bool on)
{
    const uint32_t v = on ? (e << (8u * (cell & 3u))) : 0u;
    const uint32_t row = cell >> 2;
    r.w0 |= sel(row == 0u, v, 0u);
    r.w1 |= sel(row == 1u, v, 0u);
    r.w2 |= sel(row == 2u, v, 0u);
    r.w3 |= sel(row == 3u, v, 0u);
}

// has_game_over (GameClient.py:65-100) on a board with `n_blank` empty cells:
// over iff full and no two orthogonal neighbours are equal.
R48_HD bool game_over(const Board &r, uint32_t n_blank)
{
    uint32_t eq = z80(r.w0 ^ (r.w0 >> 8)) | z80(r.w1 ^ (r.w1 >> 8)) | z80(r.w2 ^ (r.w2 >> 8)) |
                  z80(r.w3 ^ (r.w3 >> 8));  // (r,c) == (r,c+1)
    eq &= 0x00808080u;
    eq |= z80(r.w0 ^ r.w1) | z80(r.w1 ^ r.w2) | z80(r.w2 ^ r.w3);  // (r,c) == (r+1,c)
    return n_blank == 0u && eq == 0u;
}

R48_HD uint32_t row_sum(uint32_t w)
{
    uint32_t s = 0;
    for (int b = 0; b < 4; b++) {
        const uint32_t e = (w >> (8 * b)) & 0xffu;
        s += e ? (1u << (e & 31u)) : 0u;
    }
    return s;
}

R48_HD uint32_t tile_sum(const Board &r) { return row_sum(r.w0) + row_sum(r.w1) + row_sum(r.w2) + row_sum(r.w3); }

// a ^ b ^ k with k wave-uniform: ONE v_bitop3_b32 (the compiler emits two v_xor_b32 when one
// operand is an SGPR)
R48_HD uint32_t xor3_uniform(uint32_t a, uint32_t b, uint32_t k)
{
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(k));
    return r;
#else
    return a ^ b ^ k;
#endif
}

// ---- Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11) -----------------------------
// Round 0 stays in C so the compiler can move its wave-uniform counter words to the SALU;
// rounds 1-9 fold each round's two XORs into one v_bitop3_b32.
R48_HD void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1)
{
    R48_UNROLL
    for (int i = 0; i < 10; i++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        uint32_t n0, n2;
        if (i == 0) {
            n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
            n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        } else {
            n0 = xor3_uniform((uint32_t)(p1 >> 32), c[1], k0);
            n2 = xor3_uniform((uint32_t)(p0 >> 32), c[3], k1);
        }
        c[1] = (uint32_t)p1;
        c[3] = (uint32_t)p0;
        c[0] = n0;
        c[2] = n2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// Draw-word contract (DESIGN.md "Philox mode"; restated in oracle/r48_oracle.c)
static constexpr uint32_t kStepTag = 0x2048u;
static constexpr uint32_t kResetTag = 0x5E7u;
static constexpr uint32_t kFillTag = 0xF111u;   // synthetic start boards (r48_env_fill_random)
static constexpr uint32_t kFourThresh = 0x1999999Au;     // P(4) = 0.1   (GameClient.py:125)
static constexpr uint32_t kFourThresh30 = 0x06666666u;   // same on 30 bits (P = 0.1 - 4e-10)
static constexpr uint32_t kFourThresh28 = 0x0199999Au;   // same on 28 bits

// The env step's draw words of board `gid` at step `step` (the k_step contract of r48_env.hip,
// DESIGN.md section 7): boards 2q, 2q + 1 share Philox4x32-10(key, {q lo, q hi, step, kStepTag});
// the even board takes (x, y) = (w0, w1), the odd one (w2, w3).
R48_HD void step_draw(uint64_t gid, uint32_t step, uint32_t k0, uint32_t k1, uint32_t &x, uint32_t &y)
{
    const uint64_t q = gid >> 1;
    uint32_t w[4] = {(uint32_t)q, (uint32_t)(q >> 32), step, kStepTag};
    philox4x32_10(w, k0, k1);
    x = (gid & 1u) ? w[2] : w[0];
    y = (gid & 1u) ? w[3] : w[1];
}

struct StepOut {
    uint32_t changed, done, n_blank, reward, score;
};

// One env step on registers (Game.step, GameClient.py:40-51) given the action and the
// two spawn draws. `rank_word` is either a Philox word (rank = mulhi(word, n_blank)) or,
// when RANK_IS_INDEX, the injected rank itself (taken modulo n_blank). VALID_ACTION: the
// caller guarantees a < 4 (in-kernel random policy), so the moved board is taken as is -- an
// unchanged move maps back to the same board (from_lines inverts to_lines exactly).
template <bool REWARD, bool RANK_IS_INDEX, bool VALID_ACTION = false>
R48_HD StepOut step_board(Board &r, uint32_t a, uint32_t rank_word, bool four)
{
    StepOut o;
    const bool valid = VALID_ACTION || a < 4u;
    const uint32_t ac = a & 3u;
    Board L = to_lines(r, ac);
    const Board L0 = L;
    o.reward = move_lines<REWARD>(L);
    const uint32_t diff = (L.w0 ^ L0.w0) | (L.w1 ^ L0.w1) | (L.w2 ^ L0.w2) | (L.w3 ^ L0.w3);
    const bool changed = valid && diff != 0u;
    const Board moved = from_lines(L, ac);
    if (VALID_ACTION)
        r = moved;
    else
        r = Board{sel(changed, moved.w0, r.w0), sel(changed, moved.w1, r.w1), sel(changed, moved.w2, r.w2),
                  sel(changed, moved.w3, r.w3)};
    o.reward = changed ? o.reward : 0u;
    const Blanks bl = blanks(r);
    o.n_blank = bl.n;
    uint32_t rank;
    if (RANK_IS_INDEX)
        rank = bl.n ? rank_word % bl.n : 0u;
    else
        rank = mulhi(rank_word, bl.n);
    spawn_at_rank(r, bl, rank, four ? 2u : 1u, changed);
    o.changed = changed;
    o.done = game_over(r, bl.n - (changed ? 1u : 0u));
    return o;
}

// Game.reset (GameClient.py:33-38): empty board + one tile at `cell`.
R48_HD void reset_board(Board &r, uint32_t cell, bool four)
{
    r = Board{0u, 0u, 0u, 0u};
    place(r, cell & 15u, four ? 2u : 1u, true);
}

}  // namespace r48
