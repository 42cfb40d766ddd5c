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

// v_bitop3_b32: any bitwise function of three words in ONE full-rate instruction (truth table
// TT, bit index 4*a + 2*b + c). The compiler otherwise picks half-rate forms for some of them
// (v_bfi_b32 for selects, v_or3_b32; measured issue costs in profiles/r02/instr_rate.txt).
template <unsigned TT>
R48_HD uint32_t bitop3(uint32_t a, uint32_t b, uint32_t c)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, c, TT);
#else
    uint32_t r = 0;
    for (int i = 0; i < 8; i++)
        if ((TT >> i) & 1u)
            r |= ((i & 4) ? a : ~a) & ((i & 2) ? b : ~b) & ((i & 1) ? c : ~c);
    return r;
#endif
}
// bytewise select m ? x : y (one v_bitop3_b32)
R48_HD uint32_t bsel(uint32_t m, uint32_t x, uint32_t y) { return bitop3<0xCAu>(m, x, y); }
R48_HD uint32_t or3(uint32_t a, uint32_t b, uint32_t c) { return bitop3<0xFEu>(a, b, c); }

// Byte-lane predicates, valid while every byte is <= 0x80 (cell exponents are 0..30):
// 0x80 in each byte that is nonzero / zero.
R48_HD uint32_t nz80(uint32_t x) { return (x + 0x7F7F7F7Fu) & 0x80808080u; }
R48_HD uint32_t z80(uint32_t x) { return ~(x + 0x7F7F7F7Fu) & 0x80808080u; }
// Bit-7 flags f -> 0x7F byte masks (f - f >> 7: two full-rate instructions). A 0x7F mask selects
// a whole cell: cells are exponents <= 30, so bit 7 of every board byte is 0.
R48_HD uint32_t m7f(uint32_t f) { return f - (f >> 7); }
// 0x7F in each nonzero byte of x (bytes <= 0x80)
R48_HD uint32_t nz7f(uint32_t x) { return m7f(nz80(x)); }

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
// values) when REWARD, else 0. Every instruction is full rate (add/sub/shift/bitop3; byte masks
// are 0x7F from m7f, not 0xFF from v_perm): ~50 VALU for all four lines.
template <bool REWARD>
R48_HD uint32_t move_lines(Board &L)
{
    uint32_t l0 = L.w0, l1 = L.w1, l2 = L.w2, l3 = L.w3;
    // (1) compaction, from the far side in: where line cell i is empty, the cells behind it
    //     shift one place toward L[0] (GameClient.py:147-160: j skips empties, i takes j).
    //     Where cell i is empty it is 0, so "i takes i+1" is i | (i+1 & ~k).
    uint32_t k = nz7f(l2);
    l2 = bitop3<0xF4u>(l2, l3, k);   // l2 | (l3 & ~k)
    l3 &= k;
    k = nz7f(l1);
    l1 = bitop3<0xF4u>(l1, l2, k);
    l2 = bsel(k, l2, l3);
    l3 &= k;
    k = nz7f(l0);
    l0 = bitop3<0xF4u>(l0, l1, k);
    l1 = bsel(k, l1, l2);
    l2 = bsel(k, l2, l3);
    l3 &= k;
    // (2) merge adjacent equal tiles once, nearest the wall first (GameClient.py:162-167):
    //     (0,1) always wins, (1,2) only if (0,1) did not, (2,3) unless (1,2) merged.
    //     Flags live in bit 7 of each byte: equal = bit 7 of 0x80 - (a^b) set, nonzero = bit 7
    //     of b + 0x7F set (after compaction a nonzero b has a nonzero a before it).
    const uint32_t e01 = bitop3<0x80u>(0x80808080u - (l0 ^ l1), l1 + 0x7F7F7F7Fu, 0x80808080u);
    const uint32_t e12 = bitop3<0x80u>(0x80808080u - (l1 ^ l2), l2 + 0x7F7F7F7Fu, 0x80808080u);
    const uint32_t e23 = bitop3<0x80u>(0x80808080u - (l2 ^ l3), l3 + 0x7F7F7F7Fu, 0x80808080u);
    const uint32_t f01 = e01;
    const uint32_t f12 = e12 & ~e01;
    const uint32_t f23 = bitop3<0xD0u>(e23, e01, e12);   // e23 & (e01 | ~e12)
    const uint32_t i01 = f01 >> 7, i12 = f12 >> 7, i23 = f23 >> 7;   // 0x01 per merging pair
    const uint32_t m01 = f01 - i01, m12 = f12 - i12, m23 = f23 - i23;  // 0x7F per merging pair
    uint32_t reward = 0;
    // apply the far pair first so the nearer pairs' shifts carry its result along
    l2 += i23;
    if (REWARD) {
        for (int b = 0; b < 4; b++)
            reward += ((i23 >> (8 * b)) & 1u) << ((l2 >> (8 * b)) & 31u);
    }
    l3 &= ~m23;
    l1 += i12;
    if (REWARD) {
        for (int b = 0; b < 4; b++)
            reward += ((i12 >> (8 * b)) & 1u) << ((l1 >> (8 * b)) & 31u);
    }
    l2 = bsel(m12, l3, l2);
    l3 &= ~m12;
    l0 += i01;
    if (REWARD) {
        for (int b = 0; b < 4; b++)
            reward += ((i01 >> (8 * b)) & 1u) << ((l0 >> (8 * b)) & 31u);
    }
    l1 = bsel(m01, l2, l1);
    l2 = bsel(m01, l3, l2);
    l3 &= ~m01;
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

// select_blank + place in one, full-rate VALU only. The row of the rank-th blank is the last k
// with rank >= p_k: n_k = (rank - p_k) >> 31 (arithmetic) is -1 for the rows after it, and
// three bitop3 selects each pick the row's blank flags z and the rank within the row j. In the
// row, the blank whose inclusive byte prefix count (f * 0x01010101, f = 0x01 per blank) equals
// j + 1 is the one: its byte of P ^ splat(j + 1) is 0. `on` is a lane mask (0 / ~0): nothing
// is placed where it is 0 (an unchanged move spawns nothing, GameClient.py:48-49).
R48_HD void spawn_at_rank_m(Board &r, const Blanks &b, uint32_t rank, uint32_t e, uint32_t on)
{
    const uint32_t d1 = rank - b.p1, d2 = rank - b.p2, d3 = rank - b.p3;
    uint32_t n1 = (uint32_t)((int32_t)d1 >> 31), n2 = (uint32_t)((int32_t)d2 >> 31),
             n3 = (uint32_t)((int32_t)d3 >> 31);
#if defined(__HIP_DEVICE_COMPILE__)
    // opaque to the optimiser: knowing they are sign masks, it rebuilds n2 & ~n1 as a
    // compare + v_cndmask (two instructions, one half rate) instead of one v_bitop3
    asm("" : "+v"(n1), "+v"(n2), "+v"(n3));
#endif
    uint32_t z = bsel(n1, b.z0, b.z1);
    z = bsel(n2, z, b.z2);
    z = bsel(n3, z, b.z3);
    uint32_t j = bsel(n1, rank, d1);
    j = bsel(n2, j, d2);
    j = bsel(n3, j, d3);
    const uint32_t P = (z >> 7) * 0x01010101u;
    const uint32_t S = (j + 1u) * 0x01010101u;
    const uint32_t hit = bitop3<0x80u>(0x80808080u - (P ^ S), z, on);   // 0x80 in the chosen cell
    const uint32_t v = hit >> (8u - e);                                   // e = 1 (tile 2) or 2 (tile 4)
    r.w0 = bitop3<0xF8u>(r.w0, v, n1);        // w | (v & n1): row 0
    r.w1 = bitop3<0xF8u>(r.w1, v, n2 & ~n1);  // row 1
    r.w2 = bitop3<0xF8u>(r.w2, v, n3 & ~n2);  // row 2
    r.w3 = bitop3<0xF4u>(r.w3, v, n3);        // w | (v & ~n3): row 3
}

R48_HD void spawn_at_rank(Board &r, const Blanks &b, uint32_t rank, uint32_t e, bool on)
{
    spawn_at_rank_m(r, b, rank, e, on ? ~0u : 0u);
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
    // bit 7 of 0x80 - x per byte: that byte of x is 0. Horizontal pairs: w ^ (w >> 8), whose
    // top byte is the last cell itself (0 only on a board that is not full anyway).
    const uint32_t h = or3(0x80808080u - (r.w0 ^ (r.w0 >> 8)), 0x80808080u - (r.w1 ^ (r.w1 >> 8)),
                           0x80808080u - (r.w2 ^ (r.w2 >> 8)));
    const uint32_t v = or3(0x80808080u - (r.w3 ^ (r.w3 >> 8)), 0x80808080u - (r.w0 ^ r.w1),
                           0x80808080u - (r.w1 ^ r.w2));
    const uint32_t eq = or3(h, v, 0x80808080u - (r.w2 ^ r.w3)) & 0x80808080u;
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

// ---- Philox4x32-R (Salmon, Moraes, Dror, Shaw, SC'11) -----------------------------
// Round 0 stays in C so the compiler can move its wave-uniform counter words to the SALU;
// rounds 1.. fold each round's two XORs into one v_bitop3_b32.
template <int ROUNDS>
R48_HD void philox4x32_r(uint32_t c[4], uint32_t k0, uint32_t k1)
{
    R48_UNROLL
    for (int i = 0; i < ROUNDS; i++) {
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
#if defined(__HIP_DEVICE_COMPILE__)
        // the round keys are recomputed by two s_add per round instead of being hoisted out of
        // the callers' step loops into 20 SGPRs: the k_step_n kernels must stay under the SGPR
        // budget of 8 waves per SIMD (measured: 87 SGPRs + the trap handler's allocate 7)
        asm volatile("" : "+s"(k0), "+s"(k1));
#endif
    }
}

R48_HD void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) { philox4x32_r<10>(c, k0, k1); }

// Draw-word contract (DESIGN.md "Philox mode"; restated in oracle/r48_oracle.c)
static constexpr uint32_t kStepTag = 0x2048u;
// the env step's draws use Philox4x32-7, the fewest rounds the Philox authors found to pass
// BigCrush (draw contract version 3, round 4: the step's Philox was ~1/6 of the env kernels' VALU
// issue); every other draw (reset, fill, sampling, replay) keeps the default 10 rounds
static constexpr int kStepRounds = 7;
static constexpr uint32_t kResetTag = 0x5E7u;
static constexpr uint32_t kFillTag = 0xF111u;   // synthetic start boards (r48_env_fill_random)
static constexpr uint32_t kFourThresh = 0x1999999Au;     // P(4) = 0.1   (GameClient.py:125)
static constexpr uint32_t kFourThresh30 = 0x06666666u;   // same on 30 bits (P = 0.1 - 4e-10)
static constexpr uint32_t kFourThresh28 = 0x0199999Au;   // same on 28 bits

// The env step's draw words of board `gid` at step `step` (the k_step contract of r48_env.hip,
// DESIGN.md section 7): boards 2q, 2q + 1 share Philox4x32-7(key, {q lo, q hi, step, kStepTag});
// the even board takes (x, y) = (w0, w1), the odd one (w2, w3).
R48_HD void step_draw(uint64_t gid, uint32_t step, uint32_t k0, uint32_t k1, uint32_t &x, uint32_t &y)
{
    const uint64_t q = gid >> 1;
    uint32_t w[4] = {(uint32_t)q, (uint32_t)(q >> 32), step, kStepTag};
    philox4x32_r<kStepRounds>(w, k0, k1);
    x = (gid & 1u) ? w[2] : w[0];
    y = (gid & 1u) ? w[3] : w[1];
}

struct StepOut {
    uint32_t changed, done, n_blank, reward, score;
};

// ---- Orientations ---------------------------------------------------------------------
// A board may be held in the line form of any action o (to_lines(rows, o)) instead of in
// rows. Going from the line form of o to that of action a is one element of the 4x4
// board's symmetry group, M = P(a) o P(o)^-1 with P(UP) = I, P(DOWN) = Rev (word order
// reversed), P(LEFT) = T, P(RIGHT) = Rev T. The six elements that occur (I, Rev, T, Rev T,
// Br T = T Rev, Rev Br T; Br = byte order reversed within each word) all fit one 8-perm
// network with per-lane selectors:
//     X0 = perm(w1, w0, x0)   X1 = perm(w1, w0, x1)   Y0 = perm(w3, w2, x0)   Y1 = perm(w3, w2, x1)
//     L0 = perm(Y0, X0, te)   L1 = perm(Y1, X1, te)   L2 = perm(Y0, X0, to)   L3 = perm(Y1, X1, to)
// so a step needs 8 v_perm_b32 and one 16-byte selector record {x0, x1, te, to} per board
// (the k_step_n kernels read it from a 256-byte LDS table, kOrient[o][a]) instead of
// to_lines + from_lines (16 perms + 16 per-lane selects).
struct Orient {
    uint32_t x0, x1, te, to;
};

#define R48_OR_I {0x03020100u, 0x07060504u, 0x03020100u, 0x07060504u}
#define R48_OR_REV {0x07060504u, 0x03020100u, 0x07060504u, 0x03020100u}
#define R48_OR_T {0x06020400u, 0x07030501u, 0x05040100u, 0x07060302u}
#define R48_OR_REVT {0x05010703u, 0x04000602u, 0x05040100u, 0x07060302u}
#define R48_OR_BRT {0x06020400u, 0x07030501u, 0x00010405u, 0x02030607u}
#define R48_OR_REVBRT {0x05010703u, 0x04000602u, 0x00010405u, 0x02030607u}
// kOrient[4 * o + a]: from the line form of o (0 UP = rows, 1 DOWN, 2 LEFT, 3 RIGHT) to that of a
static constexpr Orient kOrient[16] = {
    R48_OR_I,   R48_OR_REV,    R48_OR_T,   R48_OR_REVT,     // o = UP (rows)
    R48_OR_REV, R48_OR_I,      R48_OR_BRT, R48_OR_REVBRT,   // o = DOWN
    R48_OR_T,   R48_OR_REVT,   R48_OR_I,   R48_OR_REV,      // o = LEFT
    R48_OR_BRT, R48_OR_REVBRT, R48_OR_REV, R48_OR_I,        // o = RIGHT
};
#undef R48_OR_I
#undef R48_OR_REV
#undef R48_OR_T
#undef R48_OR_REVT
#undef R48_OR_BRT
#undef R48_OR_REVBRT

R48_HD Board reorient(const Board &w, const Orient &s)
{
    const uint32_t X0 = perm(w.w1, w.w0, s.x0), X1 = perm(w.w1, w.w0, s.x1);
    const uint32_t Y0 = perm(w.w3, w.w2, s.x0), Y1 = perm(w.w3, w.w2, s.x1);
    return Board{perm(Y0, X0, s.te), perm(Y1, X1, s.te), perm(Y0, X0, s.to), perm(Y1, X1, s.to)};
}

// The move + spawn + game-over of one Philox-mode step on a board ALREADY in the line form
// of action a (Game.step, GameClient.py:40-51). The spawn rank counts blanks in line order --
// L[0] bytes 0..3, then L[1], ... (distance from the wall the tiles move toward, then line
// index) -- the build's Philox contract: the rank is uniform, so the
// spawned cell is uniform over the blanks in any fixed order, as random_fill_grid's is
// (GameClient.py:109-122); the reference's row-major order is kept by the injected-draw path
// (step_board<.., RANK_IS_INDEX = true>). Game over is invariant under the board's symmetries.
// VALID_ACTION: a < 4 is guaranteed (in-kernel random policy), so the moved lines are taken as
// they are (an unchanged move leaves them as they were).
template <bool REWARD, bool VALID_ACTION>
R48_HD StepOut step_lines(Board &L, uint32_t a, uint32_t rank_word, bool four)
{
    StepOut o;
    const Board L0 = L;
    o.reward = move_lines<REWARD>(L);
    const uint32_t diff = or3(L.w0 ^ L0.w0, L.w1 ^ L0.w1, L.w2 ^ L0.w2) | (L.w3 ^ L0.w3);
    // changed as a lane mask (0 / ~0) without a compare + select: bit 31 of diff | -diff
    uint32_t on = (uint32_t)((int32_t)(diff | (0u - diff)) >> 31);
    if (!VALID_ACTION) {
        on = a < 4u ? on : 0u;
        L = Board{bsel(on, L.w0, L0.w0), bsel(on, L.w1, L0.w1), bsel(on, L.w2, L0.w2), bsel(on, L.w3, L0.w3)};
    }
    o.reward = REWARD ? (o.reward & on) : 0u;
    const Blanks bl = blanks(L);
    o.n_blank = bl.n;
    spawn_at_rank_m(L, bl, mulhi(rank_word, bl.n), four ? 2u : 1u, on);
    o.changed = on & 1u;
    o.done = game_over(L, bl.n + on);   // blanks after the spawn: n - 1 where one was placed
    return o;
}

// One env step on row words (Game.step, GameClient.py:40-51) given the action and the two
// spawn draws. `rank_word` is either a Philox word (rank = mulhi(word, n_blank), blanks in
// line order: step_lines) or, when RANK_IS_INDEX, the injected rank itself (taken modulo
// n_blank, blanks in the reference's row-major order, GameClient.py:109-114). VALID_ACTION:
// the caller guarantees a < 4 (in-kernel random policy), so the moved board is taken as is --
// an unchanged move maps back to the same board (from_lines inverts to_lines exactly).
template <bool REWARD, bool RANK_IS_INDEX, bool VALID_ACTION = false>
R48_HD StepOut step_board(Board &r, uint32_t a, uint32_t rank_word, bool four)
{
    const uint32_t ac = a & 3u;
    Board L = to_lines(r, ac);
    if (!RANK_IS_INDEX) {
        const StepOut o = step_lines<REWARD, VALID_ACTION>(L, a, rank_word, four);
        r = from_lines(L, ac);
        return o;
    }
    StepOut o;
    const bool valid = VALID_ACTION || a < 4u;
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
    const uint32_t rank = bl.n ? rank_word % bl.n : 0u;
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
