// r48_sample.h -- the A3C action-sample draw (LocalAgent.choose_action, algorithm/a3c/a3c.py:89-93:
// np.random.choice over the softmax), shared by r48_sample_actions (r48_a3c.hip), the fused policies
// (r48_policy.hip, r48_mlp.hip) and their rollout megakernels.
//
// The uniform of board `gid` at sample counter `ctr` is word (ctr & 3) of
//   Philox4x32-10(key = {seed lo, seed hi}, counter = {gid lo, gid hi, ctr >> 2, 0xA3C}),
// its top 24 bits scaled to [0, 1) (draw contract version 4, include/rein48.h R48_DRAW_CONTRACT;
// oracle: tests/test_a3c_gpu.py restates it over oracle/r48_oracle.c's Philox). One block serves
// four consecutive counters of a board, so a rollout that keeps the board in registers computes it
// every fourth step and carries the words (SampleWords) instead of one block per board-step, of
// which it used one word (version <= 3).
#pragma once
#include <cstdint>

#include "r48_board.h"

namespace r48 {

constexpr uint32_t kSampleTag = 0xA3Cu;

R48_HD void sample_block(uint64_t gid, uint32_t ctr, uint32_t k0, uint32_t k1, uint32_t w[4])
{
    w[0] = (uint32_t)gid;
    w[1] = (uint32_t)(gid >> 32);
    w[2] = ctr >> 2;
    w[3] = kSampleTag;
    philox4x32_10(w, k0, k1);
}

// the sample word of (gid, ctr) on its own (one block per call: the per-step kernels)
R48_HD uint32_t sample_word(uint64_t gid, uint32_t ctr, uint32_t k0, uint32_t k1)
{
    uint32_t w[4];
    sample_block(gid, ctr, k0, k1, w);
    const uint32_t j = ctr & 3u;
    return j == 0u ? w[0] : j == 1u ? w[1] : j == 2u ? w[2] : w[3];
}

// the words of counters ctr, ctr + 1, ... for a rollout: next(ctr) returns the word of ctr, computing
// a block only at the first call and whenever ctr is a multiple of 4. Calls must come with
// consecutive counters; `ctr` is the same in every lane (the branch is wave-uniform).
struct SampleWords {
    uint32_t w[4];
    bool started = false;
    R48_HD uint32_t next(uint64_t gid, uint32_t ctr, uint32_t k0, uint32_t k1)
    {
        if (!started || (ctr & 3u) == 0u) {
            sample_block(gid, ctr, k0, k1, w);
            for (uint32_t j = 0; j < (ctr & 3u); j++) {   // first call only: skip the block's earlier words
                w[0] = w[1];
                w[1] = w[2];
                w[2] = w[3];
            }
            started = true;
        }
        const uint32_t cur = w[0];
        w[0] = w[1];
        w[1] = w[2];
        w[2] = w[3];
        return cur;
    }
};

// inverse CDF of the softmax of z at u = word >> 8 (24 bits): the first action whose cumulative
// probability exceeds u (np.random.choice's searchsorted(..., side='right'))
__device__ __forceinline__ uint32_t sample_from_word(const float (&z)[4], uint32_t word)
{
    const float m = fmaxf(fmaxf(z[0], z[1]), fmaxf(z[2], z[3]));
    const float e0 = __expf(z[0] - m), e1 = __expf(z[1] - m), e2 = __expf(z[2] - m), e3 = __expf(z[3] - m);
    const float inv = 1.0f / (e0 + e1 + e2 + e3);
    const float p0 = e0 * inv, c1 = p0 + e1 * inv, c2 = c1 + e2 * inv;
    const float u = (float)(word >> 8) * (1.0f / 16777216.0f);
    return (p0 > u) ? 0u : (c1 > u) ? 1u : (c2 > u) ? 2u : 3u;
}

}  // namespace r48
