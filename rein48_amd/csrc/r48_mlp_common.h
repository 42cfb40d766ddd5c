// r48_mlp_common.h -- what the MLP kernels (r48_mlp.hip: forward / rollout, r48_mlp_train.hip: the
// fused update) share: the weight blob's section offsets (rein48_amd/a3c/fused.py pack_mlp) and the
// board-cell -> network-input map (a3c.py:37-39,139).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/rein48.h"

namespace r48mlp {

// blob offsets: a1 [32 pairs][16 in][2] | a1.b [64] | a2 [32 pairs][4 out][2] | a2.b [4] |
// c1 [32 pairs][16 in][2] | c1.b [64] | c2 [64] | c2.b | 3 pad
constexpr int kA1W = 0, kA1B = 1024, kA2W = 1088, kA2B = 1344, kC1W = 1348, kC1B = 2372, kC2W = 2436, kC2B = 2500;
constexpr int kBlobFloats = 2504;

// cell exponent -> network input: the raw tile value 2^e (0 for an empty cell), exact in fp32, or e
template <int MODE>
__device__ __forceinline__ float cell_input(uint32_t e)
{
    if (MODE == R48_FEAT_EXPONENTS)
        return (float)e;
    return __uint_as_float(e ? (127u + e) << 23 : 0u);
}

}  // namespace r48mlp
