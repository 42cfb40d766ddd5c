// r48_resnet.hip -- fused ResNet-10 Q-network inference on gfx950 MFMA (BASELINE config 5).
//
// rein48_amd/dqn/nets.py:ResNet10Q in eval mode (BatchNorm folded by k_resnet_pack or the host
// pack_resnet), forward only, for acting on millions of boards:
//   x   = one-hot of the 16 cell exponents (18 planes)
//   h   = relu(conv3x3(x))                                     stem, 18 -> 64
//   4 x h = relu(conv3x3(relu(conv3x3(h))) + h)                basic blocks, 64 -> 64
//   Q   = Wh . flatten(h) + bh                                 head, 1024 -> 4
// and optionally the epsilon-greedy draw of r48_egreedy_actions (same Philox contract).
//
// Cell-grouped tiling (replaced a 32x32x16 kernel with columns = 2 boards x 16 cells and the
// taps as DPP row shifts: that one issued all 144 (cell, tap) pairs with zero fill and re-read an
// LDS weight fragment every 4 MFMAs -- 14.8 ms per 2^21 boards against 8.9 ms here):
// v_mfma_f32_16x16x32_bf16 with rows = 16 output channels (four row tiles per 64-channel layer)
// and columns = 16 BOARDS at the SAME cell. A wave owns 16 boards and keeps all 16 cells of
// them in registers: x[cell][k-chunk][4] packed bf16, lane l = board l & 15, channel group
// g = l >> 4. The 3x3 tap (dr, dc) of output cell p reads input cell q = p + 4dr + dc, i.e.
// simply another register array -- no lane movement, and only the 100 in-grid (cell, tap)
// pairs are issued (the 32x32 kernel issues all 144 with zero fill). One LDS weight fragment
// (tap, row tile, k-chunk) feeds every cell that has that tap (9, 12 or 16 MFMAs).
// Accumulator layout (16x16): lane l holds rows 4g..4g+3 of column l & 15, so a finished row
// tile o leaves channels 16o + 4g + i of board l & 15 in the lane; k-chunk c of the next layer
// packs tiles 2c and 2c+1: element j <-> channel 16(2c + (j >> 2)) + 4g + (j & 3), and the
// host packs the A fragments with the same k order. Row tiles run one after another, each
// finishing with its epilogue (bias [+ residual], ReLU, bf16), so only 16 x 4 accumulators are
// live (VGPRs); the activations sit in AGPRs. A basic block's second conv starts its
// accumulators from bias + the block input (the skip connection, as an identity MFMA) and writes
// its output over that input.
// Weights stream per layer (stem 37, conv 73, head 33 fragments of 1 KiB) into a
// double-buffered LDS image by global_load_lds while the other buffer's layer computes; one
// persistent workgroup per CU, 4 waves (one per SIMD: 256 VGPR + 208 AGPR, no scratch), 64
// boards per tile.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/rein48.h"
#include "r48_board.h"
#include "r48_host.h"

namespace r48 {
void set_last_error(const std::string &msg);
}

namespace {

using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
using f32x4 = __attribute__((ext_vector_type(4))) float;
using u32x4 = __attribute__((ext_vector_type(4))) uint32_t;
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));

constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kBoardsPerTile = 16 * kWaves;
constexpr int kConvLayers = 8;
constexpr int kStemBlock = 9 * 4 + 1;        // (tap, row tile) fragments + bias fragment
constexpr int kConvBlock = 9 * 4 * 2 + 1;    // (tap, row tile, k-chunk) + bias
constexpr int kHeadBlock = 16 * 2 + 1;       // (cell, k-chunk) + bias (4 floats)
constexpr int kBufFrags = kConvBlock;        // 73 KiB per LDS buffer
constexpr int kHeadOff = kStemBlock + kConvLayers * kConvBlock;
constexpr int kBlobFrags = kHeadOff + kHeadBlock;
constexpr uint32_t kEgreedyTag = 0xD0Eu;

// wl = the lane's 16 B in a weight image (buffer base + lane, see k_resnet_q's begin): fragment f
// is one ds_read_b128 at immediate offset 1024 f
__device__ __forceinline__ bf16x8 lds_frag(const uint4 *wl, int frag, int)
{
    const uint4 v = wl[frag * 64];
    return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ bf16x8 as_b(const uint32_t (&r)[4])
{
    const u32x4 v = {r[0], r[1], r[2], r[3]};
    return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c)
{
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float bf_lo(uint32_t v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float bf_hi(uint32_t v) { return __uint_as_float(v & 0xFFFF0000u); }

// relu(lo, hi) as one packed bf16 pair (one v_cvt_pk_bf16_f32, RNE; then ReLU as signed-int16 max)
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t relu_pack(float lo, float hi)
{
    const i16x2 p = __builtin_bit_cast(i16x2, __builtin_convertvector(f32x2{lo, hi}, bf16x2_t));
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(p, i16x2{0, 0}));
}

// identity A fragment of row tile O's position in its k-chunk (O & 1): row r = lane & 15 picks
// channel 16 O + r, which sits in lane group g = r >> 2 at element 4 (O & 1) + (r & 3); MFMA-ing it
// with the block input adds the skip connection exactly (1.0 x bf16 in f32)
__device__ __forceinline__ bf16x8 identity_frag(int odd, int lane)
{
    const int r = lane & 15, g = lane >> 4;
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (g == (r >> 2)) {
        const int j = 4 * odd + (r & 3);
        w[j >> 1] = 0x3F80u << (16 * (j & 1));
    }
    return as_b(w);
}

// a packed activation defined in an AGPR: the layer activations h and y (128 registers each) live
// in the accumulator file -- they are only ever MFMA B operands, which may be AGPRs -- leaving the
// VGPRs to the live accumulators, the prefetched weight fragments and addresses (with y in VGPRs
// the scheduler had no room to read fragments ahead: 9.77 -> 8.89 ms per 2^21 boards)
__device__ __forceinline__ uint32_t in_agpr(uint32_t v)
{
    uint32_t r;
    asm("v_accvgpr_write_b32 %0, %1" : "=a"(r) : "v"(v));
    return r;
}

// tap order of a row tile: the centre (all 16 cells, starts the accumulators) first
__device__ constexpr int kTapOrder[9] = {4, 0, 1, 2, 3, 5, 6, 7, 8};

// row tile O of a layer: 9 NC fragment groups (tap, k-chunk), each one LDS fragment applied to every
// in-grid cell of its tap; the next group's fragment is read before this group's MFMAs issue
// (one group of MFMA time to land). Accumulators start at the bias (+ the skip connection through
// the identity fragment); `mid` runs between the MFMAs and the epilogue (see layer)
template <int NC, bool RESID, bool OUT_A, int O, typename Mid>
__device__ __forceinline__ void row_tile(const uint4 *wl, const float *bias, const uint32_t (&x)[16][NC][4],
                                         uint32_t (&out)[16][2][4], const bf16x8 (&ident)[2], int lane, Mid &&mid)
{
    const int g = lane >> 4;
    const f32x4 b4 = *reinterpret_cast<const f32x4 *>(bias + 16 * O + 4 * g);
    constexpr int s = O >> 1, w = 2 * (O & 1);
    constexpr int kGroups = 9 * NC;
    f32x4 acc[16];
    bf16x8 A = lds_frag(wl, (4 * 4 + O) * NC, lane);
#pragma unroll
    for (int k = 0; k < kGroups; k++) {
        const int t = kTapOrder[k / NC], c = k % NC;
        bf16x8 An = A;
        if (k + 1 < kGroups)
            An = lds_frag(wl, (kTapOrder[(k + 1) / NC] * 4 + O) * NC + (k + 1) % NC, lane);
        const int DR = t / 3 - 1, DC = t % 3 - 1;
#pragma unroll
        for (int p = 0; p < 16; p++) {
            const int r = p >> 2, cc = p & 3;
            if (r + DR < 0 || r + DR > 3 || cc + DC < 0 || cc + DC > 3)
                continue;
            if (k == 0) {
                const f32x4 init = RESID ? mfma(ident[O & 1], as_b(out[p][s]), b4) : b4;
                acc[p] = mfma(A, as_b(x[p][0]), init);
            } else {
                acc[p] = mfma(A, as_b(x[p + 4 * DR + DC][c]), acc[p]);
            }
        }
        A = An;
    }
    mid();
#pragma unroll
    for (int p = 0; p < 16; p++) {
        const uint32_t lo = relu_pack(acc[p][0], acc[p][1]), hi = relu_pack(acc[p][2], acc[p][3]);
        out[p][s][w] = OUT_A ? in_agpr(lo) : lo;
        out[p][s][w + 1] = OUT_A ? in_agpr(hi) : hi;
    }
}

template <int NC, bool RESID, bool OUT_A, typename Next>
__device__ __forceinline__ void layer(const uint4 *const (&w)[2], const uint32_t (&x)[16][NC][4],
                                      uint32_t (&out)[16][2][4], const bf16x8 (&ident)[2], int lane, Next &&next)
{
    const uint4 *wl = w[0];
    const float *bias = reinterpret_cast<const float *>(w[1] + 9 * 4 * NC * 64);
    auto none = [] {};
    row_tile<NC, RESID, OUT_A, 0>(wl, bias, x, out, ident, lane, none);
    row_tile<NC, RESID, OUT_A, 1>(wl, bias, x, out, ident, lane, none);
    row_tile<NC, RESID, OUT_A, 2>(wl, bias, x, out, ident, lane, none);
    row_tile<NC, RESID, OUT_A, 3>(wl, bias, x, out, ident, lane, next);
}

// LDS-DMA of one weight block (frags x 1 KiB): wave w moves fragments w, w + 4, ...
__device__ __forceinline__ void stage_block(const uint4 *src, uint4 *dst, int frags, int wave, int lane)
{
    for (int f = wave; f < frags; f += kWaves)
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(src + f * 64 + lane),
                                         (__attribute__((address_space(3))) void *)(dst + f * 64), 16, 0, 0);
}

__device__ __forceinline__ void stage(const uint4 *blob, int blk, uint4 *dst, int wave, int lane)
{
    // blk 0 = stem, 1..8 = conv1..8, 9 = head
    if (blk == 0)
        stage_block(blob, dst, kStemBlock, wave, lane);
    else if (blk <= kConvLayers)
        stage_block(blob + (kStemBlock + (blk - 1) * kConvBlock) * 64, dst, kConvBlock, wave, lane);
    else
        stage_block(blob + kHeadOff * 64, dst, kHeadBlock, wave, lane);
}

__global__ __launch_bounds__(kThreads, 1) void k_resnet_q(const int8_t *__restrict__ boards, int64_t n,
                                                          const uint4 *__restrict__ blob, float *__restrict__ q_out,
                                                          int8_t *__restrict__ actions, float eps, uint32_t k0,
                                                          uint32_t k1, int64_t gid0, uint32_t ctr)
{
    extern __shared__ uint4 lds[];                  // [2][kBufFrags * 64]
    auto buf = [](int i) { return lds + i * (kBufFrags * 64); };
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4;
    const int64_t tiles = (n + kBoardsPerTile - 1) / kBoardsPerTile;
    int cur = 0;
    if ((int64_t)blockIdx.x < tiles)
        stage(blob, 0, buf(0), wave, lane);

    uint32_t h[16][2][4], y[16][2][4];
    const bf16x8 ident[2] = {identity_frag(0, lane), identity_frag(1, lane)};
    for (int64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
        const int64_t b = tile * kBoardsPerTile + wave * 16 + (lane & 15);
        uint4 bd = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);   // past n: no plane set
        if (b < n)
            bd = reinterpret_cast<const uint4 *>(boards)[b];
        const uint32_t bw[4] = {bd.x, bd.y, bd.z, bd.w};
        // one-hot stem input: cell q, element j of the lane's k slots = plane 8g + j
        uint32_t oh[16][1][4];
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const uint32_t d = ((bw[q >> 2] >> (8 * (q & 3))) & 0xFFu) - (uint32_t)(8 * g);
            const uint32_t one = 0x3F80u << (16 * (d & 1u));
#pragma unroll
            for (int r = 0; r < 4; r++)
                oh[q][0][r] = (d < 8u && (d >> 1) == (uint32_t)r) ? one : 0u;
        }
        // weight block blk landed in buf(cur) (own DMA + barrier); the next block (or the next
        // tile's stem) goes into the other buffer, which every wave has finished reading
        // -> {the lane's 16 B in the image, the image base}. The lane offset is hidden from the
        // optimiser per layer, so each fragment read is one ds_read_b128 at an immediate offset
        // from it, instead of per-fragment addresses hoisted out of the tile loop (and spilled)
        auto begin = [&](int blk, const uint4 *(&w)[2]) {
            __builtin_amdgcn_s_waitcnt(0);
            __syncthreads();
            if (blk + 1 < kConvLayers + 2)
                stage(blob, blk + 1, buf(cur ^ 1), wave, lane);
            else if (tile + gridDim.x < tiles)
                stage(blob, 0, buf(cur ^ 1), wave, lane);
            int idx = cur * (kBufFrags * 64) + lane;
            asm volatile("" : "+v"(idx));
            w[0] = lds + idx;
            w[1] = buf(cur);
            cur ^= 1;
        };
        const uint4 *w[2];
        begin(0, w);
        layer<1, false, true>(w, oh, h, ident, lane, [&] { begin(1, w); });
        for (int blk = 0; blk < kConvLayers / 2; blk++) {
            // first conv of a block: h stays as the skip; second conv: bias + skip, output over h
            layer<2, false, true>(w, h, y, ident, lane, [&] { begin(2 + 2 * blk, w); });
            layer<2, true, true>(w, y, h, ident, lane, [&] { begin(3 + 2 * blk, w); });
        }
        {
            // head (its weights were begun inside the last conv): Q rows = actions (fragment
            // rows >= 4 are zero), columns = the 16 boards
            f32x4 qa = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int p = 0; p < 16; p++)
#pragma unroll
                for (int c = 0; c < 2; c++)
                    qa = mfma(lds_frag(w[0], 2 * p + c, lane), as_b(h[p][c]), qa);
            const float *hb = reinterpret_cast<const float *>(w[1] + 32 * 64);
            if (g == 0 && b < n) {
                const float4 qv = make_float4(qa[0] + hb[0], qa[1] + hb[1], qa[2] + hb[2], qa[3] + hb[3]);
                if (q_out)
                    reinterpret_cast<float4 *>(q_out)[b] = qv;
                if (actions) {
                    const uint64_t gid = (uint64_t)(gid0 + b);
                    uint32_t wv[4] = {(uint32_t)gid, (uint32_t)(gid >> 32), ctr, kEgreedyTag};
                    r48::philox4x32_10(wv, k0, k1);
                    const float u = (float)(wv[0] >> 8) * (1.0f / 16777216.0f);
                    uint32_t am = 0;
                    float mx = qv.x;
                    if (qv.y > mx) { mx = qv.y; am = 1; }
                    if (qv.z > mx) { mx = qv.z; am = 2; }
                    if (qv.w > mx) { am = 3; }
                    actions[b] = (int8_t)(u < eps ? (wv[1] >> 30) : am);
                }
            }
        }
    }
    __builtin_amdgcn_s_waitcnt(0);                     // no DMA left in flight at exit
}

// ---- packing (BN fold + fragment layout), one thread per bf16 of the blob. ptr[6 L + {0..5}] =
// conv L's weight [co][ci][3][3], bias [co], BN gamma, beta, running mean, running var (gamma
// NULL: no BN); ptr[54], ptr[55] = head weight [4][1024], bias [4]. Folding as
// ResNet10Q.folded(): s = gamma / sqrt(var + eps), w s, (b - mean) s + beta (f32, correctly rounded).
__device__ __forceinline__ float bn_scale(const float *const *p, int L, int co, float eps)
{
    const float *gm = p[6 * L + 2];
    return gm ? __fdiv_rn(gm[co], __fsqrt_rn(__fadd_rn(p[6 * L + 5][co], eps))) : 1.0f;
}

__device__ __forceinline__ float folded_bias(const float *const *p, int L, int co, float eps)
{
    const float b = p[6 * L + 1][co];
    return p[6 * L + 2] ? __fadd_rn(__fmul_rn(__fsub_rn(b, p[6 * L + 4][co]), bn_scale(p, L, co, eps)), p[6 * L + 3][co])
                        : b;
}

__global__ __launch_bounds__(256) void k_resnet_pack(const float *const *__restrict__ p, float eps,
                                                       uint16_t *__restrict__ blob)
{
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= (int64_t)kBlobFrags * 512)
        return;
    const int frag = (int)(e >> 9), within = (int)(e & 511), lane = within >> 3, j = within & 7;
    const int r = lane & 15, g = lane >> 4;
    int kind, L, f;        // kind 0 stem, 1 conv, 2 head
    if (frag < kStemBlock)
        kind = 0, L = 0, f = frag;
    else if (frag < kHeadOff)
        kind = 1, L = 1 + (frag - kStemBlock) / kConvBlock, f = (frag - kStemBlock) % kConvBlock;
    else
        kind = 2, L = 9, f = frag - kHeadOff;
    const int nfrag = kind == 0 ? 36 : kind == 1 ? 72 : 32;
    uint16_t out;
    if (f == nfrag) {      // bias fragment: f32 words (64 channels, or 4 head biases), zero padded
        const int word = within >> 1, half = within & 1;
        float v = 0.0f;
        if (kind == 2 && word < 4)
            v = p[55][word];
        else if (kind != 2 && word < 64)
            v = folded_bias(p, L, word, eps);
        out = (uint16_t)(__float_as_uint(v) >> (16 * half));
    } else {
        const int ci = 16 * (2 * (f & 1) + (j >> 2)) + 4 * g + (j & 3);   // conv / head k order
        float v = 0.0f;
        if (kind == 0) {
            const int t = f >> 2, o = f & 3, co = 16 * o + r, plane = 8 * g + j;
            if (plane < 18)
                v = __fmul_rn(p[0][((int64_t)co * 18 + plane) * 9 + t], bn_scale(p, 0, co, eps));
        } else if (kind == 1) {
            const int t = f >> 3, o = (f >> 1) & 3, co = 16 * o + r;
            v = __fmul_rn(p[6 * L][((int64_t)co * 64 + ci) * 9 + t], bn_scale(p, L, co, eps));
        } else {
            const int cell = f >> 1;
            if (r < 4)
                v = p[54][r * 1024 + cell * 64 + ci];
        }
        out = __builtin_bit_cast(uint16_t, (__bf16)v);
    }
    blob[e] = out;
}

int fail(int code, const char *msg)
{
    r48::set_last_error(msg);
    return code;
}

}  // namespace

extern "C" {

int r48_resnet_q_forward(const int8_t *boards, int64_t n, const void *wblob, float *q, int8_t *actions, float eps,
                          uint64_t seed, int64_t gid0, uint32_t ctr, void *stream)
{
    if (!boards || !wblob || n < 0 || gid0 < 0 || (!q && !actions))
        return fail(R48_EINVAL, "NULL argument, n/gid0 < 0, or neither q nor actions requested");
    if (((uintptr_t)wblob & 15u) || ((uintptr_t)boards & 15u) || (q && ((uintptr_t)q & 15u)))
        return fail(R48_EINVAL, "boards, wblob and q must be 16-byte aligned");
    if (n == 0)
        return R48_OK;
    const int dev = r48::stream_device((hipStream_t)stream);
    const int cus = r48::device_cus(dev);
    const int64_t tiles = (n + kBoardsPerTile - 1) / kBoardsPerTile;
    const int grid = (int)(tiles < cus ? tiles : cus);
    const size_t lds = (size_t)(2 * kBufFrags * 64) * 16;
    if (!r48::ensure_dynamic_lds(reinterpret_cast<const void *>(k_resnet_q), (int)lds, dev))
        return R48_EHIP;
    hipLaunchKernelGGL(k_resnet_q, dim3(grid), dim3(kThreads), lds, (hipStream_t)stream, boards, n,
                       reinterpret_cast<const uint4 *>(wblob), q, actions, eps, (uint32_t)seed,
                       (uint32_t)(seed >> 32), gid0, ctr);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        r48::set_last_error(std::string("k_resnet_q: ") + hipGetErrorString(e));
        return R48_EHIP;
    }
    return R48_OK;
}

int64_t r48_resnet_q_blob_bytes(void) { return (int64_t)kBlobFrags * 1024; }

int r48_resnet_pack(const float *const *ptrs, float bn_eps, void *wblob, void *stream)
{
    if (!ptrs || !wblob || ((uintptr_t)wblob & 15u))
        return fail(R48_EINVAL, "r48_resnet_pack: NULL or misaligned argument");
    const int64_t total = (int64_t)kBlobFrags * 512;
    hipLaunchKernelGGL(k_resnet_pack, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, ptrs,
                       bn_eps, (uint16_t *)wblob);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        r48::set_last_error(std::string("k_resnet_pack: ") + hipGetErrorString(e));
        return R48_EHIP;
    }
    return R48_OK;
}

}  // extern "C"
