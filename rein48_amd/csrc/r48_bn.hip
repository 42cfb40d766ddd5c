// r48_bn.hip -- training-mode BatchNorm + ReLU (+ residual) for the ResNet-10 Q-network's update
// (BASELINE config 5; rein48_amd/dqn/nets.py), behind include/rein48.h.
//
// Activations are channels-last bf16 x[rows][C] (rows = boards x 16 cells, C = 64): every BN of
// the net is followed by a ReLU, the second BN of each basic block by the identity add first:
//     y = relu(a[c] * x + b[c] (+ residual)),  a = gamma * invstd,  b = beta - mean * a.
// PyTorch runs this as 4 channels-last BN kernels + ReLU/add/cast passes per layer at 0.7-1.5
// TB/s; here it is two streaming passes forward (statistics, apply) and two backward (reduce,
// apply), each one read of its inputs at HBM rate:
//   forward   k_bn_stats    per-channel shifted sums S1 = sum(x - x0), S2 = sum((x - x0)^2),
//                           x0 = row 0 (no cancellation when |mean| >> std), per-block partials
//             k_bn_finish   fixed-order fp64 sum of the partials -> mean, invstd, (a, b), running
//                           statistics (momentum, unbiased variance as torch.nn.BatchNorm1d)
//             k_bn_apply    y = relu(a x + b (+ res)), bf16 out
//   backward  k_bn_bwd_reduce  g = dy * [y > 0]; partials of sum(g), sum(g (x - mean))
//             k_bn_bwd_finish  dbeta, dgamma, and dx = a g + c x + d per channel (c, d fold the
//                              mean/variance terms of the BN gradient)
//             k_bn_bwd_apply   dx (bf16) and, with a residual, g itself (the residual's gradient)
// Deterministic: fixed grid, fixed reduction order. One thread owns 8 channels of a row (one 16-B
// load); a wave covers 64 / (C / 8) rows per instruction, contiguous in memory.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/rein48.h"
#include "r48_bn_finish.h"

namespace r48 {
void set_last_error(const std::string &msg);
}

namespace {

constexpr int kBlock = 256;
constexpr int kMaxBlocks = 1024;   // partial records per reduction (256 CUs x 4)
constexpr int kUnroll = 4;         // independent 16-B loads in flight per thread

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

int fail(int code, const char *msg)
{
    r48::set_last_error(msg);
    return code;
}

int launched(const char *what)
{
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        r48::set_last_error(std::string(what) + ": " + hipGetErrorString(e));
        return R48_EHIP;
    }
    return R48_OK;
}

__device__ __forceinline__ void unpack8(const uint4 v, float f[8])
{
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        f[2 * k] = __uint_as_float(w[k] << 16);
        f[2 * k + 1] = __uint_as_float(w[k] & 0xFFFF0000u);
    }
}

__device__ __forceinline__ uint32_t pack2(float lo, float hi)
{
    const bf16x2_t v = __builtin_convertvector((f32x2{lo, hi}), bf16x2_t);   // v_cvt_pk_bf16_f32 (RNE)
    return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ uint4 pack8(const float f[8])
{
    return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}

__device__ __forceinline__ uint4 ld16(const uint16_t *p, int64_t i)
{
    return *reinterpret_cast<const uint4 *>(p + i);
}

// rows are processed in groups of RPW = 64 / (C / 8) rows per wave and 4 * RPW per block: the
// thread's channel group cg = lane % LPR stays fixed, its row advances by the grid's row stride
template <int C>
struct Geo {
    static constexpr int LPR = C / 8;             // lanes per row
    static constexpr int RPB = kBlock / LPR;      // rows per block step
    __device__ static int cg() { return (int)(threadIdx.x % LPR); }
    __device__ static int64_t row0() { return (int64_t)blockIdx.x * RPB + threadIdx.x / LPR; }
    __device__ static int64_t stride() { return (int64_t)gridDim.x * RPB; }
};

// sum the per-thread accumulators of the threads that share a channel group (same lane % LPR)
// over the block; thread t < C of the block ends up with channel t's totals in out[0..NV)
template <int C, int NV>
__device__ __forceinline__ void block_channel_sum(float acc[NV][8], float *lds /* [kBlock/LPR... ] */,
                                                  float out[NV])
{
    constexpr int LPR = C / 8;
    // within the wave: lanes l, l + LPR, l + 2 LPR, ... share channels
#pragma unroll
    for (int off = LPR; off < 64; off <<= 1)
#pragma unroll
        for (int v = 0; v < NV; v++)
#pragma unroll
            for (int k = 0; k < 8; k++)
                acc[v][k] += __shfl_xor(acc[v][k], off, 64);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane < LPR) {
#pragma unroll
        for (int v = 0; v < NV; v++)
#pragma unroll
            for (int k = 0; k < 8; k++)
                lds[(wave * NV + v) * C + 8 * lane + k] = acc[v][k];
    }
    __syncthreads();
    if ((int)threadIdx.x < C) {
#pragma unroll
        for (int v = 0; v < NV; v++) {
            float s = 0.f;
#pragma unroll
            for (int w = 0; w < kBlock / 64; w++)
                s += lds[(w * NV + v) * C + threadIdx.x];
            out[v] = s;
        }
    }
}

// ---------------------------------------------------------------- forward
template <int C>
__global__ __launch_bounds__(kBlock) void k_bn_stats(const uint16_t *__restrict__ x, int64_t rows,
                                                     float *__restrict__ part)
{
    using G = Geo<C>;
    __shared__ float lds[(kBlock / 64) * 2 * C];
    const int cg = G::cg();
    float x0[8];
    unpack8(ld16(x, 8 * cg), x0);                 // shift = row 0
    float acc[2][8] = {};
    const int64_t st = G::stride();
    int64_t r = G::row0();
    for (; r + (kUnroll - 1) * st < rows; r += kUnroll * st) {
        uint4 v[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; u++)
            v[u] = ld16(x, (r + u * st) * C + 8 * cg);
#pragma unroll
        for (int u = 0; u < kUnroll; u++) {
            float f[8];
            unpack8(v[u], f);
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const float d = f[k] - x0[k];
                acc[0][k] += d;
                acc[1][k] = fmaf(d, d, acc[1][k]);
            }
        }
    }
    for (; r < rows; r += st) {
        float f[8];
        unpack8(ld16(x, r * C + 8 * cg), f);
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const float d = f[k] - x0[k];
            acc[0][k] += d;
            acc[1][k] = fmaf(d, d, acc[1][k]);
        }
    }
    float tot[2];
    block_channel_sum<C, 2>(acc, lds, tot);
    if ((int)threadIdx.x < C) {
        part[(int64_t)blockIdx.x * 2 * C + threadIdx.x] = tot[0];
        part[(int64_t)blockIdx.x * 2 * C + C + threadIdx.x] = tot[1];
    }
}

// fixed-order fp64 sum of the two partial rows of channel c over nblk block records: one block
// per channel, thread t takes records t, t + kBlock, ... and an LDS tree finishes (deterministic)
__device__ __forceinline__ void channel_totals(const float *part, int nblk, int C, int c, double &t0, double &t1)
{
    __shared__ double red[2][kBlock];
    double s0 = 0.0, s1 = 0.0;
    for (int b = threadIdx.x; b < nblk; b += kBlock) {
        s0 += (double)part[(int64_t)b * 2 * C + c];
        s1 += (double)part[(int64_t)b * 2 * C + C + c];
    }
    red[0][threadIdx.x] = s0;
    red[1][threadIdx.x] = s1;
    __syncthreads();
    for (int h = kBlock / 2; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) {
            red[0][threadIdx.x] += red[0][threadIdx.x + h];
            red[1][threadIdx.x] += red[1][threadIdx.x + h];
        }
        __syncthreads();
    }
    t0 = red[0][0];
    t1 = red[1][0];
}

__global__ __launch_bounds__(kBlock) void k_bn_finish(const uint16_t *__restrict__ x, const float *__restrict__ part,
                                                      int nblk, int C, int64_t rows, const float *__restrict__ gamma,
                                                      const float *__restrict__ beta, float *__restrict__ running_mean,
                                                      float *__restrict__ running_var, float momentum, float eps,
                                                      float *__restrict__ save, float *__restrict__ coef)
{
    const int c = blockIdx.x;
    double s1, s2;
    channel_totals(part, nblk, C, c, s1, s2);
    if (threadIdx.x != 0)
        return;
    const double x0 = x ? (double)__uint_as_float((uint32_t)x[c] << 16) : 0.0;   // shift (NULL: unshifted sums)
    const r48_bn_finish_args f{gamma, beta, running_mean, running_var, save, coef, nullptr, nullptr, rows, momentum, eps};
    r48bn::fwd_channel(f, C, c, s1, s2, x0);
}

// mask (optional, MASK): one byte per thread and row, bit k = (y[row][8 cg + k] > 0) -- the ReLU
// derivative the backward needs, 1/16 of the bytes of y
template <int C, bool RELU, bool RES, bool MASK>
__global__ __launch_bounds__(kBlock) void k_bn_apply(const uint16_t *__restrict__ x,
                                                     const uint16_t *__restrict__ res, int64_t rows,
                                                     const float *__restrict__ coef, uint16_t *__restrict__ y,
                                                     uint8_t *__restrict__ mask)
{
    using G = Geo<C>;
    const int cg = G::cg();
    float a[8], b[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        a[k] = coef[8 * cg + k];
        b[k] = coef[C + 8 * cg + k];
    }
    const int64_t st = G::stride();
    for (int64_t r = G::row0(); r < rows; r += st) {
        const int64_t o = r * C + 8 * cg;
        float f[8];
        unpack8(ld16(x, o), f);
        float q[8];
        if (RES)
            unpack8(ld16(res, o), q);
#pragma unroll
        for (int k = 0; k < 8; k++) {
            float v = fmaf(a[k], f[k], b[k]);
            if (RES)
                v += q[k];
            f[k] = RELU ? fmaxf(v, 0.f) : v;
        }
        const uint4 out = pack8(f);
        *reinterpret_cast<uint4 *>(y + o) = out;
        if (MASK) {
            const uint32_t w[4] = {out.x, out.y, out.z, out.w};
            uint32_t m = 0;
#pragma unroll
            for (int k = 0; k < 4; k++)
                m |= ((w[k] & 0x7FFFu) != 0 && !(w[k] & 0x8000u) ? 1u : 0u) << (2 * k) |
                     ((w[k] & 0x7FFF0000u) != 0 && !(w[k] & 0x80000000u) ? 1u : 0u) << (2 * k + 1);
            mask[o >> 3] = (uint8_t)m;
        }
    }
}

// ---------------------------------------------------------------- backward
// g = dy * [y > 0] (ReLU'), or dy; with MASK the ReLU derivative comes from the forward's mask
// bits instead of y
template <bool RELU, bool MASK>
__device__ __forceinline__ void grad_in(const uint16_t *dy, const uint16_t *y, const uint8_t *mask, int64_t o,
                                        float g[8])
{
    unpack8(ld16(dy, o), g);
    if (RELU && MASK) {
        const uint32_t m = mask[o >> 3];
#pragma unroll
        for (int k = 0; k < 8; k++)
            g[k] = (m >> k) & 1u ? g[k] : 0.f;
    } else if (RELU) {
        float yy[8];
        unpack8(ld16(y, o), yy);
#pragma unroll
        for (int k = 0; k < 8; k++)
            g[k] = yy[k] > 0.f ? g[k] : 0.f;
    }
}

template <int C, bool RELU, bool MASK>
__global__ __launch_bounds__(kBlock) void k_bn_bwd_reduce(const uint16_t *__restrict__ dy,
                                                          const uint16_t *__restrict__ y,
                                                          const uint8_t *__restrict__ mask,
                                                          const uint16_t *__restrict__ x, int64_t rows,
                                                          const float *__restrict__ save, float *__restrict__ part)
{
    using G = Geo<C>;
    __shared__ float lds[(kBlock / 64) * 2 * C];
    const int cg = G::cg();
    float mean[8];
#pragma unroll
    for (int k = 0; k < 8; k++)
        mean[k] = save[8 * cg + k];
    float acc[2][8] = {};
    const int64_t st = G::stride();
    int64_t r = G::row0();
    for (; r + (kUnroll - 1) * st < rows; r += kUnroll * st) {
        uint4 vd[kUnroll], vy[kUnroll], vx[kUnroll];
        uint32_t vm[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; u++) {
            const int64_t o = (r + u * st) * C + 8 * cg;
            vd[u] = ld16(dy, o);
            if (RELU && MASK)
                vm[u] = mask[o >> 3];
            else if (RELU)
                vy[u] = ld16(y, o);
            vx[u] = ld16(x, o);
        }
#pragma unroll
        for (int u = 0; u < kUnroll; u++) {
            float g[8], f[8], yy[8];
            unpack8(vd[u], g);
            unpack8(vx[u], f);
            if (RELU && !MASK)
                unpack8(vy[u], yy);
#pragma unroll
            for (int k = 0; k < 8; k++) {
                if (RELU && MASK)
                    g[k] = (vm[u] >> k) & 1u ? g[k] : 0.f;
                else if (RELU)
                    g[k] = yy[k] > 0.f ? g[k] : 0.f;
                acc[0][k] += g[k];
                acc[1][k] = fmaf(g[k], f[k] - mean[k], acc[1][k]);
            }
        }
    }
    for (; r < rows; r += st) {
        const int64_t o = r * C + 8 * cg;
        float g[8], f[8];
        grad_in<RELU, MASK>(dy, y, mask, o, g);
        unpack8(ld16(x, o), f);
#pragma unroll
        for (int k = 0; k < 8; k++) {
            acc[0][k] += g[k];
            acc[1][k] = fmaf(g[k], f[k] - mean[k], acc[1][k]);
        }
    }
    float tot[2];
    block_channel_sum<C, 2>(acc, lds, tot);
    if ((int)threadIdx.x < C) {
        part[(int64_t)blockIdx.x * 2 * C + threadIdx.x] = tot[0];
        part[(int64_t)blockIdx.x * 2 * C + C + threadIdx.x] = tot[1];
    }
}

// dbeta = sum g, dgamma = invstd sum g (x - mean);
// dx = a (g - dbeta / n - xhat dgamma / n) = a g + c x + d
__global__ __launch_bounds__(kBlock) void k_bn_bwd_finish(const float *__restrict__ part, int nblk, int C,
                                                          int64_t rows, const float *__restrict__ gamma,
                                                          const float *__restrict__ save, float *__restrict__ dgamma,
                                                          float *__restrict__ dbeta, float *__restrict__ coef)
{
    const int c = blockIdx.x;
    double sg, sgx;
    channel_totals(part, nblk, C, c, sg, sgx);
    if (threadIdx.x != 0)
        return;
    const r48_bn_finish_args f{gamma, nullptr, nullptr, nullptr, const_cast<float *>(save), coef, dgamma, dbeta, rows,
                               0.f, 0.f};
    r48bn::bwd_channel(f, C, c, sg, sgx);
}

template <int C, bool RELU, bool DRES, bool MASK>
__global__ __launch_bounds__(kBlock) void k_bn_bwd_apply(const uint16_t *__restrict__ dy,
                                                         const uint16_t *__restrict__ y,
                                                         const uint8_t *__restrict__ mask,
                                                         const uint16_t *__restrict__ x, int64_t rows,
                                                         const float *__restrict__ coef,
                                                         uint16_t *__restrict__ dx, uint16_t *__restrict__ dres)
{
    using G = Geo<C>;
    const int cg = G::cg();
    float a[8], cc[8], d[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        a[k] = coef[8 * cg + k];
        cc[k] = coef[C + 8 * cg + k];
        d[k] = coef[2 * C + 8 * cg + k];
    }
    const int64_t st = G::stride();
    for (int64_t r = G::row0(); r < rows; r += st) {
        const int64_t o = r * C + 8 * cg;
        float g[8], f[8], out[8];
        grad_in<RELU, MASK>(dy, y, mask, o, g);
        unpack8(ld16(x, o), f);
#pragma unroll
        for (int k = 0; k < 8; k++)
            out[k] = fmaf(a[k], g[k], fmaf(cc[k], f[k], d[k]));
        *reinterpret_cast<uint4 *>(dx + o) = pack8(out);
        if (DRES)
            *reinterpret_cast<uint4 *>(dres + o) = pack8(g);
    }
}

int reduce_blocks(int64_t rows, int C)
{
    const int64_t rpb = kBlock / (C / 8);
    int64_t b = (rows + rpb * kUnroll - 1) / (rpb * kUnroll);
    return (int)(b < 1 ? 1 : (b > kMaxBlocks ? kMaxBlocks : b));
}

// elementwise passes: one row group per thread (no grid-stride loop to pipeline), so the loads of
// many resident waves hide the latency
int apply_blocks(int64_t rows, int C)
{
    const int64_t rpb = kBlock / (C / 8);
    int64_t b = (rows + rpb - 1) / rpb;
    return (int)(b < 1 ? 1 : (b > 0x7FFFFFFF ? 0x7FFFFFFF : b));
}

bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

int check_args(const void *x, int64_t rows, int32_t C)
{
    if (!x || rows < 1)
        return fail(R48_EINVAL, "r48_bn: null activation or rows < 1");
    if (C != 32 && C != 64 && C != 128)
        return fail(R48_EINVAL, "r48_bn: C must be 32, 64 or 128");
    if (!aligned16(x))
        return fail(R48_EINVAL, "r48_bn: activations must be 16-byte aligned");
    return R48_OK;
}

template <int C, bool RELU, bool RES>
void launch_apply(dim3 g, hipStream_t s, const uint16_t *x, const uint16_t *res, int64_t rows, const float *coef,
                  uint16_t *y, uint8_t *mask)
{
    if (mask)
        hipLaunchKernelGGL((k_bn_apply<C, RELU, RES, true>), g, dim3(kBlock), 0, s, x, res, rows, coef, y, mask);
    else
        hipLaunchKernelGGL((k_bn_apply<C, RELU, RES, false>), g, dim3(kBlock), 0, s, x, res, rows, coef, y, mask);
}

template <int C>
int forward_c(const uint16_t *x, const uint16_t *res, int64_t rows, const float *gamma, const float *beta,
              float *rm, float *rv, float momentum, float eps, int relu, float *save, float *ws, uint16_t *y,
              uint8_t *mask, hipStream_t s)
{
    const int nb = reduce_blocks(rows, C);
    float *coef = ws + (int64_t)nb * 2 * C;
    hipLaunchKernelGGL(k_bn_stats<C>, dim3(nb), dim3(kBlock), 0, s, x, rows, ws);
    hipLaunchKernelGGL(k_bn_finish, dim3(C), dim3(kBlock), 0, s, x, ws, nb, C, rows, gamma, beta, rm, rv, momentum, eps,
                       save, coef);
    const dim3 g(apply_blocks(rows, C));
    if (relu && res)
        launch_apply<C, true, true>(g, s, x, res, rows, coef, y, mask);
    else if (relu)
        launch_apply<C, true, false>(g, s, x, res, rows, coef, y, mask);
    else if (res)
        launch_apply<C, false, true>(g, s, x, res, rows, coef, y, mask);
    else
        launch_apply<C, false, false>(g, s, x, res, rows, coef, y, mask);
    return launched("k_bn_apply");
}

// finish + apply from per-block sums a producer computed (r48_conv3x3 `stats`: unshifted)
template <int C>
int apply_c(const uint16_t *x, const uint16_t *res, int64_t rows, const float *coef, int relu, uint16_t *y, uint8_t *mask,
            hipStream_t s)
{
    const dim3 g(apply_blocks(rows, C));
    if (relu && res)
        launch_apply<C, true, true>(g, s, x, res, rows, coef, y, mask);
    else if (relu)
        launch_apply<C, true, false>(g, s, x, res, rows, coef, y, mask);
    else if (res)
        launch_apply<C, false, true>(g, s, x, res, rows, coef, y, mask);
    else
        launch_apply<C, false, false>(g, s, x, res, rows, coef, y, mask);
    return launched("k_bn_apply");
}

template <int C>
int forward_stats_c(const float *part, int nblk, const uint16_t *x, const uint16_t *res, int64_t rows,
                    const float *gamma, const float *beta, float *rm, float *rv, float momentum, float eps, int relu,
                    float *save, float *coef, uint16_t *y, uint8_t *mask, hipStream_t s)
{
    hipLaunchKernelGGL(k_bn_finish, dim3(C), dim3(kBlock), 0, s, nullptr, part, nblk, C, rows, gamma, beta, rm, rv,
                       momentum, eps, save, coef);
    const dim3 g(apply_blocks(rows, C));
    if (relu && res)
        launch_apply<C, true, true>(g, s, x, res, rows, coef, y, mask);
    else if (relu)
        launch_apply<C, true, false>(g, s, x, res, rows, coef, y, mask);
    else if (res)
        launch_apply<C, false, true>(g, s, x, res, rows, coef, y, mask);
    else
        launch_apply<C, false, false>(g, s, x, res, rows, coef, y, mask);
    return launched("k_bn_apply");
}

template <int C, bool RELU, bool MASK>
void launch_bwd(int nb, dim3 g, hipStream_t s, const uint16_t *dy, const uint16_t *y, const uint8_t *mask,
                const uint16_t *x, int64_t rows, const float *gamma, const float *save, float *ws, float *coef,
                uint16_t *dx, uint16_t *dres, float *dgamma, float *dbeta)
{
    hipLaunchKernelGGL((k_bn_bwd_reduce<C, RELU, MASK>), dim3(nb), dim3(kBlock), 0, s, dy, y, mask, x, rows, save, ws);
    hipLaunchKernelGGL(k_bn_bwd_finish, dim3(C), dim3(kBlock), 0, s, ws, nb, C, rows, gamma, save, dgamma, dbeta, coef);
    if (dres)
        hipLaunchKernelGGL((k_bn_bwd_apply<C, RELU, true, MASK>), g, dim3(kBlock), 0, s, dy, y, mask, x, rows, coef, dx,
                           dres);
    else
        hipLaunchKernelGGL((k_bn_bwd_apply<C, RELU, false, MASK>), g, dim3(kBlock), 0, s, dy, y, mask, x, rows, coef,
                           dx, dres);
}

// finish + apply from per-block sums a producer computed (r48_conv3x3_bn_grad)
template <int C>
int backward_part_c(const float *part, int nblk, const uint16_t *dy, const uint8_t *mask, const uint16_t *x,
                    int64_t rows, const float *gamma, const float *save, float *coef, uint16_t *dx, uint16_t *dres,
                    float *dgamma, float *dbeta, hipStream_t s)
{
    hipLaunchKernelGGL(k_bn_bwd_finish, dim3(C), dim3(kBlock), 0, s, part, nblk, C, rows, gamma, save, dgamma, dbeta,
                       coef);
    const dim3 g(apply_blocks(rows, C));
    const uint16_t *y = nullptr;
    if (dres)
        hipLaunchKernelGGL((k_bn_bwd_apply<C, true, true, true>), g, dim3(kBlock), 0, s, dy, y, mask, x, rows, coef,
                           dx, dres);
    else
        hipLaunchKernelGGL((k_bn_bwd_apply<C, true, false, true>), g, dim3(kBlock), 0, s, dy, y, mask, x, rows, coef,
                           dx, dres);
    return launched("k_bn_bwd_apply");
}

template <int C>
int backward_c(const uint16_t *dy, const uint16_t *y, const uint8_t *mask, const uint16_t *x, int64_t rows,
               const float *gamma, const float *save, int relu, float *ws, uint16_t *dx, uint16_t *dres,
               float *dgamma, float *dbeta, hipStream_t s)
{
    const int nb = reduce_blocks(rows, C);
    float *coef = ws + (int64_t)nb * 2 * C;
    const dim3 g(apply_blocks(rows, C));
    if (relu && mask)
        launch_bwd<C, true, true>(nb, g, s, dy, y, mask, x, rows, gamma, save, ws, coef, dx, dres, dgamma, dbeta);
    else if (relu)
        launch_bwd<C, true, false>(nb, g, s, dy, y, mask, x, rows, gamma, save, ws, coef, dx, dres, dgamma, dbeta);
    else
        launch_bwd<C, false, false>(nb, g, s, dy, y, mask, x, rows, gamma, save, ws, coef, dx, dres, dgamma, dbeta);
    return launched("k_bn_bwd_apply");
}

}  // namespace

extern "C" {

int64_t r48_bn_workspace_floats(int64_t rows, int32_t C)
{
    if (rows < 1 || C < 8)
        return 0;
    return (int64_t)reduce_blocks(rows, C) * 2 * C + 3 * (int64_t)C;
}

int r48_bn_forward(const void *x, const void *residual, int64_t rows, int32_t C, const float *gamma,
                   const float *beta, float *running_mean, float *running_var, float momentum, float eps,
                   int32_t relu, float *save, float *workspace, void *y, uint8_t *mask, void *stream)
{
    int rc = check_args(x, rows, C);
    if (rc)
        return rc;
    if (!gamma || !beta || !save || !workspace || !y || !aligned16(y) || (residual && !aligned16(residual)))
        return fail(R48_EINVAL, "r48_bn_forward: null or misaligned argument");
    if ((running_mean == nullptr) != (running_var == nullptr))
        return fail(R48_EINVAL, "r48_bn_forward: running_mean and running_var go together");
    const uint16_t *xs = (const uint16_t *)x, *rs = (const uint16_t *)residual;
    hipStream_t s = (hipStream_t)stream;
    switch (C) {
    case 32:
        return forward_c<32>(xs, rs, rows, gamma, beta, running_mean, running_var, momentum, eps, relu, save,
                             workspace, (uint16_t *)y, mask, s);
    case 64:
        return forward_c<64>(xs, rs, rows, gamma, beta, running_mean, running_var, momentum, eps, relu, save,
                             workspace, (uint16_t *)y, mask, s);
    default:
        return forward_c<128>(xs, rs, rows, gamma, beta, running_mean, running_var, momentum, eps, relu, save,
                              workspace, (uint16_t *)y, mask, s);
    }
}

int r48_bn_forward_stats(const float *part, int32_t nblk, const void *x, const void *residual, int64_t rows, int32_t C,
                         const float *gamma, const float *beta, float *running_mean, float *running_var,
                         float momentum, float eps, int32_t relu, float *save, float *workspace, void *y, uint8_t *mask,
                         void *stream)
{
    int rc = check_args(x, rows, C);
    if (rc)
        return rc;
    if (!part || nblk < 1 || !gamma || !beta || !save || !workspace || !y || !aligned16(y) ||
        (residual && !aligned16(residual)))
        return fail(R48_EINVAL, "r48_bn_forward_stats: null or misaligned argument");
    if ((running_mean == nullptr) != (running_var == nullptr))
        return fail(R48_EINVAL, "r48_bn_forward_stats: running_mean and running_var go together");
    const uint16_t *xs = (const uint16_t *)x, *rs = (const uint16_t *)residual;
    hipStream_t s = (hipStream_t)stream;
    float *coef = workspace + (int64_t)reduce_blocks(rows, C) * 2 * C;
    switch (C) {
    case 32:
        return forward_stats_c<32>(part, nblk, xs, rs, rows, gamma, beta, running_mean, running_var, momentum, eps,
                                   relu, save, coef, (uint16_t *)y, mask, s);
    case 64:
        return forward_stats_c<64>(part, nblk, xs, rs, rows, gamma, beta, running_mean, running_var, momentum, eps,
                                   relu, save, coef, (uint16_t *)y, mask, s);
    default:
        return forward_stats_c<128>(part, nblk, xs, rs, rows, gamma, beta, running_mean, running_var, momentum, eps,
                                    relu, save, coef, (uint16_t *)y, mask, s);
    }
}

int r48_bn_finish(const float *part, int32_t nblk, int64_t rows, int32_t C, const float *gamma, const float *beta,
                  float *running_mean, float *running_var, float momentum, float eps, float *save, float *coef,
                  void *stream)
{
    if (!part || nblk < 1 || rows < 1 || (C != 32 && C != 64 && C != 128) || !gamma || !beta || !save || !coef)
        return fail(R48_EINVAL, "r48_bn_finish: null argument, rows < 1 or C not 32/64/128");
    if ((running_mean == nullptr) != (running_var == nullptr))
        return fail(R48_EINVAL, "r48_bn_finish: running_mean and running_var go together");
    hipLaunchKernelGGL(k_bn_finish, dim3(C), dim3(kBlock), 0, (hipStream_t)stream, nullptr, part, nblk, C, rows, gamma,
                       beta, running_mean, running_var, momentum, eps, save, coef);
    return launched("k_bn_finish");
}

int r48_bn_backward_part(const float *part, int32_t nblk, const void *dy, const uint8_t *mask, const void *x,
                         int64_t rows, int32_t C, const float *gamma, const float *save, float *workspace, void *dx,
                         void *dresidual, float *dgamma, float *dbeta, void *stream)
{
    int rc = check_args(x, rows, C);
    if (rc)
        return rc;
    if (!part || nblk < 1 || !dy || !aligned16(dy) || !mask || !gamma || !save || !workspace || !dx ||
        !aligned16(dx) || (dresidual && !aligned16(dresidual)))
        return fail(R48_EINVAL, "r48_bn_backward_part: null or misaligned argument");
    const uint16_t *d = (const uint16_t *)dy, *xs = (const uint16_t *)x;
    hipStream_t s = (hipStream_t)stream;
    float *coef = workspace + (int64_t)reduce_blocks(rows, C) * 2 * C;
    switch (C) {
    case 32:
        return backward_part_c<32>(part, nblk, d, mask, xs, rows, gamma, save, coef, (uint16_t *)dx,
                                   (uint16_t *)dresidual, dgamma, dbeta, s);
    case 64:
        return backward_part_c<64>(part, nblk, d, mask, xs, rows, gamma, save, coef, (uint16_t *)dx,
                                   (uint16_t *)dresidual, dgamma, dbeta, s);
    default:
        return backward_part_c<128>(part, nblk, d, mask, xs, rows, gamma, save, coef, (uint16_t *)dx,
                                    (uint16_t *)dresidual, dgamma, dbeta, s);
    }
}

int r48_bn_apply(const void *x, const void *residual, int64_t rows, int32_t C, const float *coef, int32_t relu, void *y,
                 uint8_t *mask, void *stream)
{
    int rc = check_args(x, rows, C);
    if (rc)
        return rc;
    if (!coef || !y || !aligned16(y) || (residual && !aligned16(residual)))
        return fail(R48_EINVAL, "r48_bn_apply: null or misaligned argument");
    const uint16_t *xs = (const uint16_t *)x, *rs = (const uint16_t *)residual;
    uint16_t *ys = (uint16_t *)y;
    hipStream_t s = (hipStream_t)stream;
    switch (C) {
    case 32:
        return apply_c<32>(xs, rs, rows, coef, relu, ys, mask, s);
    case 64:
        return apply_c<64>(xs, rs, rows, coef, relu, ys, mask, s);
    default:
        return apply_c<128>(xs, rs, rows, coef, relu, ys, mask, s);
    }
}

int r48_bn_backward_apply(const void *dy, const uint8_t *mask, const void *x, int64_t rows, int32_t C, const float *coef,
                          void *dx, void *stream)
{
    int rc = check_args(x, rows, C);
    if (rc)
        return rc;
    if (!dy || !aligned16(dy) || !mask || !coef || !dx || !aligned16(dx))
        return fail(R48_EINVAL, "r48_bn_backward_apply: null or misaligned argument");
    const uint16_t *d = (const uint16_t *)dy, *xs = (const uint16_t *)x, *y = nullptr;
    uint16_t *o = (uint16_t *)dx;
    hipStream_t s = (hipStream_t)stream;
    switch (C) {
    case 32:
        hipLaunchKernelGGL((k_bn_bwd_apply<32, true, false, true>), dim3(apply_blocks(rows, 32)), dim3(kBlock), 0, s, d,
                           y, mask, xs, rows, coef, o, nullptr);
        break;
    case 64:
        hipLaunchKernelGGL((k_bn_bwd_apply<64, true, false, true>), dim3(apply_blocks(rows, 64)), dim3(kBlock), 0, s, d,
                           y, mask, xs, rows, coef, o, nullptr);
        break;
    default:
        hipLaunchKernelGGL((k_bn_bwd_apply<128, true, false, true>), dim3(apply_blocks(rows, 128)), dim3(kBlock), 0, s,
                           d, y, mask, xs, rows, coef, o, nullptr);
    }
    return launched("k_bn_bwd_apply");
}

int r48_bn_backward(const void *dy, const void *y, const uint8_t *mask, const void *x, int64_t rows, int32_t C,
                    const float *gamma, const float *save, int32_t relu, float *workspace, void *dx, void *dresidual,
                    float *dgamma, float *dbeta, void *stream)
{
    int rc = check_args(x, rows, C);
    if (rc)
        return rc;
    if (!dy || !aligned16(dy) || !gamma || !save || !workspace || !dx || !aligned16(dx) ||
        (relu && !mask && (!y || !aligned16(y))) || (dresidual && !aligned16(dresidual)))
        return fail(R48_EINVAL, "r48_bn_backward: null or misaligned argument");
    const uint16_t *d = (const uint16_t *)dy, *ys = (const uint16_t *)y, *xs = (const uint16_t *)x;
    hipStream_t s = (hipStream_t)stream;
    switch (C) {
    case 32:
        return backward_c<32>(d, ys, mask, xs, rows, gamma, save, relu, workspace, (uint16_t *)dx,
                              (uint16_t *)dresidual, dgamma, dbeta, s);
    case 64:
        return backward_c<64>(d, ys, mask, xs, rows, gamma, save, relu, workspace, (uint16_t *)dx,
                              (uint16_t *)dresidual, dgamma, dbeta, s);
    default:
        return backward_c<128>(d, ys, mask, xs, rows, gamma, save, relu, workspace, (uint16_t *)dx,
                               (uint16_t *)dresidual, dgamma, dbeta, s);
    }
}

}  // extern "C"
