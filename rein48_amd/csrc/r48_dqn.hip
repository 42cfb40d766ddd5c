// r48_dqn.hip -- gfx950 kernels around the env step for value-based training (BASELINE
// config 5: ResNet-10 Q-network, DQN replay resident in HBM), behind include/rein48.h.
//
//   k_onehot    board int8[16] -> bf16/f32 [16 positions][18 planes] one-hot of the exponent
//               (e = 0..17; the largest tile a 4x4 board can hold is 2^17). Position-major,
//               plane-minor: the layout the structured-GEMM stem and the fused kernel read.
//   k_egreedy   epsilon-greedy over Q float[n][4]: u < eps -> uniform action, else the first
//               argmax (np.argmax tie rule). Philox4x32-10(key = seed, counter = {gid lo,
//               gid hi, ctr, 0xD0E}): u = (w0 >> 8) / 2^24, random action = w1 >> 30.
//   k_td_target y = r + gamma * (1 - done) * Q'(s', a*), a* = argmax_a Q'(s') (DQN) or
//               argmax_a Q(s') of the online net (double DQN); fp32.
// All are memory-bound one-row-per-lane kernels.
#include <hip/hip_runtime.h>

#include <cmath>

#include <cstdint>
#include <string>

#include "../../include/rein48.h"
#include "r48_board.h"

namespace r48 {
void set_last_error(const std::string &msg);
}

namespace {

constexpr int kBlock = 256;
constexpr uint32_t kEgreedyTag = 0xD0Eu;
constexpr int kPlanes = 18;

inline dim3 grid_for(int64_t n) { return dim3((unsigned)((n + kBlock - 1) / kBlock)); }

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

// one lane per (board, position): writes 18 values (36 B bf16 / 72 B f32)
template <typename T>
__global__ __launch_bounds__(kBlock) void k_onehot(const int8_t *__restrict__ boards, int64_t n_cells,
                                                   T *__restrict__ out)
{
    const int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (c >= n_cells)
        return;
    const uint32_t e = (uint32_t)(uint8_t)boards[c];
    T *o = out + kPlanes * c;
#pragma unroll
    for (int k = 0; k < kPlanes; ++k)
        o[k] = (T)(e == (uint32_t)k ? 1.0f : 0.0f);
}

__device__ __forceinline__ uint32_t argmax4(float4 q)
{
    uint32_t a = 0;
    float m = q.x;
    if (q.y > m) { m = q.y; a = 1; }
    if (q.z > m) { m = q.z; a = 2; }
    if (q.w > m) { a = 3; }
    return a;
}

__device__ __forceinline__ float pick(float4 q, uint32_t a)
{
    return a == 0 ? q.x : a == 1 ? q.y : a == 2 ? q.z : q.w;
}

__global__ __launch_bounds__(kBlock) void k_egreedy(const float *__restrict__ q, int64_t n, float eps, uint32_t k0,
                                                    uint32_t k1, int64_t gid0, uint32_t ctr,
                                                    int8_t *__restrict__ actions)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    const uint64_t gid = (uint64_t)(gid0 + i);
    uint32_t w[4] = {(uint32_t)gid, (uint32_t)(gid >> 32), ctr, kEgreedyTag};
    r48::philox4x32_10(w, k0, k1);
    const float u = (float)(w[0] >> 8) * (1.0f / 16777216.0f);
    const float4 qv = reinterpret_cast<const float4 *>(q)[i];
    actions[i] = (int8_t)(u < eps ? (w[1] >> 30) : argmax4(qv));
}

template <bool DOUBLE, bool LOG2>
__global__ __launch_bounds__(kBlock) void k_td_target(const float *__restrict__ reward,
                                                      const uint8_t *__restrict__ done,
                                                      const float *__restrict__ q_next_target,
                                                      const float *__restrict__ q_next_online, int64_t n,
                                                      float gamma, float *__restrict__ y)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    const float4 qt = reinterpret_cast<const float4 *>(q_next_target)[i];
    const uint32_t a = DOUBLE ? argmax4(reinterpret_cast<const float4 *>(q_next_online)[i]) : argmax4(qt);
    const float boot = (done && done[i]) ? 0.0f : pick(qt, a);
    const float r = LOG2 ? log2f(1.0f + reward[i]) : reward[i];   // trainer.py _reward, torch.log2(1.0 + r)
    y[i] = r + gamma * boot;
}

// ---- Huber loss of Q(s)[a] against the TD target and its gradient (DQNLearner.learn):
// d = q[i][a_i] - y_i; loss = mean(0.5 d^2 if |d| < 1 else |d| - 0.5) (smooth L1, beta 1);
// dq[i][a] = clamp(d, -1, 1) / n for a = a_i, else 0; also mean(q[i][a_i]). Per-block fp32 partials
// in a fixed grid and order, summed by one block (deterministic).
constexpr int kHuberBlocks = 256;

__global__ __launch_bounds__(kBlock) void k_huber_grad(const float *__restrict__ q, const int8_t *__restrict__ action,
                                                      const float *__restrict__ y, int64_t n, float *__restrict__ dq,
                                                      float *__restrict__ part)
{
    __shared__ float red[2][kBlock];
    float sl = 0.f, sq = 0.f;
    const float inv_n = 1.0f / (float)n;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        const float4 qi = reinterpret_cast<const float4 *>(q)[i];
        const int a = action[i] & 3;
        const float qa = pick(qi, (uint32_t)a);
        const float d = qa - y[i], ad = fabsf(d);
        sl += ad < 1.0f ? 0.5f * d * d : ad - 0.5f;
        sq += qa;
        const float g = fminf(fmaxf(d, -1.0f), 1.0f) * inv_n;
        reinterpret_cast<float4 *>(dq)[i] =
            make_float4(a == 0 ? g : 0.f, a == 1 ? g : 0.f, a == 2 ? g : 0.f, a == 3 ? g : 0.f);
    }
    red[0][threadIdx.x] = sl;
    red[1][threadIdx.x] = sq;
    __syncthreads();
    for (int h = kBlock / 2; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) {
            red[0][threadIdx.x] += red[0][threadIdx.x + h];
            red[1][threadIdx.x] += red[1][threadIdx.x + h];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = red[0][0];
        part[2 * blockIdx.x + 1] = red[1][0];
    }
}

// Adam over one flat fp32 parameter buffer, the update of torch.optim.Adam (eps outside the
// square root, bias corrections c1 = 1 - b1^t, c2 = 1 - b2^t): m = b1 m + (1 - b1) g,
// v = b2 v + (1 - b2) g^2, p -= (lr / c1) m / (sqrt(v / c2) + eps). One pass, 16-byte pieces;
// replaces the ~8 elementwise launches of trainer.Adam's torch form on the GPU.
__global__ __launch_bounds__(kBlock) void k_adam(float4 *__restrict__ p, const float4 *__restrict__ g,
                                               float4 *__restrict__ m, float4 *__restrict__ v, int64_t n4, float b1,
                                               float b2, float step_size, float c2, float eps)
{
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kBlock) {
        const float4 gi = g[i];
        float4 mi = m[i], vi = v[i], pi = p[i];
        float *mf = &mi.x, *vf = &vi.x, *pf = &pi.x;
        const float *gf = &gi.x;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            mf[k] = b1 * mf[k] + (1.0f - b1) * gf[k];
            vf[k] = b2 * vf[k] + (1.0f - b2) * gf[k] * gf[k];
            pf[k] -= step_size * (mf[k] / (sqrtf(vf[k] / c2) + eps));
        }
        m[i] = mi;
        v[i] = vi;
        p[i] = pi;
    }
}

__global__ __launch_bounds__(kBlock) void k_huber_finish(const float *__restrict__ part, int nblk, int64_t n,
                                                        float *__restrict__ out)
{
    __shared__ double red[2][kBlock];
    double s0 = 0.0, s1 = 0.0;
    for (int b = threadIdx.x; b < nblk; b += kBlock) {
        s0 += (double)part[2 * b];
        s1 += (double)part[2 * b + 1];
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
    if (threadIdx.x == 0) {
        out[0] = (float)(red[0][0] / (double)n);
        out[1] = (float)(red[1][0] / (double)n);
    }
}

// ---- structured 3x3 conv weight on the 4x4 grid (rein48_amd/dqn/nets.py dense_conv_weight)
// dense[P co + o][Q ci + i] = w[o][i][dr + 1][dc + 1] when input cell Q = P + 4 dr + dc is one of
// output cell P's in-grid 3x3 neighbours, else 0 (100 of the 256 (P, Q) blocks are nonzero). One
// thread writes 8 consecutive columns of one row; bf16 or f32 out (the zeros, the scatter and
// the cast of the PyTorch path in one pass).
__device__ __forceinline__ int tap_of(int P, int Q)
{
    const int dr = (Q >> 2) - (P >> 2), dc = (Q & 3) - (P & 3);
    return (dr < -1 || dr > 1 || dc < -1 || dc > 1) ? -1 : (dr + 1) * 3 + (dc + 1);
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_struct_weight(const float *__restrict__ w, int co, int ci,
                                                          T *__restrict__ dense)
{
    const int cols = 16 * ci, groups = cols / 8;
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= (int64_t)16 * co * groups)
        return;
    const int row = (int)(t / groups), c0 = (int)(t % groups) * 8;
    const int P = row / co, o = row % co;
    T out[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int col = c0 + k, Q = col / ci, i = col % ci;
        const int tap = tap_of(P, Q);
        out[k] = (T)(tap < 0 ? 0.0f : w[((int64_t)o * ci + i) * 9 + tap]);
    }
    __builtin_memcpy(dense + (int64_t)row * cols + c0, out, sizeof(out));
}

// gradient: gw[o][i][tap] = sum over the (P, Q) blocks of that tap of gd[P co + o][Q ci + i]
// (fixed block order: deterministic); gd bf16 or f32, gw f32. One thread per (o, i, tap), i fastest.
template <typename T>
__global__ __launch_bounds__(kBlock) void k_struct_weight_grad(const T *__restrict__ gd, int co, int ci,
                                                               float *__restrict__ gw)
{
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= (int64_t)9 * co * ci)
        return;
    const int i = (int)(t % ci), o = (int)((t / ci) % co), tap = (int)(t / ((int64_t)ci * co));
    const int dr = tap / 3 - 1, dc = tap % 3 - 1;
    const int64_t cols = 16 * (int64_t)ci;
    float s = 0.0f;
    for (int P = 0; P < 16; P++) {
        const int r = (P >> 2) + dr, c = (P & 3) + dc;
        if (r < 0 || r > 3 || c < 0 || c > 3)
            continue;
        const int Q = 4 * r + c;
        s += (float)gd[((int64_t)P * co + o) * cols + (int64_t)Q * ci + i];
    }
    gw[((int64_t)o * ci + i) * 9 + tap] = s;
}

bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

}  // namespace

extern "C" {

int r48_board_onehot(const int8_t *boards, int64_t n, int32_t out_dtype, void *out, void *stream)
{
    if (!boards || !out || n < 0 || (out_dtype != R48_F32 && out_dtype != R48_BF16))
        return fail(R48_EINVAL, "boards/out NULL, n < 0 or bad dtype");
    if (n == 0)
        return R48_OK;
    const int64_t cells = 16 * n;
    if (out_dtype == R48_F32)
        hipLaunchKernelGGL(k_onehot<float>, grid_for(cells), dim3(kBlock), 0, (hipStream_t)stream, boards, cells,
                           (float *)out);
    else
        hipLaunchKernelGGL(k_onehot<__bf16>, grid_for(cells), dim3(kBlock), 0, (hipStream_t)stream, boards, cells,
                           (__bf16 *)out);
    return launched("k_onehot");
}

int r48_egreedy_actions(const float *q, int64_t n, float eps, uint64_t seed, int64_t gid0, uint32_t ctr,
                        int8_t *actions, void *stream)
{
    if (!q || !actions || n < 0 || gid0 < 0 || !aligned16(q))
        return fail(R48_EINVAL, "q/actions NULL, q not 16-byte aligned, n < 0 or gid0 < 0");
    if (n == 0)
        return R48_OK;
    hipLaunchKernelGGL(k_egreedy, grid_for(n), dim3(kBlock), 0, (hipStream_t)stream, q, n, eps, (uint32_t)seed,
                       (uint32_t)(seed >> 32), gid0, ctr, actions);
    return launched("k_egreedy");
}

int r48_td_target(const float *reward, const uint8_t *done, const float *q_next_target,
                  const float *q_next_online, int64_t n, float gamma, int32_t log2_reward, float *y, void *stream)
{
    if (!reward || !q_next_target || !y || n < 0 || !aligned16(q_next_target) ||
        (q_next_online && !aligned16(q_next_online)))
        return fail(R48_EINVAL, "reward/q_next_target/y NULL, n < 0 or Q not 16-byte aligned");
    if (n == 0)
        return R48_OK;
    hipStream_t s = (hipStream_t)stream;
    if (q_next_online && log2_reward)
        hipLaunchKernelGGL((k_td_target<true, true>), grid_for(n), dim3(kBlock), 0, s, reward, done, q_next_target,
                           q_next_online, n, gamma, y);
    else if (q_next_online)
        hipLaunchKernelGGL((k_td_target<true, false>), grid_for(n), dim3(kBlock), 0, s, reward, done, q_next_target,
                           q_next_online, n, gamma, y);
    else if (log2_reward)
        hipLaunchKernelGGL((k_td_target<false, true>), grid_for(n), dim3(kBlock), 0, s, reward, done, q_next_target,
                           nullptr, n, gamma, y);
    else
        hipLaunchKernelGGL((k_td_target<false, false>), grid_for(n), dim3(kBlock), 0, s, reward, done, q_next_target,
                           nullptr, n, gamma, y);
    return launched("k_td_target");
}

int r48_struct_conv_weight(const float *w, int32_t co, int32_t ci, int32_t out_dtype, void *dense, void *stream)
{
    if (!w || !dense || co < 1 || ci < 1 || (16 * ci) % 8 || (out_dtype != R48_F32 && out_dtype != R48_BF16) ||
        !aligned16(dense))
        return fail(R48_EINVAL, "r48_struct_conv_weight: NULL/misaligned argument, bad dtype or 16 ci % 8 != 0");
    const int64_t threads = (int64_t)16 * co * (16 * ci / 8);
    if (out_dtype == R48_F32)
        hipLaunchKernelGGL(k_struct_weight<float>, grid_for(threads), dim3(kBlock), 0, (hipStream_t)stream, w, co, ci,
                           (float *)dense);
    else
        hipLaunchKernelGGL(k_struct_weight<__bf16>, grid_for(threads), dim3(kBlock), 0, (hipStream_t)stream, w, co,
                           ci, (__bf16 *)dense);
    return launched("k_struct_weight");
}

int r48_struct_conv_weight_grad(const void *gdense, int32_t co, int32_t ci, int32_t in_dtype, float *gw,
                                void *stream)
{
    if (!gdense || !gw || co < 1 || ci < 1 || (in_dtype != R48_F32 && in_dtype != R48_BF16))
        return fail(R48_EINVAL, "r48_struct_conv_weight_grad: NULL argument or bad dtype");
    const int64_t threads = (int64_t)9 * co * ci;
    if (in_dtype == R48_F32)
        hipLaunchKernelGGL(k_struct_weight_grad<float>, grid_for(threads), dim3(kBlock), 0, (hipStream_t)stream,
                           (const float *)gdense, co, ci, gw);
    else
        hipLaunchKernelGGL(k_struct_weight_grad<__bf16>, grid_for(threads), dim3(kBlock), 0, (hipStream_t)stream,
                           (const __bf16 *)gdense, co, ci, gw);
    return launched("k_struct_weight_grad");
}

int r48_huber_grad(const float *q, const int8_t *action, const float *y, int64_t n, float *dq, float *out,
                   float *workspace, void *stream)
{
    if (!q || !action || !y || !dq || !out || !workspace || n < 1 || !aligned16(q) || !aligned16(dq))
        return fail(R48_EINVAL, "r48_huber_grad: NULL argument, n < 1 or q/dq not 16-byte aligned");
    const int64_t want = (n + kBlock - 1) / kBlock;
    const int nb = (int)(want < kHuberBlocks ? want : kHuberBlocks);
    hipLaunchKernelGGL(k_huber_grad, dim3(nb), dim3(kBlock), 0, (hipStream_t)stream, q, action, y, n, dq, workspace);
    hipLaunchKernelGGL(k_huber_finish, dim3(1), dim3(kBlock), 0, (hipStream_t)stream, workspace, nb, n, out);
    return launched("k_huber_grad");
}

int r48_adam(float *param, const float *grad, float *m, float *v, int64_t n, float lr, float beta1, float beta2,
             float eps, int64_t step, void *stream)
{
    if (!param || !grad || !m || !v || n < 1 || n % 4 || step < 1 || !aligned16(param) || !aligned16(grad) ||
        !aligned16(m) || !aligned16(v))
        return fail(R48_EINVAL, "r48_adam: NULL argument, n < 1, n not a multiple of 4, step < 1 or a buffer not "
                                "16-byte aligned");
    const double c1 = 1.0 - std::pow((double)beta1, (double)step), c2 = 1.0 - std::pow((double)beta2, (double)step);
    const int64_t n4 = n / 4, want = (n4 + kBlock - 1) / kBlock;
    const int nb = (int)(want < 4096 ? want : 4096);
    hipLaunchKernelGGL(k_adam, dim3(nb), dim3(kBlock), 0, (hipStream_t)stream, reinterpret_cast<float4 *>(param),
                       reinterpret_cast<const float4 *>(grad), reinterpret_cast<float4 *>(m),
                       reinterpret_cast<float4 *>(v), n4, beta1, beta2, (float)(lr / c1), (float)c2, eps);
    return launched("k_adam");
}

}  // extern "C"

