// r48_conv.hip -- the 3x3 (pad 1) convolutions of the ResNet-10 Q-network's UPDATE on the 4x4 grid
// (BASELINE config 5; rein48_amd/dqn/nets.py), hand-written for gfx950 MFMA, behind include/rein48.h.
//
// Activations are channels-last bf16 [boards][16 cells][C]. Only the 100 in-grid (cell, tap) pairs
// of the 144 are computed (the dense structured GEMM of the PyTorch path does 1.44x their work at
// 64 channels and reads/writes the same bytes through hipBLASLt).
//
// k_conv3x3 (forward, and the data gradient: the same kernel with the flipped, transposed taps)
//   v_mfma_f32_16x16x32_bf16, rows = 16 output channels (row tile O of 4), columns = 16 BOARDS at
//   the same cell (the layout of the inference kernel r48_resnet.hip): a wave loads all 16 cells of
//   its 16 boards (16-byte chunks, lane = board l & 15, channel group g = l >> 4) and the 3x3 tap
//   (dr, dc) of output cell p is just the input cell p + 4dr + dc of the same lane -- no lane
//   movement; one LDS weight fragment (tap, O, k-chunk) feeds every cell that has the tap (9, 12
//   or 16 MFMAs). Accumulators start at the bias; a finished row tile stores 4 channels (8 B) per
//   lane and cell. Weights: 9 x 4 x NC fragments of 1 KiB in LDS (72 KiB at 64 input channels),
//   two workgroups of 4 waves per CU.
// k_conv_wgrad (weight gradient, summed over boards and cells)
//   dW[t][co][ci] = sum over (board, cell p in grid for t) of dy[b][p][co] x[b][p + off(t)][ci]:
//   a contraction over rows, so rows go to the MFMA K dimension through LDS images read back with
//   ds_read_b64_tr_b16. Per step a workgroup stages 4 boards (64 rows) of dy and x (double-buffered
//   images, the global loads two steps ahead in registers); the x operand of tap t is the same image
//   read with per-lane row addresses shifted by the tap (rows outside the grid point at a zero row).
//   Wave w owns input-channel tile (16 channels) w for every tap and output tile: 36 accumulators of
//   16x16 (AGPRs). Each workgroup writes one fp32 record; k_conv_wgrad_reduce sums the records in a
//   fixed order (deterministic).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/rein48.h"

namespace r48 {
void set_last_error(const std::string &msg);
}

namespace {

using bf16x8 = __attribute__((ext_vector_type(8))) short;
using f32x4 = __attribute__((ext_vector_type(4))) float;
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
#define R48_LDS __attribute__((address_space(3)))

constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kCout = 64;

// tap t = 3 (dr + 1) + (dc + 1); centre first (all 16 cells: it starts every accumulator)
__device__ constexpr int kTapOrder[9] = {4, 0, 1, 2, 3, 5, 6, 7, 8};

__host__ __device__ constexpr bool in_grid(int p, int t)
{
    const int r = (p >> 2) + t / 3 - 1, c = (p & 3) + t % 3 - 1;
    return r >= 0 && r < 4 && c >= 0 && c < 4;
}
__host__ __device__ constexpr int tap_off(int t) { return 4 * (t / 3 - 1) + (t % 3 - 1); }

__device__ __forceinline__ bf16x8 as_frag(const uint4 &v) { return __builtin_bit_cast(bf16x8, v); }

__device__ __forceinline__ uint32_t pack2(float lo, float hi)
{
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2{lo, hi}), bf16x2_t));
}

int fail(int code, const std::string &msg)
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

int cu_count()
{
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return cus;
}

// ---------------------------------------------------------------------------------- forward
// x bf16 [boards][16][32 NC], wfrag (tap, O, c) fragments: lane l element j = W[16 O + (l & 15)]
// [32 c + 8 (l >> 4) + j][tap] (rein48_amd/dqn/conv.py pack_conv), bias fp32 [64] or null,
// y bf16 [boards][16][64].
template <int NC>
__global__ __launch_bounds__(kThreads, 2) void k_conv3x3(const uint16_t *__restrict__ x, int64_t boards,
                                                        const uint4 *__restrict__ wfrag,
                                                        const float *__restrict__ bias, uint16_t *__restrict__ y)
{
    constexpr int kFrags = 9 * 4 * NC;
    constexpr int kCin = 32 * NC;
    __shared__ uint4 w_lds[kFrags * 64];
    __shared__ __attribute__((aligned(16))) float b_lds[kCout];
    for (int i = threadIdx.x; i < kFrags * 64; i += kThreads)
        w_lds[i] = wfrag[i];
    if (threadIdx.x < kCout)
        b_lds[threadIdx.x] = bias ? bias[threadIdx.x] : 0.0f;
    __syncthreads();
    const int lane = threadIdx.x & 63, n = lane & 15, g = lane >> 4;
    const int wave = threadIdx.x >> 6;
    const int64_t n_tiles = (boards + 15) / 16;
    const int64_t stride = (int64_t)gridDim.x * kWaves;
    for (int64_t tile = (int64_t)blockIdx.x * kWaves + wave; tile < n_tiles; tile += stride) {
        const int64_t b = tile * 16 + n;
        const bool live = b < boards;
        const int64_t bb = live ? b : boards - 1;
        // all 16 cells of this lane's board, input channels 32 c + 8 g .. + 7 per chunk c
        uint4 xv[16][NC];
        const uint16_t *xr = x + bb * 16 * kCin + 8 * g;
#pragma unroll
        for (int q = 0; q < 16; q++)
#pragma unroll
            for (int c = 0; c < NC; c++)
                xv[q][c] = *reinterpret_cast<const uint4 *>(xr + q * kCin + 32 * c);
        uint16_t *yr = y + bb * 16 * kCout + 4 * g;
#pragma unroll
        for (int O = 0; O < 4; O++) {
            const f32x4 b4 = *reinterpret_cast<const f32x4 *>(b_lds + 16 * O + 4 * g);
            f32x4 acc[16];
#pragma unroll
            for (int k = 0; k < 9 * NC; k++) {
                const int t = kTapOrder[k / NC], c = k % NC;
                const bf16x8 A = as_frag(w_lds[((t * 4 + O) * NC + c) * 64 + lane]);
#pragma unroll
                for (int p = 0; p < 16; p++) {
                    if (!in_grid(p, t))
                        continue;
                    acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, as_frag(xv[p + tap_off(t)][c]),
                                                                     k == 0 ? b4 : acc[p], 0, 0, 0);
                }
            }
            if (live) {
#pragma unroll
                for (int p = 0; p < 16; p++)
                    *reinterpret_cast<uint2 *>(yr + p * kCout + 16 * O) =
                        make_uint2(pack2(acc[p][0], acc[p][1]), pack2(acc[p][2], acc[p][3]));
            }
        }
    }
}

// --------------------------------------------------------------------------------- wgrad
// Per step a workgroup stages kStepRows rows (kStepRows / 16 boards) of dy [rows][64] and x
// [rows][CIN] into LDS images (row-major, the 16-byte chunk index XOR-ed with the row so the
// staging stores are conflict free), plus one zero row per image. The global loads of step s + 2
// are issued while step s computes (a two-step register ring), so a workgroup keeps ~32 KB in flight.
constexpr int kStepRows = 64;
constexpr int kKSteps = kStepRows / 32;

template <int COLS>
__device__ __forceinline__ int wimg(int row, int col)
{
    constexpr int kChunks = COLS / 8;
    return row * COLS + ((((col >> 3) ^ row) & (kChunks - 1)) << 3) + (col & 7);
}

__device__ __forceinline__ bf16x8 tr_pair(const uint16_t *p0, const uint16_t *p1)
{
    const i16x4 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((R48_LDS i16x4 *)(p0));
    const i16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((R48_LDS i16x4 *)(p1));
    bf16x8 f;
    __builtin_memcpy(&f, &r0, 8);
    __builtin_memcpy(reinterpret_cast<char *>(&f) + 8, &r1, 8);
    return f;
}

// gradient accumulation in AGPRs; operands straight from LDS reads (no VALU wait states needed)
__device__ __forceinline__ void acc16(f32x4 &acc, const bf16x8 &a, const bf16x8 &b)
{
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// partial record per workgroup: [9 taps][64 co][CIN ci] fp32
template <int CIN>
__global__ __launch_bounds__(kThreads, 1) void k_conv_wgrad(const uint16_t *__restrict__ dy,
                                                           const uint16_t *__restrict__ x, int64_t boards,
                                                           float *__restrict__ partials)
{
    constexpr int NCT = CIN / 16;                                // input-channel tiles of 16
    constexpr int kCoT = NCT >= kWaves ? 4 : 4 * NCT / kWaves;   // output tiles per wave (4 or 2)
    constexpr int kDyImg = (kStepRows + 1) * kCout, kXImg = (kStepRows + 1) * CIN;
    constexpr int kBuf = kDyImg + kXImg;
    constexpr int kDyChunks = kStepRows * kCout / 8, kXChunks = kStepRows * CIN / 8;
    constexpr int kPerThread = (kDyChunks + kXChunks) / kThreads;   // 16-byte chunks per thread per step
    static_assert((kDyChunks + kXChunks) % kThreads == 0 && kDyChunks % kThreads == 0, "staging split");
    __shared__ __attribute__((aligned(16))) uint16_t lds[2 * kBuf];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i16 = lane & 15, g = lane >> 4;
    const int ct = NCT >= kWaves ? wave : wave % NCT;            // input-channel tile of this wave
    const int cot0 = NCT >= kWaves ? 0 : (wave / NCT) * kCoT;    // first output tile of this wave
    for (int i = threadIdx.x; i < kCout; i += kThreads) {        // zero rows (never overwritten)
        lds[kStepRows * kCout + i] = 0;
        lds[kBuf + kStepRows * kCout + i] = 0;
    }
    for (int i = threadIdx.x; i < CIN; i += kThreads) {
        lds[kDyImg + kStepRows * CIN + i] = 0;
        lds[kBuf + kDyImg + kStepRows * CIN + i] = 0;
    }
    // transposed-read addresses. A (dy^T, lanes = co) of k-step ks: rows 32 ks + 8g + 4u + q,
    // columns 16 cot + 4p (lane 4q + p of a 16-lane group addresses row q of the group's 4-row
    // block). B (x^T shifted by tap t, lanes = ci): row + off(t) when that cell is in the grid,
    // else the zero row.
    const int q = i16 >> 2, p4 = i16 & 3;
    int a_off[kKSteps][kCoT][2], b_off[kKSteps][9][2];
#pragma unroll
    for (int ks = 0; ks < kKSteps; ks++)
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int row = 32 * ks + 8 * g + 4 * u + q;
#pragma unroll
            for (int j = 0; j < kCoT; j++)
                a_off[ks][j][u] = wimg<kCout>(row, 16 * (cot0 + j) + 4 * p4);
#pragma unroll
            for (int t = 0; t < 9; t++) {
                const int src = in_grid(row & 15, t) ? row + tap_off(t) : kStepRows;
                b_off[ks][t][u] = kDyImg + wimg<CIN>(src, 16 * ct + 4 * p4);
            }
        }
    f32x4 acc[9][kCoT];
#pragma unroll
    for (int t = 0; t < 9; t++)
#pragma unroll
        for (int j = 0; j < kCoT; j++)
            acc[t][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // this workgroup's steps: a contiguous range
    const int64_t rows_total = boards * 16;
    const int64_t steps_total = (rows_total + kStepRows - 1) / kStepRows;
    const int64_t per = (steps_total + gridDim.x - 1) / gridDim.x;
    const int64_t s0 = (int64_t)blockIdx.x * per, s1 = s0 + per < steps_total ? s0 + per : steps_total;
    // chunk c of a step: c < kDyChunks -> dy row c / 8, 16-byte column c % 8; else x
    auto load = [&](int64_t step, uint4 (&v)[kPerThread]) {
#pragma unroll
        for (int k = 0; k < kPerThread; k++) {
            const int c = threadIdx.x + k * kThreads;
            const bool is_dy = c < kDyChunks;
            const int cc = is_dy ? c : c - kDyChunks, cols = is_dy ? kCout : CIN;
            const int r = cc / (cols / 8), ch = cc % (cols / 8);
            const int64_t row = step * kStepRows + r;
            v[k] = make_uint4(0, 0, 0, 0);
            if (step < s1 && row < rows_total)
                v[k] = *reinterpret_cast<const uint4 *>((is_dy ? dy : x) + row * cols + 8 * ch);
        }
    };
    auto store = [&](const uint4 (&v)[kPerThread], int buf) {
        uint16_t *dimg = lds + buf * kBuf, *ximg = dimg + kDyImg;
#pragma unroll
        for (int k = 0; k < kPerThread; k++) {
            const int c = threadIdx.x + k * kThreads;
            if (c < kDyChunks)
                *reinterpret_cast<uint4 *>(dimg + wimg<kCout>(c / (kCout / 8), 8 * (c % (kCout / 8)))) = v[k];
            else
                *reinterpret_cast<uint4 *>(ximg + wimg<CIN>((c - kDyChunks) / (CIN / 8),
                                                            8 * ((c - kDyChunks) % (CIN / 8)))) = v[k];
        }
    };
    uint4 ra[kPerThread], rb[kPerThread];
    load(s0, ra);
    load(s0 + 1, rb);
    store(ra, 0);
    __syncthreads();
    for (int64_t s = s0; s < s1; s++) {
        const int buf = (int)((s - s0) & 1);
        // ring: rb holds step s + 1; ra is free -> step s + 2
        load(s + 2, ra);
        const uint16_t *img = lds + buf * kBuf;
#pragma unroll
        for (int ks = 0; ks < kKSteps; ks++) {
            bf16x8 A[kCoT];
#pragma unroll
            for (int j = 0; j < kCoT; j++)
                A[j] = tr_pair(img + a_off[ks][j][0], img + a_off[ks][j][1]);
#pragma unroll
            for (int t = 0; t < 9; t++) {
                const bf16x8 B = tr_pair(img + b_off[ks][t][0], img + b_off[ks][t][1]);
#pragma unroll
                for (int j = 0; j < kCoT; j++)
                    acc16(acc[t][j], A[j], B);
            }
        }
        store(rb, buf ^ 1);      // step s + 1 into the other buffer (its readers passed the last barrier)
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kPerThread; k++)
            rb[k] = ra[k];
    }
    // record: D[m = co 16][n = ci 16], lane l: column i16 (ci), rows 4g + i (co). 24 wait states
    // between the last accumulating MFMA and the AGPR reads
    asm volatile("s_nop 15\n\ts_nop 7" ::: "memory");
    float *rec = partials + (int64_t)blockIdx.x * 9 * kCout * CIN;
#pragma unroll
    for (int t = 0; t < 9; t++)
#pragma unroll
        for (int j = 0; j < kCoT; j++)
#pragma unroll
            for (int i = 0; i < 4; i++)
                rec[(t * kCout + 16 * (cot0 + j) + 4 * g + i) * CIN + 16 * ct + i16] = acc[t][j][i];
}

// out[co][ci][t] (torch's [co, ci, 3, 3] layout) = fixed-order sum over the records [t][co][ci]
template <int CIN>
__global__ __launch_bounds__(256) void k_conv_wgrad_reduce(const float *__restrict__ partials, int n_rec,
                                                          float *__restrict__ out)
{
    const int k = blockIdx.x * 256 + threadIdx.x;      // record index: (t * 64 + co) * CIN + ci
    if (k >= 9 * kCout * CIN)
        return;
    float s = 0.f;
    for (int r = 0; r < n_rec; r++)
        s += partials[(int64_t)r * 9 * kCout * CIN + k];
    const int t = k / (kCout * CIN), co = (k / CIN) % kCout, ci = k % CIN;
    out[(co * CIN + ci) * 9 + t] = s;
}

// one lane per (board, cell): the one-hot of the exponent over 32 bf16 planes (e = 0..17, planes
// 18..31 zero: the stem's input channels padded to one 32-channel k-chunk), four 16-byte stores
__global__ __launch_bounds__(256) void k_onehot32(const int8_t *__restrict__ boards, int64_t n_cells,
                                                 uint4 *__restrict__ out)
{
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= n_cells)
        return;
    const uint32_t e = (uint32_t)(uint8_t)boards[c];
    uint32_t w[16];
#pragma unroll
    for (int k = 0; k < 16; k++)
        w[k] = (e == 2u * k ? 0x3F80u : 0u) | (e == 2u * k + 1u ? 0x3F800000u : 0u);
#pragma unroll
    for (int k = 0; k < 4; k++)
        out[4 * c + k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
}

}  // namespace

extern "C" {

int r48_board_onehot32(const int8_t *boards, int64_t n, void *out, void *stream)
{
    if (!boards || !out || n < 0 || (reinterpret_cast<uintptr_t>(out) & 15u))
        return fail(R48_EINVAL, "r48_board_onehot32: NULL argument, n < 0 or out not 16-byte aligned");
    if (n == 0)
        return R48_OK;
    const int64_t cells = 16 * n;
    hipLaunchKernelGGL(k_onehot32, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, (hipStream_t)stream, boards,
                       cells, (uint4 *)out);
    return launched("k_onehot32");
}

int r48_conv3x3(const void *x, int64_t boards, int32_t cin, const void *wfrag, const float *bias, void *y,
                void *stream)
{
    if (!x || !wfrag || !y || boards < 1 || (cin != 32 && cin != 64))
        return fail(R48_EINVAL, "r48_conv3x3: NULL argument, boards < 1 or cin not 32/64");
    if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(wfrag) | reinterpret_cast<uintptr_t>(y) |
         reinterpret_cast<uintptr_t>(bias)) & 15u)
        return fail(R48_EINVAL, "r48_conv3x3: x, wfrag, bias and y must be 16-byte aligned");
    const int64_t tiles = (boards + 15) / 16;
    const int64_t want = (tiles + kWaves - 1) / kWaves;
    const int grid = (int)(want < 2 * cu_count() ? want : 2 * cu_count());
    if (cin == 64)
        hipLaunchKernelGGL(k_conv3x3<2>, dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, (const uint16_t *)x,
                           boards, (const uint4 *)wfrag, bias, (uint16_t *)y);
    else
        hipLaunchKernelGGL(k_conv3x3<1>, dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, (const uint16_t *)x,
                           boards, (const uint4 *)wfrag, bias, (uint16_t *)y);
    return launched("k_conv3x3");
}

int64_t r48_conv_wgrad_workspace_floats(int32_t cin)
{
    return (int64_t)cu_count() * 9 * kCout * (cin == 32 ? 32 : 64);
}

int r48_conv3x3_wgrad(const void *dy, const void *x, int64_t boards, int32_t cin, float *workspace, float *dw,
                      void *stream)
{
    if (!dy || !x || !workspace || !dw || boards < 1 || (cin != 32 && cin != 64))
        return fail(R48_EINVAL, "r48_conv3x3_wgrad: NULL argument, boards < 1 or cin not 32/64");
    if ((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(x)) & 15u)
        return fail(R48_EINVAL, "r48_conv3x3_wgrad: dy and x must be 16-byte aligned");
    const int grid = cu_count();
    const int n_out = 9 * kCout * cin;
    if (cin == 64) {
        hipLaunchKernelGGL(k_conv_wgrad<64>, dim3(grid), dim3(kThreads), 0, (hipStream_t)stream,
                           (const uint16_t *)dy, (const uint16_t *)x, boards, workspace);
        hipLaunchKernelGGL(k_conv_wgrad_reduce<64>, dim3((n_out + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                           workspace, grid, dw);
    } else {
        hipLaunchKernelGGL(k_conv_wgrad<32>, dim3(grid), dim3(kThreads), 0, (hipStream_t)stream,
                           (const uint16_t *)dy, (const uint16_t *)x, boards, workspace);
        hipLaunchKernelGGL(k_conv_wgrad_reduce<32>, dim3((n_out + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                           workspace, grid, dw);
    }
    return launched("k_conv_wgrad");
}

}  // extern "C"
