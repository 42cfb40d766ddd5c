// r48_game.hip -- the drop-in single-board Game.step (nevertiree/Rein48 game/GameClient.py:40-51)
// as one gfx950 launch: the board travels in the kernel arguments and one wave evaluates the move
// and every spawn outcome, so the host's spawn draw (the global `random`, which must see the
// post-move blank count) needs no second launch or round trip (include/rein48.h r48_game_step1).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/rein48.h"
#include "r48_board.h"

namespace r48 {
void set_last_error(const std::string &msg);
}

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// out: [32][16] candidate boards, [512] changed, [513] blanks after the move, [516..519] game-over
// mask (bit l: candidate l is over).
constexpr int kStep1Out = 520;

// Lane l = 2r + f takes the move and then the spawn of tile 2 (f = 0) or 4 (f = 1) at blank rank r
// in the reference's row-major order (GameClient.py:109-114; step_board<.., RANK_IS_INDEX>) and
// has_game_over of the result (:74-93). Ranks >= the blank count repeat rank mod count (unused).
// An unchanged move spawns nothing (GameClient.py:49): every candidate is the unchanged board.
__global__ __launch_bounds__(64) void k_game_step1(u32x4 board, uint32_t action, uint8_t *__restrict__ out)
{
    const uint32_t l = threadIdx.x;
    r48::Board b{board.x, board.y, board.z, board.w};
    const r48::StepOut o = r48::step_board<false, true>(b, action, l >> 1, (l & 1u) != 0u);
    const unsigned long long over = __ballot(l < 32 && o.done);
    if (l < 32)
        *reinterpret_cast<u32x4 *>(out + 16 * l) = u32x4{b.w0, b.w1, b.w2, b.w3};
    if (l == 0) {
        out[512] = (uint8_t)o.changed;
        out[513] = (uint8_t)o.n_blank;
        *reinterpret_cast<uint32_t *>(out + 516) = (uint32_t)over;
    }
}

int fail(int code, const std::string &msg)
{
    r48::set_last_error(msg);
    return code;
}

}  // namespace

extern "C" {

int r48_game_step1(const int8_t *board, int32_t action, uint8_t *out, void *stream)
{
    if (!board || !out || action < 0 || action > 3)
        return fail(R48_EINVAL, "board/out NULL or action outside 0..3");
    if (reinterpret_cast<uintptr_t>(out) & 15u)
        return fail(R48_EINVAL, "out must be 16-byte aligned");
    for (int k = 0; k < 16; k++)
        if (board[k] < 0 || board[k] > 30)
            return fail(R48_EINVAL, "board cells must be exponents 0..30");
    u32x4 v;
    __builtin_memcpy(&v, board, 16);
    hipLaunchKernelGGL(k_game_step1, dim3(1), dim3(64), 0, (hipStream_t)stream, v, (uint32_t)action, out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(R48_EHIP, std::string("k_game_step1: ") + hipGetErrorString(e));
    return R48_OK;
}

int r48_game_step1_out_bytes(void) { return kStep1Out; }

void *r48_host_alloc(int64_t bytes, void **device_ptr)
{
    void *h = nullptr;
    if (bytes <= 0 || !device_ptr)
        return nullptr;
    if (hipHostMalloc(&h, (size_t)bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
        return nullptr;
    if (hipHostGetDevicePointer(device_ptr, h, 0) != hipSuccess) {
        (void)hipHostFree(h);
        return nullptr;
    }
    return h;
}

int r48_host_free(void *host_ptr)
{
    if (host_ptr && hipHostFree(host_ptr) != hipSuccess)
        return fail(R48_EHIP, "hipHostFree failed");
    return R48_OK;
}

}  // extern "C"
