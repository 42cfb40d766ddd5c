// r48_replay.hip -- HBM-resident transition store for DQN-style training (config 5) behind the
// C-ABI (include/rein48.h, r48_replay_*).
//
// Reference anchor: algorithm/ddpg/replay.py:8-47 (Replay: store() appends until max_size and
// then drops, sample() = random.sample without replacement -- or the whole buffer in insertion
// order when it holds fewer than batch_size -- followed by clear()). That is the
// R48_REPLAY_FILL_DRAIN mode; R48_REPLAY_RING is the usual DQN ring (overwrite the oldest,
// sample uniformly with replacement), which BASELINE config 5 asks for at 16M boards.
//
// Layout: structure of arrays over `capacity` slots, 38 B per transition --
//   state int8[cap][16] | next_state int8[cap][16] | action int8[cap] | done uint8[cap] |
//   reward float[cap]
// so a store of n transitions from the env's contiguous arrays is n coalesced 16-B rows per
// board plane, and a sampled gather reads one 16-B row per board plane per lane.
// Random draws are Philox4x32-10 keyed by the store's seed with a per-call sample counter:
//   ring:   counter {i lo, i hi, sample_ctr, 0x5A4}, index = mulhi64(w0 | w1 << 32, size)
//   drain:  a 4-round Feistel permutation of [0, 4^h) (2h >= ceil(log2 size), h >= 1), round j
//           F(R) = Philox({R, sample_ctr, j, 0x5A3}).w0 & (2^h - 1), cycle-walked into
//           [0, size): output i < batch <= size is slot perm(i) -- sampling without replacement
//           (batch > size returns every slot in insertion order, as replay.py:31-32 does).
// Both restated in oracle/r48_oracle.c (orc_replay_ring_index / orc_replay_perm_index).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/rein48.h"
#include "r48_board.h"

namespace r48 {
void set_last_error(const std::string &msg);
}

struct r48_replay {
    int device;
    uint32_t mode;
    int64_t cap, size, head;
    uint64_t seed;
    uint32_t sample_ctr;
    int8_t *state, *next, *action;
    uint8_t *done;
    float *reward;
    unsigned long long *err;  // device counter of invalid gather indices
};

namespace {

constexpr int kBlock = 256;
constexpr uint32_t kPermTag = 0x5A3u;
constexpr uint32_t kRingTag = 0x5A4u;
constexpr int kMaxWalk = 4096;  // cycle-walk bound (domain <= 4 x size: P(> 4096) ~ 0.75^4096)

enum Src { SRC_GIVEN = 0, SRC_RING = 1, SRC_PERM = 2, SRC_IDENT = 3 };

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

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) == hipSuccess && prev != dev)
            (void)hipSetDevice(dev);
    }
    ~DeviceGuard()
    {
        int cur;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev)
            (void)hipSetDevice(prev);
    }
};

__device__ __forceinline__ uint32_t philox_w0(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                              uint32_t k1, uint32_t *w1 = nullptr)
{
    uint32_t w[4] = {c0, c1, c2, c3};
    r48::philox4x32_10(w, k0, k1);
    if (w1)
        *w1 = w[1];
    return w[0];
}

__device__ __forceinline__ uint64_t feistel(uint64_t x, uint32_t h, uint32_t ctr, uint32_t k0, uint32_t k1)
{
    const uint64_t mask = (1ull << h) - 1ull;
    uint64_t L = x >> h, R = x & mask;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const uint64_t F = philox_w0((uint32_t)R, ctr, j, kPermTag, k0, k1) & mask;
        const uint64_t nl = R;
        R = L ^ F;
        L = nl;
    }
    return (L << h) | R;
}

__global__ __launch_bounds__(kBlock) void k_store(int8_t *__restrict__ st, int8_t *__restrict__ nx,
                                                  int8_t *__restrict__ ac, uint8_t *__restrict__ dn,
                                                  float *__restrict__ rw, int64_t cap, int64_t head, int64_t n,
                                                  const int8_t *__restrict__ s, const int8_t *__restrict__ a,
                                                  const float *__restrict__ r, const int8_t *__restrict__ s2,
                                                  const uint8_t *__restrict__ d)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    int64_t slot = head + i;
    if (slot >= cap)
        slot -= cap;
    *reinterpret_cast<uint4 *>(st + 16 * slot) = *reinterpret_cast<const uint4 *>(s + 16 * i);
    *reinterpret_cast<uint4 *>(nx + 16 * slot) = *reinterpret_cast<const uint4 *>(s2 + 16 * i);
    ac[slot] = a[i];
    rw[slot] = r ? r[i] : 0.0f;
    dn[slot] = d ? d[i] : (uint8_t)0;
}

template <int SRC>
__global__ __launch_bounds__(kBlock) void k_gather(const int8_t *__restrict__ st, const int8_t *__restrict__ nx,
                                                   const int8_t *__restrict__ ac, const uint8_t *__restrict__ dn,
                                                   const float *__restrict__ rw, int64_t size, int64_t n,
                                                   const int64_t *__restrict__ given, uint32_t h, uint32_t ctr,
                                                   uint32_t k0, uint32_t k1, int8_t *__restrict__ os,
                                                   int8_t *__restrict__ oa, float *__restrict__ orw,
                                                   int8_t *__restrict__ os2, uint8_t *__restrict__ od,
                                                   int64_t *__restrict__ oidx, unsigned long long *err)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    int64_t idx;
    bool ok = true;
    if (SRC == SRC_GIVEN) {
        idx = given[i];
        ok = idx >= 0 && idx < size;
    } else if (SRC == SRC_RING) {
        uint32_t w1;
        const uint32_t w0 = philox_w0((uint32_t)i, (uint32_t)((uint64_t)i >> 32), ctr, kRingTag, k0, k1, &w1);
        idx = (int64_t)__umul64hi((uint64_t)w0 | ((uint64_t)w1 << 32), (uint64_t)size);
    } else if (SRC == SRC_PERM) {
        uint64_t x = (uint64_t)i;
        int walk = 0;
        do {
            x = feistel(x, h, ctr, k0, k1);
        } while (x >= (uint64_t)size && ++walk < kMaxWalk);
        idx = (int64_t)x;
        ok = x < (uint64_t)size;
    } else {
        idx = i;
    }
    if (!ok) {
        atomicAdd(err, 1ull);
        idx = 0;
    }
    uint4 zero = make_uint4(0, 0, 0, 0);
    if (os)
        *reinterpret_cast<uint4 *>(os + 16 * i) = ok ? *reinterpret_cast<const uint4 *>(st + 16 * idx) : zero;
    if (os2)
        *reinterpret_cast<uint4 *>(os2 + 16 * i) = ok ? *reinterpret_cast<const uint4 *>(nx + 16 * idx) : zero;
    if (oa)
        oa[i] = ok ? ac[idx] : (int8_t)0;
    if (orw)
        orw[i] = ok ? rw[idx] : 0.0f;
    if (od)
        od[i] = ok ? dn[idx] : (uint8_t)0;
    if (oidx)
        oidx[i] = ok ? idx : -1;
}

bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

int check_rep(const r48_replay *rep)
{
    if (!rep || !rep->state)
        return fail(R48_EINVAL, "NULL replay handle");
    return R48_OK;
}

// Feistel half width: 2h >= ceil(log2(size)), h >= 1.
uint32_t half_bits(int64_t size)
{
    uint32_t k = 1;
    while (k < 63 && ((int64_t)1 << k) < size)
        ++k;
    return (k + 1) / 2;
}

int gather(r48_replay *rep, int src, const int64_t *given, int64_t n, int8_t *state, int8_t *action, float *reward,
           int8_t *next_state, uint8_t *done, int64_t *index, void *stream)
{
    if ((state && !aligned16(state)) || (next_state && !aligned16(next_state)))
        return fail(R48_EINVAL, "state/next_state outputs must be 16-byte aligned");
    if (n == 0)
        return R48_OK;
    DeviceGuard g(rep->device);
    const uint32_t h = half_bits(rep->size);
    const uint32_t k0 = (uint32_t)rep->seed, k1 = (uint32_t)(rep->seed >> 32);
#define R48_GATHER(S)                                                                                            \
    hipLaunchKernelGGL(k_gather<S>, grid_for(n), dim3(kBlock), 0, (hipStream_t)stream, rep->state, rep->next,   \
                       rep->action, rep->done, rep->reward, rep->size, n, given, h, rep->sample_ctr, k0, k1, state, \
                       action, reward, next_state, done, index, rep->err)
    switch (src) {
    case SRC_GIVEN: R48_GATHER(SRC_GIVEN); break;
    case SRC_RING: R48_GATHER(SRC_RING); break;
    case SRC_PERM: R48_GATHER(SRC_PERM); break;
    default: R48_GATHER(SRC_IDENT); break;
    }
#undef R48_GATHER
    return launched("k_gather");
}

}  // namespace

extern "C" {

int r48_replay_create(r48_replay **out, int device, int64_t capacity, uint32_t mode, uint64_t seed)
{
    if (!out || capacity < 1 || mode > R48_REPLAY_FILL_DRAIN)
        return fail(R48_EINVAL, "out NULL, capacity < 1 or unknown mode");
    *out = nullptr;
    DeviceGuard g(device);
    r48_replay *rep = new r48_replay{};
    rep->device = device;
    rep->mode = mode;
    rep->cap = capacity;
    rep->seed = seed;
    const size_t c = (size_t)capacity;
    bool ok = hipMalloc(&rep->state, 16 * c) == hipSuccess && hipMalloc(&rep->next, 16 * c) == hipSuccess &&
              hipMalloc(&rep->action, c) == hipSuccess && hipMalloc(&rep->done, c) == hipSuccess &&
              hipMalloc(&rep->reward, 4 * c) == hipSuccess &&
              hipMalloc(&rep->err, sizeof(unsigned long long)) == hipSuccess &&
              hipMemset(rep->err, 0, sizeof(unsigned long long)) == hipSuccess;
    if (!ok) {
        (void)hipGetLastError();
        r48_replay_destroy(rep);
        return fail(R48_ENOMEM, "hipMalloc of the replay planes failed");
    }
    *out = rep;
    return R48_OK;
}

int r48_replay_destroy(r48_replay *rep)
{
    if (!rep)
        return R48_OK;
    DeviceGuard g(rep->device);
    (void)hipDeviceSynchronize();
    for (void *p : {(void *)rep->state, (void *)rep->next, (void *)rep->action, (void *)rep->done,
                    (void *)rep->reward, (void *)rep->err})
        if (p)
            (void)hipFree(p);
    delete rep;
    return R48_OK;
}

int r48_replay_get_counters(const r48_replay *rep, int64_t *size, int64_t *head, uint32_t *sample_ctr)
{
    if (int s = check_rep(rep))
        return s;
    if (size)
        *size = rep->size;
    if (head)
        *head = rep->head;
    if (sample_ctr)
        *sample_ctr = rep->sample_ctr;
    return R48_OK;
}

int r48_replay_set_counters(r48_replay *rep, int64_t size, int64_t head, uint32_t sample_ctr)
{
    if (int s = check_rep(rep))
        return s;
    if (size < 0 || size > rep->cap || head < 0 || head >= rep->cap)
        return fail(R48_EINVAL, "size must be in [0, capacity], head in [0, capacity)");
    rep->size = size;
    rep->head = head;
    rep->sample_ctr = sample_ctr;
    return R48_OK;
}

int64_t r48_replay_capacity(const r48_replay *rep) { return rep ? rep->cap : -1; }

int r48_replay_planes(const r48_replay *rep, int8_t **state, int8_t **action, float **reward, int8_t **next_state,
                      uint8_t **done)
{
    if (int s = check_rep(rep))
        return s;
    if (state)
        *state = rep->state;
    if (action)
        *action = rep->action;
    if (reward)
        *reward = rep->reward;
    if (next_state)
        *next_state = rep->next;
    if (done)
        *done = rep->done;
    return R48_OK;
}

int r48_replay_clear(r48_replay *rep)
{
    if (int s = check_rep(rep))
        return s;
    rep->size = 0;
    rep->head = 0;
    return R48_OK;
}

int r48_replay_store(r48_replay *rep, const int8_t *state, const int8_t *action, const float *reward,
                     const int8_t *next_state, const uint8_t *done, int64_t n, int64_t *stored, void *stream)
{
    if (int s = check_rep(rep))
        return s;
    if (!state || !action || !next_state || n < 0)
        return fail(R48_EINVAL, "state/action/next_state NULL or n < 0");
    if (!aligned16(state) || !aligned16(next_state))
        return fail(R48_EINVAL, "state/next_state must be 16-byte aligned");
    int64_t skip = 0, m = n;
    if (rep->mode == R48_REPLAY_FILL_DRAIN) {
        m = n < rep->cap - rep->size ? n : rep->cap - rep->size;  // replay.py:18-21: drop when full
    } else if (n > rep->cap) {
        skip = n - rep->cap;                                      // only the newest cap survive
        m = rep->cap;
    }
    if (stored)
        *stored = m;
    if (m == 0)
        return R48_OK;
    DeviceGuard g(rep->device);
    const int64_t head = rep->mode == R48_REPLAY_FILL_DRAIN ? rep->size : (rep->head + skip) % rep->cap;
    hipLaunchKernelGGL(k_store, grid_for(m), dim3(kBlock), 0, (hipStream_t)stream, rep->state, rep->next, rep->action,
                       rep->done, rep->reward, rep->cap, head, m, state + 16 * skip, action + skip,
                       reward ? reward + skip : nullptr, next_state + 16 * skip, done ? done + skip : nullptr);
    rep->head = (head + m) % rep->cap;
    rep->size = rep->size + m < rep->cap ? rep->size + m : rep->cap;
    return launched("k_store");
}

int r48_replay_sample(r48_replay *rep, int64_t batch, int8_t *state, int8_t *action, float *reward,
                      int8_t *next_state, uint8_t *done, int64_t *index, int64_t *count, void *stream)
{
    if (int s = check_rep(rep))
        return s;
    if (batch < 0)
        return fail(R48_EINVAL, "batch < 0");
    int64_t m;
    int src;
    if (rep->mode == R48_REPLAY_FILL_DRAIN) {
        // replay.py:23-34: the whole buffer in insertion order when batch > len, else
        // random.sample (without replacement; batch == len is a permutation); then clear()
        // (:26, :45-47).
        m = batch < rep->size ? batch : rep->size;
        src = batch > rep->size ? SRC_IDENT : SRC_PERM;
    } else {
        if (rep->size == 0 && batch > 0)
            return fail(R48_EINVAL, "sampling an empty ring");
        m = batch;
        src = SRC_RING;
    }
    if (count)
        *count = m;
    int s = gather(rep, src, nullptr, m, state, action, reward, next_state, done, index, stream);
    if (s)
        return s;
    rep->sample_ctr++;
    if (rep->mode == R48_REPLAY_FILL_DRAIN) {
        rep->size = 0;
        rep->head = 0;
    }
    return R48_OK;
}

int r48_replay_gather(r48_replay *rep, const int64_t *index, int64_t n, int8_t *state, int8_t *action,
                      float *reward, int8_t *next_state, uint8_t *done, void *stream)
{
    if (int s = check_rep(rep))
        return s;
    if (!index || n < 0)
        return fail(R48_EINVAL, "index NULL or n < 0");
    return gather(rep, SRC_GIVEN, index, n, state, action, reward, next_state, done, nullptr, stream);
}

int r48_replay_error_count(const r48_replay *rep, uint64_t *count)
{
    if (int s = check_rep(rep))
        return s;
    if (!count)
        return fail(R48_EINVAL, "count NULL");
    DeviceGuard g(rep->device);
    if (hipMemcpy(count, rep->err, sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
        return fail(R48_EHIP, "hipMemcpy of the error counter failed");
    return R48_OK;
}

}  // extern "C"
