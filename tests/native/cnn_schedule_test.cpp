// Compile-time checks of the fused CNN kernels' weight-fragment read schedules
// (rein48_amd/csrc/r48_cnn_common.h): every read names a valid fragment, the policy order reads each
// of its 33 fragments exactly once (heads after the conv2 half they consume, conv1 first); the chain
// order (training kernel) reads conv1 and head fragments once and every conv2 fragment once per
// output position.
// Built by tests/test_board_logic_host.py with `hipcc --offload-host-only -fsyntax-only`.
#include "../../rein48_amd/csrc/r48_cnn_common.h"

using namespace r48cnn;

constexpr bool chain_order_counts()
{
    int cnt[kFrags] = {};
    for (int i = 0; i < kFwdMfmas; i++) {
        const int f = fwd_frag(i);
        if (f < 0 || f >= kFrags)
            return false;
        cnt[f]++;
    }
    for (int f = 0; f < kFrags; f++) {
        const int want = (f >= kFragW1 && f < kFragW1 + kFragW2) ? 4 : 1;
        if (cnt[f] != want)
            return false;
    }
    return true;
}

// the policy kernels' order (heads on 16x16x32 MFMAs, H16(p, g) at kFragW1 + kFragW2 + 2p + g)
constexpr bool policy_reads_each_fragment_once()
{
    int cnt[kFragsPolicy] = {};
    for (int i = 0; i < kPolicyReads; i++) {
        const int f = policy_frag(i);
        if (f < 0 || f >= kFragsPolicy)
            return false;
        cnt[f]++;
    }
    for (int f = 0; f < kFragsPolicy; f++)
        if (cnt[f] != 1)
            return false;
    for (int i = 0; i < 9; i++)
        if (policy_frag(i) != i)
            return false;
    return true;
}

constexpr bool policy_heads_after_their_half()
{
    int last_w2[2] = {-1, -1}, first_head[2] = {1 << 20, 1 << 20};
    for (int i = 0; i < kPolicyReads; i++) {
        const int f = policy_frag(i);
        if (f >= kFragW1 && f < kFragW1 + kFragW2) {
            last_w2[(f - kFragW1) >> 3] = i;
        } else if (f >= kFragW1 + kFragW2) {
            const int g = (f - kFragW1 - kFragW2) & 1;
            if (i < first_head[g])
                first_head[g] = i;
        }
    }
    return last_w2[0] < first_head[0] && last_w2[1] < first_head[1];
}

static_assert(kPolicyReads == kFragsPolicy && kFragsPolicy == 33, "policy schedule length");
static_assert(policy_reads_each_fragment_once(), "policy schedule reads every fragment once, conv1 first");
static_assert(policy_heads_after_their_half(), "policy head fragments follow the conv2 half they consume");
static_assert(chain_order_counts(), "chain schedule: conv2 fragments once per position");
