// r48_bn_finish.h -- the per-channel arithmetic of a training-mode BatchNorm's finish, forward
// (batch statistics -> mean / invstd, apply coefficients, running statistics) and backward (the
// reduction's two sums -> dgamma, dbeta, the input gradient's coefficients), shared by the
// standalone finish kernels (r48_bn.hip) and the conv kernels that finish the BN of their own
// output in the workgroup that writes the last statistics record (r48_conv.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/rein48.h"

namespace r48bn {

// forward: s1 = sum (x - x0), s2 = sum (x - x0)^2 over `rows` values of channel c (x0 the shift of
// the sums, 0 for unshifted ones); torch.nn.BatchNorm's training-mode statistics (biased variance
// for the normalisation, unbiased for the running variance, momentum update)
__device__ inline void fwd_channel(const r48_bn_finish_args &f, int C, int c, double s1, double s2, double x0)
{
    const double n = (double)f.rows;
    const double dm = s1 / n;
    double var = s2 / n - dm * dm;
    var = var > 0.0 ? var : 0.0;
    const double mean = x0 + dm;
    const double invstd = 1.0 / sqrt(var + (double)f.eps);
    f.save[c] = (float)mean;
    f.save[C + c] = (float)invstd;
    const double a = (double)f.gamma[c] * invstd;
    f.coef[c] = (float)a;
    f.coef[C + c] = (float)((double)f.beta[c] - mean * a);
    if (f.running_mean) {
        const double unb = f.rows > 1 ? var * n / (n - 1.0) : var;
        f.running_mean[c] = (float)((1.0 - f.momentum) * (double)f.running_mean[c] + f.momentum * mean);
        f.running_var[c] = (float)((1.0 - f.momentum) * (double)f.running_var[c] + f.momentum * unb);
    }
}

// backward: sg = sum g, sgx = sum g (x - mean) of channel c (g = the output gradient through the
// ReLU mask); dbeta = sg, dgamma = invstd sgx, and dx = a g + cc x + d (coef = a | cc | d)
__device__ inline void bwd_channel(const r48_bn_finish_args &f, int C, int c, double sg, double sgx)
{
    const double mean = f.save[c], invstd = f.save[C + c], n = (double)f.rows;
    const double dg = sgx * invstd;
    if (f.dgamma)
        f.dgamma[c] = (float)dg;
    if (f.dbeta)
        f.dbeta[c] = (float)sg;
    const double a = (double)f.gamma[c] * invstd;
    const double cc = -a * invstd * dg / n;
    f.coef[c] = (float)a;
    f.coef[C + c] = (float)cc;
    f.coef[2 * C + c] = (float)(-a * sg / n - cc * mean);
}

// The finish over NREC per-workgroup records [sum 0 (C)][sum 1 (C)] by one workgroup of 4 * 2C
// threads: thread (quarter q, stat s) sums records q NREC/4 .. in record order in fp64, the four
// quarters are added in order ((q0 + q1) + q2) + q3 -- a fixed order (deterministic). lds: 8 * C
// doubles. The records were written with agent-scope atomic stores (r48_conv.hip), read here with
// agent-scope atomic loads.
template <int C, int NREC, bool BWD>
__device__ inline void finish_records(const float *rec, const r48_bn_finish_args &f, double *lds)
{
    static_assert(NREC % 4 == 0, "four equal quarters");
    constexpr int kPer = NREC / 4;
    const int t = threadIdx.x, s = t % (2 * C), q = t / (2 * C);
    double acc = 0.0;
#pragma unroll 16
    for (int r = 0; r < kPer; r++)   // device-coherent loads: the records of every workgroup
        acc += (double)__hip_atomic_load(rec + (int64_t)(q * kPer + r) * 2 * C + s, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    lds[q * 2 * C + s] = acc;
    __syncthreads();
    if (t < C) {
        double v[2];
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int i = k * C + t;
            v[k] = ((lds[i] + lds[2 * C + i]) + lds[4 * C + i]) + lds[6 * C + i];
        }
        if (BWD)
            bwd_channel(f, C, t, v[0], v[1]);
        else
            fwd_channel(f, C, t, v[0], v[1], 0.0);
    }
}

}  // namespace r48bn
