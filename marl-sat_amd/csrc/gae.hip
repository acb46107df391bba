// GAE reverse scan + global advantage normalisation (gfx950).
//
// Reference: src/learners/mappo_gnn_sat_learner.py:504-532
//   delta = r0 + GAMMA * V' * (1-d) - V ;  A = delta + GAMMA*LAMBDA * (1-d) * A'
//   targets = A + V ; A <- (A - mean) / (std + 1e-8)   (population std over all T*B)
// One lane per env walks t = T-1..0 (loads of one t are coalesced across lanes);
// the normalisation statistics are reduced in fp64 in a fixed order
// (per-block partials, every block of the second kernel re-reduces them), so the
// result is bitwise reproducible run to run.  HBM-bound: 17 B per (t, env).
#include <algorithm>

#include "common.h"

namespace msat {

constexpr int kGaeThreads = 256;

__global__ void __launch_bounds__(kGaeThreads)
gae_scan_kernel(int T, int B, const float *__restrict__ reward, int rstride, const uint8_t *__restrict__ done,
                const float *__restrict__ value, const float *__restrict__ last_val, float gamma, float gl,
                float *__restrict__ adv, float *__restrict__ targets, double *__restrict__ partial) {
    __shared__ double s_sum[kGaeThreads / 64], s_sq[kGaeThreads / 64];
    const int b = blockIdx.x * kGaeThreads + threadIdx.x;
    double sum = 0.0, sq = 0.0;
    if (b < B) {
        float gae = 0.0f, next_v = last_val[b];
        for (int t = T - 1; t >= 0; --t) {
            const size_t i = (size_t)t * B + b;
            const float nd = done[i] ? 0.0f : 1.0f;
            const float v = value[i];
            const float delta = __fsub_rn(__fadd_rn(reward[i * rstride], __fmul_rn(__fmul_rn(gamma, next_v), nd)), v);
            gae = __fadd_rn(delta, __fmul_rn(__fmul_rn(gl, nd), gae));
            adv[i] = gae;
            targets[i] = __fadd_rn(gae, v);
            next_v = v;
            sum += (double)gae;
            sq += (double)gae * (double)gae;
        }
    }
    sum = wave_sum_f64(sum);
    sq = wave_sum_f64(sq);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_sum[w] = sum;
        s_sq[w] = sq;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = 0.0, c = 0.0;
        for (int k = 0; k < kGaeThreads / 64; ++k) {
            a += s_sum[k];
            c += s_sq[k];
        }
        partial[2 * blockIdx.x] = a;
        partial[2 * blockIdx.x + 1] = c;
    }
}

__global__ void __launch_bounds__(kGaeThreads)
gae_normalize_kernel(size_t n, int nparts, const double *__restrict__ partial, float *__restrict__ adv,
                     double *__restrict__ stats) {
    __shared__ float s_meanf, s_stdf;
    if (threadIdx.x == 0) {
        double a = 0.0, c = 0.0;
        for (int k = 0; k < nparts; ++k) {
            a += partial[2 * k];
            c += partial[2 * k + 1];
        }
        const double mean = a / (double)n;
        const double var = fmax(c / (double)n - mean * mean, 0.0);
        const double stdv = sqrt(var) + 1e-8;
        s_meanf = (float)mean;
        s_stdf = (float)stdv;
        if (blockIdx.x == 0) {
            stats[0] = mean;
            stats[1] = stdv;
        }
    }
    __syncthreads();
    const float mf = s_meanf, sf = s_stdf;
    for (size_t i = (size_t)blockIdx.x * kGaeThreads + threadIdx.x; i < n; i += (size_t)gridDim.x * kGaeThreads)
        adv[i] = __fdiv_rn(__fsub_rn(adv[i], mf), sf);
}

// out[0] += sum x, out[1] += sum x^2 (fp64, per-block partials combined by one block)
__global__ void __launch_bounds__(kGaeThreads)
moments_kernel(const float *__restrict__ x, size_t n, double *__restrict__ part) {
    __shared__ double s1[kGaeThreads / 64], s2[kGaeThreads / 64];
    double a = 0.0, b = 0.0;
    for (size_t i = (size_t)blockIdx.x * kGaeThreads + threadIdx.x; i < n; i += (size_t)gridDim.x * kGaeThreads) {
        const double v = x[i];
        a += v;
        b += v * v;
    }
    a = wave_sum_f64(a);
    b = wave_sum_f64(b);
    if ((threadIdx.x & 63) == 0) {
        s1[threadIdx.x >> 6] = a;
        s2[threadIdx.x >> 6] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = s1[0] + s1[1] + s1[2] + s1[3];
        part[2 * blockIdx.x + 1] = s2[0] + s2[1] + s2[2] + s2[3];
    }
}

__global__ void moments_reduce_kernel(const double *__restrict__ part, int nb, double *__restrict__ out) {
    if (threadIdx.x == 0) {
        double a = 0.0, b = 0.0;
        for (int k = 0; k < nb; ++k) {
            a += part[2 * k];
            b += part[2 * k + 1];
        }
        out[0] = a;
        out[1] = b;
    }
}

__global__ void standardize_kernel(float *__restrict__ x, size_t n, float mean, float stdv) {
    for (size_t i = (size_t)blockIdx.x * kGaeThreads + threadIdx.x; i < n; i += (size_t)gridDim.x * kGaeThreads)
        x[i] = __fdiv_rn(__fsub_rn(x[i], mean), stdv);
}

}  // namespace msat

using namespace msat;

static int stat_blocks(size_t n) { return (int)std::min<size_t>((n + kGaeThreads - 1) / kGaeThreads, 1024); }

extern "C" int msat_moments(const float *x, size_t n, double *out2, void *workspace, void *stream) {
    MSAT_REQUIRE(x && out2 && workspace, "NULL pointer");
    const int nb = std::max(1, stat_blocks(n));
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(moments_kernel, dim3(nb), dim3(kGaeThreads), 0, s, x, n, (double *)workspace);
    int rc = check_launch("moments_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(moments_reduce_kernel, dim3(1), dim3(64), 0, s, (const double *)workspace, nb, out2);
    return check_launch("moments_reduce_kernel");
}

extern "C" int msat_standardize(float *x, size_t n, float mean, float stdv, void *stream) {
    MSAT_REQUIRE(x, "NULL pointer");
    if (!n) return MSAT_OK;
    hipLaunchKernelGGL(standardize_kernel, dim3(stat_blocks(n)), dim3(kGaeThreads), 0, (hipStream_t)stream, x, n, mean,
                       stdv);
    return check_launch("standardize_kernel");
}

static int gae_blocks(int B) { return (B + kGaeThreads - 1) / kGaeThreads; }

extern "C" size_t msat_gae_workspace_bytes(int32_t T, int32_t B) {
    (void)T;
    return (size_t)(2 * gae_blocks(B) + 2) * sizeof(double);
}

extern "C" int msat_gae(int32_t T, int32_t B, const float *reward, int32_t reward_stride, const uint8_t *done,
                        const float *value, const float *last_val, float gamma, float gamma_lambda,
                        int32_t normalize, float *advantages, float *targets, void *workspace, void *stream) {
    MSAT_REQUIRE(T >= 1 && B >= 1, "bad dims T=%d B=%d", T, B);
    MSAT_REQUIRE(reward && done && value && last_val && advantages && targets && workspace, "NULL pointer");
    MSAT_REQUIRE(reward_stride >= 1, "reward_stride %d < 1", reward_stride);
    hipStream_t s = (hipStream_t)stream;
    const int nb = gae_blocks(B);
    double *partial = (double *)workspace;
    double *stats = partial + 2 * nb;
    hipLaunchKernelGGL(gae_scan_kernel, dim3(nb), dim3(kGaeThreads), 0, s, T, B, reward, reward_stride, done, value,
                       last_val, gamma, gamma_lambda, advantages, targets, partial);
    int rc = check_launch("gae_scan_kernel");
    if (rc || !normalize) return rc;
    const size_t n = (size_t)T * B;
    const int grid = (int)std::min<size_t>((n + kGaeThreads - 1) / kGaeThreads, 1024);
    hipLaunchKernelGGL(gae_normalize_kernel, dim3(grid), dim3(kGaeThreads), 0, s, n, nb, partial, advantages, stats);
    return check_launch("gae_normalize_kernel");
}
