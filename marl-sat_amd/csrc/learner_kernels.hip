// Learner glue on the device (learner:148-195, 562-719 around the network calls): the PPO epoch's
// row permutation, the micro-batch row gather, the graph batch's row bases and the cycle metrics.
// They replaced torch ops (randperm on the host + copy, index kernels, cumsum, fp64 reductions) so
// that nothing on the timed MAPPO path computes outside this library.
#include <stdint.h>

#include "common.h"
#include "marlsat_net.h"

namespace msat {

// ---------------------------------------------------------------------------------------------
// Permutation of [0, N): a 4-round balanced Feistel network on k-bit words (2^k >= N, k even) keyed
// from (seed, counter), restricted to [0, N) by cycle walking (x -> F(x) until x < N; F is a bijection
// of [0, 2^k) so the walk returns to [0, N), on average in <= 2^k / N <= 4 applications).  Replaces
// jax.random.permutation (learner:576): JAX's threefry stream cannot be reproduced, any keyed uniform-
// looking bijection serves the minibatching; deterministic for a given (seed, counter).
__device__ __forceinline__ uint32_t perm_round(uint32_t r, uint32_t key) {
    uint32_t h = (r ^ key) * 0x9E3779B1u;
    h ^= h >> 15;
    h *= 0x85EBCA77u;
    h ^= h >> 13;
    h *= 0xC2B2AE3Du;
    return h ^ (h >> 16);
}

__global__ void permutation_kernel(int N, int half, uint4 keys, int32_t *__restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const uint32_t mask = (1u << half) - 1u;
    const uint32_t k[4] = {keys.x, keys.y, keys.z, keys.w};
    uint32_t x = (uint32_t)i;
    do {
        uint32_t L = x >> half, R = x & mask;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t nl = R;
            R = L ^ (perm_round(R, k[r]) & mask);
            L = nl;
        }
        x = (L << half) | R;
    } while (x >= (uint32_t)N);
    out[i] = (int32_t)x;
}

// ---------------------------------------------------------------------------------------------
// dst_f[s] = src_f[idx[s]] for up to 8 fields of fixed row size (bytes), one workgroup per 4 rows.
struct GatherFields {
    const uint8_t *src[8];
    uint8_t *dst[8];
    int row_bytes[8];
    int n;
};

__global__ void __launch_bounds__(256) gather_rows_kernel(const int32_t *__restrict__ idx, int S, GatherFields f) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int s = blockIdx.x * 4 + w;
    if (s >= S) return;
    const size_t r = (size_t)idx[s];
    for (int q = 0; q < f.n; ++q) {
        const int rb = f.row_bytes[q];
        const uint8_t *src = f.src[q] + r * rb;
        uint8_t *dst = f.dst[q] + (size_t)s * rb;
        if ((rb & 3) == 0 && ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 3) == 0) {
            const uint32_t *s4 = reinterpret_cast<const uint32_t *>(src);
            uint32_t *d4 = reinterpret_cast<uint32_t *>(dst);
            for (int j = lane; j < rb / 4; j += 64) d4[j] = s4[j];
        } else {
            for (int j = lane; j < rb; j += 64) dst[j] = src[j];
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Cycle metrics (learner:661-719) over the N = T*B transitions, fp64, one workgroup, fixed-order
// reduction (bitwise reproducible):
//   out[0] = sum reward, [1] = sum done, [2] = sum solved&done, [3] = sum unsat*done,
//   [4] = sum episode_step*(solved&done), [5] = sum tg, [6] = sum tg^2, [7] = sum d, [8] = sum d^2
// with d = tg - vpred (explained variance of the re-run critic).
constexpr int kMetT = 1024;

__global__ void __launch_bounds__(kMetT) cycle_metrics_kernel(int N, const float *__restrict__ reward,
                                                              const uint8_t *__restrict__ done,
                                                              const uint8_t *__restrict__ solved,
                                                              const int32_t *__restrict__ unsat,
                                                              const int32_t *__restrict__ steps,
                                                              const float *__restrict__ tg,
                                                              const float *__restrict__ vpred,
                                                              double *__restrict__ out) {
    __shared__ double red[9][kMetT / 64];
    double a[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = threadIdx.x; i < N; i += kMetT) {
        const double dn = done[i] ? 1.0 : 0.0, sv = (solved[i] && done[i]) ? 1.0 : 0.0;
        const double t = (double)tg[i], d = t - (double)vpred[i];
        a[0] += (double)reward[i];
        a[1] += dn;
        a[2] += sv;
        a[3] += (double)unsat[i] * dn;
        a[4] += (double)steps[i] * sv;
        a[5] += t;
        a[6] += t * t;
        a[7] += d;
        a[8] += d * d;
    }
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < 9; ++q) {
        double v = a[q];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if (lane == 0) red[q][w] = v;
    }
    __syncthreads();
    if (threadIdx.x < 9) {
        double v = 0.0;
        for (int j = 0; j < kMetT / 64; ++j) v += red[threadIdx.x][j];
        out[threadIdx.x] = v;
    }
}

// ---------------------------------------------------------------------------------------------
// Row bases of a graph batch: for samples s < S of instances inst[s], with per-instance row counts
// (var rows, clause rows, incidences) nv[i], nc[i], ne[i], bases[s] = exclusive prefix sums (S, 3) and
// totals[3] = the sums, or -1 for a sum above INT32_MAX (the batch's int32 row indices would wrap;
// the caller refuses the batch).  One workgroup (the batch is at most a few ten thousand samples): each thread
// sums a contiguous chunk, the chunk sums are scanned in LDS, then every chunk is re-walked.
constexpr int kScanT = 1024;

__global__ void __launch_bounds__(kScanT) graph_bases_kernel(int S, const int32_t *__restrict__ inst,
                                                             const int32_t *__restrict__ nv,
                                                             const int32_t *__restrict__ nc,
                                                             const int32_t *__restrict__ ne,
                                                             int32_t *__restrict__ bases, int32_t *__restrict__ totals) {
    __shared__ long long sc[3][kScanT];
    const int t = threadIdx.x, per = (S + kScanT - 1) / kScanT;
    const int b = min(S, t * per), e = min(S, b + per);
    long long a[3] = {0, 0, 0};
    for (int s = b; s < e; ++s) {
        const int i = inst[s];
        a[0] += nv[i];
        a[1] += nc[i];
        a[2] += ne[i];
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) sc[q][t] = a[q];
    __syncthreads();
    for (int o = 1; o < kScanT; o <<= 1) {  // Hillis-Steele inclusive scan of the chunk sums
        long long v[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) v[q] = t >= o ? sc[q][t - o] : 0;
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 3; ++q) sc[q][t] += v[q];
        __syncthreads();
    }
    long long run[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) run[q] = sc[q][t] - a[q];  // exclusive base of this chunk
    for (int s = b; s < e; ++s) {
        const int i = inst[s];
        bases[3 * s] = (int32_t)run[0];
        bases[3 * s + 1] = (int32_t)run[1];
        bases[3 * s + 2] = (int32_t)run[2];
        run[0] += nv[i];
        run[1] += nc[i];
        run[2] += ne[i];
    }
    if (t == kScanT - 1) {
#pragma unroll
        for (int q = 0; q < 3; ++q) totals[q] = sc[q][t] > (long long)INT32_MAX ? -1 : (int32_t)sc[q][t];
    }
}

__host__ inline uint64_t splitmix64(uint64_t &s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

}  // namespace msat

using namespace msat;

extern "C" int msat_permutation(int32_t N, uint64_t seed, uint64_t counter, int32_t *out, void *stream) {
    MSAT_REQUIRE(N >= 0 && (N == 0 || out), "permutation: bad args");
    if (N == 0) return MSAT_OK;
    int k = 2;
    while ((1ll << k) < (long long)N) ++k;
    if (k & 1) ++k;
    MSAT_REQUIRE(k <= 31, "permutation: N too large");
    uint64_t st = seed ^ (counter * 0xD1B54A32D192ED03ull);
    uint4 keys;
    keys.x = (uint32_t)splitmix64(st);
    keys.y = (uint32_t)splitmix64(st);
    keys.z = (uint32_t)splitmix64(st);
    keys.w = (uint32_t)splitmix64(st);
    hipLaunchKernelGGL(permutation_kernel, dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream, N, k / 2, keys,
                       out);
    return check_launch("permutation_kernel");
}

extern "C" int msat_gather_rows(const int32_t *idx, int32_t S, int32_t nfields, const void *const *src,
                                void *const *dst, const int32_t *row_bytes, void *stream) {
    MSAT_REQUIRE(S >= 0 && nfields >= 0 && nfields <= 8, "gather_rows: 0 <= nfields <= 8");
    if (S == 0 || nfields == 0) return MSAT_OK;
    MSAT_REQUIRE(idx && src && dst && row_bytes, "gather_rows: NULL pointer");
    GatherFields f = {};
    f.n = nfields;
    for (int q = 0; q < nfields; ++q) {
        MSAT_REQUIRE(src[q] && dst[q] && row_bytes[q] > 0, "gather_rows: field %d", q);
        f.src[q] = static_cast<const uint8_t *>(src[q]);
        f.dst[q] = static_cast<uint8_t *>(dst[q]);
        f.row_bytes[q] = row_bytes[q];
    }
    hipLaunchKernelGGL(gather_rows_kernel, dim3((S + 3) / 4), dim3(256), 0, (hipStream_t)stream, idx, S, f);
    return check_launch("gather_rows_kernel");
}

extern "C" int msat_cycle_metrics(int32_t N, const float *reward, const uint8_t *done, const uint8_t *solved,
                                  const int32_t *num_unsatisfied, const int32_t *episode_step, const float *targets,
                                  const float *vpred, double *out, void *stream) {
    MSAT_REQUIRE(N >= 0 && out, "cycle_metrics: bad args");
    MSAT_REQUIRE(N == 0 || (reward && done && solved && num_unsatisfied && episode_step && targets && vpred),
                 "cycle_metrics: NULL input");
    hipLaunchKernelGGL(cycle_metrics_kernel, dim3(1), dim3(kMetT), 0, (hipStream_t)stream, N, reward, done, solved,
                       num_unsatisfied, episode_step, targets, vpred, out);
    return check_launch("cycle_metrics_kernel");
}

extern "C" int msat_graph_bases(int32_t S, const int32_t *inst, const int32_t *nv, const int32_t *nc, const int32_t *ne,
                                int32_t *bases, int32_t *totals, void *stream) {
    MSAT_REQUIRE(S >= 0 && totals && (S == 0 || (inst && nv && nc && ne && bases)), "graph_bases: bad args");
    hipLaunchKernelGGL(graph_bases_kernel, dim3(1), dim3(kScanT), 0, (hipStream_t)stream, S, inst, nv, nc, ne, bases,
                       totals);
    return check_launch("graph_bases_kernel");
}
