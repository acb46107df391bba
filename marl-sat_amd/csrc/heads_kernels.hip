// Actor / critic heads, PPO loss, policy sampling and Adam (gfx950).
//
// Reference: src/learners/mappo_gnn_sat_learner.py
//   critic pooling + MLP          :340-350
//   actor pooling / local context :264-301,  flip / no-op heads :304-325 (mode 0), :327-335 (mode 1)
//   Categorical sample / log_prob :397-403 (distrax), entropy :637
//   PPO loss                      :597-645 (jnp.minimum / maximum / clip VJPs split ties 0.5/0.5)
//   Adam                          :650 + src/runners/mappo_runner.py:198 (optax.adam defaults)
// Graph-batch layout: sample s, graph g (0 = critic, 1+i = agent i) owns var rows
// [vbase, vbase+nv) and clause rows [cbase, cbase+nc); an agent graph lists its own
// vars first.  All reductions run in a fixed order (bitwise reproducible).
#include <math.h>

#include "common.h"

namespace msat {

struct GraphRef {
    const int *vbase, *nv, *cbase, *nc;  // (S*G) each
    int G;                               // graphs per sample
};

// ---------------------------------------------------------------- critic ----
// pooled (S, 6H) = [mean_v(2H) | max_v(2H) | mean_c(H) | max_c(H)] over graph 0 of each sample.
// The row loops of the pooling kernels are unrolled 8 deep so eight independent row loads fly per
// round trip (a plain loop waited on each load: one HBM latency per row); the accumulation order is
// unchanged, so the results are bit-identical.  Measured (uf100 x 4096 MAPPO leg, rocprof): critic
// pool 282 -> 91 us, its backward 753 -> 435 us, actor pool 577 -> 517 us; the actor pool backward (a
// read-modify-write stream over 8,200 blocks, already ~3.9 TB/s) ran 622 -> 700 us unrolled and is not.
__global__ void __launch_bounds__(256)
critic_pool_kernel(const float *__restrict__ Hp, const float *__restrict__ Hn, const float *__restrict__ Hc, int H,
                   GraphRef gr, float *__restrict__ pooled) {
    const int s = blockIdx.x, gid = s * gr.G;
    const int vb = gr.vbase[gid], nv = gr.nv[gid], cb = gr.cbase[gid], nc = gr.nc[gid];
    float *out = pooled + (size_t)s * 6 * H;
    for (int j = threadIdx.x; j < 3 * H; j += blockDim.x) {
        const bool var = j < 2 * H;
        const float *src;
        int ld = H, base, n, col;
        if (var) {
            src = j < H ? Hp : Hn;
            col = j < H ? j : j - H;
            base = vb;
            n = nv;
        } else {
            src = Hc;
            col = j - 2 * H;
            base = cb;
            n = nc;
        }
        float sum = 0.f, mx = -INFINITY;
        #pragma unroll 8
        for (int r = 0; r < n; ++r) {
            const float v = src[(size_t)(base + r) * ld + col];
            sum += v;
            mx = fmaxf(mx, v);
        }
        const float mean = sum / (float)n;
        if (var) {
            out[j] = mean;
            out[2 * H + j] = mx;
        } else {
            out[4 * H + col] = mean;
            out[5 * H + col] = mx;
        }
    }
}

// dHp/dHn/dHc (+)= grads of the critic pooling (max: ties split equally, jnp.max VJP).
__global__ void __launch_bounds__(256)
critic_pool_bwd_kernel(const float *__restrict__ Hp, const float *__restrict__ Hn, const float *__restrict__ Hc, int H,
                       GraphRef gr, const float *__restrict__ dpooled, float *__restrict__ dHp,
                       float *__restrict__ dHn, float *__restrict__ dHc) {
    const int s = blockIdx.x, gid = s * gr.G;
    const int vb = gr.vbase[gid], nv = gr.nv[gid], cb = gr.cbase[gid], nc = gr.nc[gid];
    const float *dp = dpooled + (size_t)s * 6 * H;
    for (int j = threadIdx.x; j < 3 * H; j += blockDim.x) {
        const bool var = j < 2 * H;
        const float *src;
        float *dst;
        int base, n, col;
        float dmean, dmax;
        if (var) {
            const bool pos = j < H;
            src = pos ? Hp : Hn;
            dst = pos ? dHp : dHn;
            col = pos ? j : j - H;
            base = vb;
            n = nv;
            dmean = dp[j];
            dmax = dp[2 * H + j];
        } else {
            src = Hc;
            dst = dHc;
            col = j - 2 * H;
            base = cb;
            n = nc;
            dmean = dp[4 * H + col];
            dmax = dp[5 * H + col];
        }
        float mx = -INFINITY;
        #pragma unroll 8
        for (int r = 0; r < n; ++r) mx = fmaxf(mx, src[(size_t)(base + r) * H + col]);
        int cnt = 0;
        #pragma unroll 8
        for (int r = 0; r < n; ++r) cnt += src[(size_t)(base + r) * H + col] == mx;
        const float gm = dmean / (float)n, gx = dmax / (float)cnt;
        #pragma unroll 8
        for (int r = 0; r < n; ++r) {
            const size_t i = (size_t)(base + r) * H + col;
            dst[i] += gm + (src[i] == mx ? gx : 0.f);
        }
    }
}

// ----------------------------------------------------------------- actor ----
// Block per (s, agent).  my_emb (S*A*M, 2H): own var rows (zeros in padded slots);
// ctx (S*A, 5H+E) = [mean own (2H) | mean nbr (2H) | mean clauses (H) | id embedding (E)].
__global__ void __launch_bounds__(256)
actor_pool_kernel(const float *__restrict__ Hp, const float *__restrict__ Hn, const float *__restrict__ Hc, int H,
                  GraphRef gr, int A, int M, int base_sz, int rem, const float *__restrict__ id_emb, int E,
                  float *__restrict__ my_emb, float *__restrict__ ctx) {
    const int sa = blockIdx.x, s = sa / A, i = sa - s * A;
    const int gid = s * gr.G + 1 + i;
    const int vb = gr.vbase[gid], nv = gr.nv[gid], cb = gr.cbase[gid], nc = gr.nc[gid];
    const int nown = base_sz + (i < rem ? 1 : 0);
    const int CW = 5 * H + E;
    float *cx = ctx + (size_t)sa * CW;
    for (int j = threadIdx.x; j < 2 * H; j += blockDim.x) {
        const float *src = j < H ? Hp : Hn;
        const int col = j < H ? j : j - H;
        float so = 0.f, sn = 0.f;
        #pragma unroll 8
        for (int r = 0; r < nv; ++r) {
            const float v = src[(size_t)(vb + r) * H + col];
            if (r < nown) {
                so += v;
                if (r < M) my_emb[((size_t)sa * M + r) * 2 * H + j] = v;
            } else {
                sn += v;
            }
        }
        #pragma unroll 8
        for (int r = nown; r < M; ++r) my_emb[((size_t)sa * M + r) * 2 * H + j] = 0.f;
        cx[j] = so / (float)max(nown, 1);
        cx[2 * H + j] = sn / (float)max(nv - nown, 1);
    }
    for (int j = threadIdx.x; j < H; j += blockDim.x) {
        float sc = 0.f;
        #pragma unroll 8
        for (int r = 0; r < nc; ++r) sc += Hc[(size_t)(cb + r) * H + j];
        cx[4 * H + j] = sc / (float)max(nc, 1);
    }
    for (int j = threadIdx.x; j < E; j += blockDim.x) cx[5 * H + j] = id_emb[i * E + j];
}

__global__ void __launch_bounds__(256)
actor_pool_bwd_kernel(int H, GraphRef gr, int A, int M, int base_sz, int rem, int E, const float *__restrict__ dmy,
                      const float *__restrict__ dctx, float *__restrict__ dHp, float *__restrict__ dHn,
                      float *__restrict__ dHc, float *__restrict__ did) {
    const int sa = blockIdx.x, s = sa / A, i = sa - s * A;
    const int gid = s * gr.G + 1 + i;
    const int vb = gr.vbase[gid], nv = gr.nv[gid], cb = gr.cbase[gid], nc = gr.nc[gid];
    const int nown = base_sz + (i < rem ? 1 : 0);
    const int CW = 5 * H + E;
    const float *dc = dctx + (size_t)sa * CW;
    for (int j = threadIdx.x; j < 2 * H; j += blockDim.x) {
        float *dst = j < H ? dHp : dHn;
        const int col = j < H ? j : j - H;
        const float go = dc[j] / (float)max(nown, 1), gn = dc[2 * H + j] / (float)max(nv - nown, 1);
        for (int r = 0; r < nv; ++r) {
            float g;
            if (r < nown)
                g = go + (r < M ? dmy[((size_t)sa * M + r) * 2 * H + j] : 0.f);
            else
                g = gn;
            dst[(size_t)(vb + r) * H + col] += g;
        }
    }
    for (int j = threadIdx.x; j < H; j += blockDim.x) {
        const float g = dc[4 * H + j] / (float)max(nc, 1);
        for (int r = 0; r < nc; ++r) dHc[(size_t)(cb + r) * H + j] += g;
    }
    for (int j = threadIdx.x; j < E; j += blockDim.x) did[(size_t)sa * E + j] = dc[5 * H + j];
}

// rows r of Q (R*M rows, grouped by M) += P[r / M]; optional relu.
__global__ void bcast_add_relu_kernel(float *__restrict__ Q, const float *__restrict__ P, int R, int M, int W) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)R * M * W) return;
    const size_t row = t / W, col = t - row * W;
    Q[t] = fmaxf(Q[t] + P[(row / M) * W + col], 0.0f);
}

// dP[r] = sum_{m<M} dQ[r*M + m]  (fixed order)
__global__ void group_sum_kernel(const float *__restrict__ dQ, int R, int M, int W, float *__restrict__ dP) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)R * W) return;
    const size_t r = t / W, col = t - r * W;
    float s = 0.f;
    for (int m = 0; m < M; ++m) s += dQ[(r * M + m) * W + col];
    dP[t] = s;
}

// logits (S*A, M+1) = [flip (M) | noop], padded slots (j >= size_i) = -inf (mode 0).
__global__ void assemble_logits_kernel(const float *__restrict__ flip, const float *__restrict__ noop, int SA, int A,
                                       int M, int base_sz, int rem, float *__restrict__ logits) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= SA * (M + 1)) return;
    const int r = t / (M + 1), j = t - r * (M + 1), i = r % A;
    const int n = base_sz + (i < rem ? 1 : 0);
    float v;
    if (j == M)
        v = noop[r];
    else
        v = j < n ? flip[(size_t)r * M + j] : -INFINITY;
    logits[t] = v;
}

// mode 1: logits (S*A*M, 2) with padded slots -inf
__global__ void mask_var_logits_kernel(float *__restrict__ logits, int SA, int A, int M, int base_sz, int rem) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= SA * M) return;
    const int r = t / M, j = t - r * M, i = r % A;
    const int n = base_sz + (i < rem ? 1 : 0);
    if (j >= n) logits[2 * (size_t)t] = logits[2 * (size_t)t + 1] = -INFINITY;
}

// split dlogits (S*A, M+1) -> dflip (S*A*M), dnoop (S*A)
__global__ void split_dlogits_kernel(const float *__restrict__ dl, int SA, int M, float *__restrict__ dflip,
                                     float *__restrict__ dnoop) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= SA * (M + 1)) return;
    const int r = t / (M + 1), j = t - r * (M + 1);
    if (j == M)
        dnoop[r] = dl[t];
    else
        dflip[(size_t)r * M + j] = dl[t];
}

// -------------------------------------------------------------- categorical --
// One wave per distribution row of width W (logits may hold -inf).
__device__ __forceinline__ void row_softmax_stats(const float *__restrict__ lg, int W, float &mx, float &lse) {
    const int lane = threadIdx.x & 63;
    float m = -INFINITY;
    for (int j = lane; j < W; j += 64) m = fmaxf(m, lg[j]);
    m = wave_max_f32(m);
    float s = 0.f;
    for (int j = lane; j < W; j += 64) s += __expf(lg[j] - m);
    s = wave_sum_f32(s);
    mx = m;
    lse = m + __logf(s);
}

// Gumbel-max sample (greedy=0) or argmax (greedy=1) + log_prob of the action.
__global__ void __launch_bounds__(256)
sample_kernel(const float *__restrict__ logits, int R, int W, int greedy, uint64_t seed, uint64_t ctr,
              int32_t *__restrict__ action, float *__restrict__ logp) {
    const int lane = threadIdx.x & 63;
    for (int r = blockIdx.x * 4 + (threadIdx.x >> 6); r < R; r += gridDim.x * 4) {
        const float *lg = logits + (size_t)r * W;
        float mx, lse;
        row_softmax_stats(lg, W, mx, lse);
        float best = -INFINITY;
        int bi = 0x7FFFFFFF;
        for (int j = lane; j < W; j += 64) {
            float v = lg[j];
            if (!greedy && v > -INFINITY) {
                const uint4 q = philox4x32_10(make_uint4((uint32_t)ctr, (uint32_t)(ctr >> 32), (uint32_t)r, (uint32_t)j),
                                              (uint32_t)seed, (uint32_t)(seed >> 32));
                const float u = ((float)(q.x >> 8) + 0.5f) * (1.0f / 16777216.0f);  // (0,1)
                v += -__logf(-__logf(u));
            }
            if (v > best || (v == best && j < bi)) {
                best = v;
                bi = j;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float ob = __shfl_xor(best, o, 64);
            const int oi = __shfl_xor(bi, o, 64);
            if (ob > best || (ob == best && oi < bi)) {
                best = ob;
                bi = oi;
            }
        }
        if (lane == 0) {
            action[r] = bi;
            // a row with no finite logit (mode-1 padded variable slot) stores log-prob 0: distrax gives
            // NaN there (-inf - logsumexp(-inf)), which would poison the PPO ratio
            logp[r] = mx > -INFINITY ? lg[bi] - lse : 0.f;
        }
    }
}

// -------------------------------------------------------------------- PPO ----
struct PpoCfg {
    float clip_eps, vf_clip, ent_coef, vf_coef;
    float inv_n_actor;  // 1 / (MB * A) (mode 0) ; 1 / (MB * A) for the joint ratio (mode 1)
    float inv_n_ent;    // 1 / (#entropy terms)
    float inv_n_value;  // 1 / MB
    int mode;           // action_mode
};

__device__ __forceinline__ float clip_grad(float r, float lo, float hi) {
    // d/dr jnp.clip(r, lo, hi) = min(max(r, lo), hi) with balanced ties
    const float a = r > lo ? 1.0f : (r == lo ? 0.5f : 0.0f);
    return r < hi ? a : (r == hi ? 0.5f * a : 0.0f);
}

// d/dr of -min(r*g, clip(r)*g) (jnp.minimum: ties 0.5/0.5)
__device__ __forceinline__ float surrogate_grad(float r, float g, float eps) {
    const float lo = 1.0f - eps, hi = 1.0f + eps;
    const float c = fminf(fmaxf(r, lo), hi);
    const float u = r * g, v = c * g;
    const float du = g, dv = g * clip_grad(r, lo, hi);
    const float d = u < v ? du : (v < u ? dv : 0.5f * (du + dv));
    return -d;
}

// Mode 0: one wave per (s, agent) row of width W = M+1.  Writes dlogits (scaled by
// 1/N), per-row actor / entropy terms; value terms by the lane-0 of agent 0 rows.
__global__ void __launch_bounds__(256)
ppo_loss_kernel(const float *__restrict__ logits, int R, int A, int W, const int32_t *__restrict__ action,
                const float *__restrict__ old_logp, const float *__restrict__ gae, const float *__restrict__ value,
                const float *__restrict__ old_value, const float *__restrict__ targets, PpoCfg cfg,
                float *__restrict__ dlogits, float *__restrict__ dvalue, float *__restrict__ row_terms) {
    const int lane = threadIdx.x & 63;
    for (int r = blockIdx.x * 4 + (threadIdx.x >> 6); r < R; r += gridDim.x * 4) {
        const float *lg = logits + (size_t)r * W;
        float *dl = dlogits + (size_t)r * W;
        const int s = r / A;
        float mx, lse;
        row_softmax_stats(lg, W, mx, lse);
        // entropy H = -sum p log p
        float h = 0.f;
        for (int j = lane; j < W; j += 64) {
            const float lp = lg[j] - lse;
            const float p = __expf(lp);
            h -= lg[j] > -INFINITY ? p * lp : 0.f;
        }
        h = wave_sum_f32(h);
        const int a = min(max(action[r], 0), W - 1);  // never index outside the row
        const float lpa = lg[a] - lse;
        const float ratio = __expf(lpa - old_logp[r]);
        const float g = gae[s];
        const float lo = 1.0f - cfg.clip_eps, hi = 1.0f + cfg.clip_eps;
        const float surr = -fminf(ratio * g, fminf(fmaxf(ratio, lo), hi) * g);
        const float dlpa = surrogate_grad(ratio, g, cfg.clip_eps) * ratio * cfg.inv_n_actor;
        const float dh = -cfg.ent_coef * cfg.inv_n_ent;
        for (int j = lane; j < W; j += 64) {
            float d = 0.f;
            if (lg[j] > -INFINITY) {
                const float lp = lg[j] - lse;
                const float p = __expf(lp);
                d = dlpa * ((j == a ? 1.0f : 0.0f) - p) + dh * (-p * (lp + h));
            }
            dl[j] = d;
        }
        if (lane == 0) {
            row_terms[2 * (size_t)r] = surr;
            row_terms[2 * (size_t)r + 1] = h;
            if (r % A == 0) {
                const float v = value[s], vo = old_value[s], t = targets[s];
                const float vc = vo + fminf(fmaxf(v - vo, -cfg.vf_clip), cfg.vf_clip);
                const float a1 = (v - t) * (v - t), a2 = (vc - t) * (vc - t);
                const float dvc = clip_grad(v - vo, -cfg.vf_clip, cfg.vf_clip);
                const float g1 = 2.0f * (v - t), g2 = 2.0f * (vc - t) * dvc;
                const float gm = a1 > a2 ? g1 : (a2 > a1 ? g2 : 0.5f * (g1 + g2));
                dvalue[s] = cfg.vf_coef * 0.5f * gm * cfg.inv_n_value;
                row_terms[2 * (size_t)R + s] = 0.5f * fmaxf(a1, a2);
            }
        }
    }
}

// Mode 1: per (s, agent) the M binary variables; joint log-prob = sum over valid vars.
__global__ void __launch_bounds__(256)
ppo_loss_multi_kernel(const float *__restrict__ logits, int R, int A, int M, int base_sz, int rem,
                      const int32_t *__restrict__ action, const float *__restrict__ old_logp,
                      const float *__restrict__ gae, const float *__restrict__ value,
                      const float *__restrict__ old_value, const float *__restrict__ targets, PpoCfg cfg,
                      float *__restrict__ dlogits, float *__restrict__ dvalue, float *__restrict__ row_terms) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;  // one thread per (s, agent)
    if (r >= R) return;
    const int s = r / A, i = r - s * A;
    const int n = base_sz + (i < rem ? 1 : 0);
    float lp_new = 0.f, lp_old = 0.f, hsum = 0.f;
    for (int j = 0; j < M; ++j) {
        const float *lg = logits + ((size_t)r * M + j) * 2;
        if (j >= n) {
            // padded slot, both logits -inf: distrax log_prob / entropy are NaN there in JAX, which
            // would turn the joint ratio and every gradient into NaN.  The slot contributes 0 to the
            // joint log-probs (new and old, whatever the caller stored) and to the entropy.
            continue;
        }
        lp_old += old_logp[(size_t)r * M + j];
        const float m = fmaxf(lg[0], lg[1]);
        const float lse = m + __logf(__expf(lg[0] - m) + __expf(lg[1] - m));
        const int a = action[(size_t)r * M + j] & 1;
        lp_new += lg[a] - lse;
        const float p0 = __expf(lg[0] - lse), p1 = __expf(lg[1] - lse);
        hsum -= p0 * (lg[0] - lse) + p1 * (lg[1] - lse);
    }
    const float ratio = __expf(lp_new - lp_old);
    const float g = gae[s];
    const float lo = 1.0f - cfg.clip_eps, hi = 1.0f + cfg.clip_eps;
    const float surr = -fminf(ratio * g, fminf(fmaxf(ratio, lo), hi) * g);
    const float dlp = surrogate_grad(ratio, g, cfg.clip_eps) * ratio * cfg.inv_n_actor;
    const float dh = -cfg.ent_coef * cfg.inv_n_ent;
    for (int j = 0; j < M; ++j) {
        const float *lg = logits + ((size_t)r * M + j) * 2;
        float *dl = dlogits + ((size_t)r * M + j) * 2;
        if (j >= n) {
            dl[0] = dl[1] = 0.f;
            continue;
        }
        const float m = fmaxf(lg[0], lg[1]);
        const float lse = m + __logf(__expf(lg[0] - m) + __expf(lg[1] - m));
        const float l0 = lg[0] - lse, l1 = lg[1] - lse, p0 = __expf(l0), p1 = __expf(l1);
        const float hj = -(p0 * l0 + p1 * l1);
        const int a = action[(size_t)r * M + j] & 1;
        dl[0] = dlp * ((a == 0 ? 1.f : 0.f) - p0) + dh * (-p0 * (l0 + hj));
        dl[1] = dlp * ((a == 1 ? 1.f : 0.f) - p1) + dh * (-p1 * (l1 + hj));
    }
    row_terms[2 * (size_t)r] = surr;
    row_terms[2 * (size_t)r + 1] = hsum;
    if (i == 0) {
        const float v = value[s], vo = old_value[s], t = targets[s];
        const float vc = vo + fminf(fmaxf(v - vo, -cfg.vf_clip), cfg.vf_clip);
        const float a1 = (v - t) * (v - t), a2 = (vc - t) * (vc - t);
        const float dvc = clip_grad(v - vo, -cfg.vf_clip, cfg.vf_clip);
        const float g1 = 2.0f * (v - t), g2 = 2.0f * (vc - t) * dvc;
        const float gm = a1 > a2 ? g1 : (a2 > a1 ? g2 : 0.5f * (g1 + g2));
        dvalue[s] = cfg.vf_coef * 0.5f * gm * cfg.inv_n_value;
        row_terms[2 * (size_t)R + s] = 0.5f * fmaxf(a1, a2);
    }
}

// sums[0..2] += (value_loss_sum, actor_surrogate_sum, entropy_sum) in fp64, fixed order
__global__ void __launch_bounds__(256)
loss_sums_kernel(const float *__restrict__ row_terms, int R, int S, double *__restrict__ sums) {
    __shared__ double red[3][256];
    double a = 0, e = 0, v = 0;
    for (int r = threadIdx.x; r < R; r += 256) {
        a += row_terms[2 * (size_t)r];
        e += row_terms[2 * (size_t)r + 1];
    }
    for (int s = threadIdx.x; s < S; s += 256) v += row_terms[2 * (size_t)R + s];
    red[0][threadIdx.x] = v;
    red[1][threadIdx.x] = a;
    red[2][threadIdx.x] = e;
    __syncthreads();
    if (threadIdx.x < 3) {
        double t = 0;
        for (int k = 0; k < 256; ++k) t += red[threadIdx.x][k];
        sums[threadIdx.x] += t;
    }
}

// ------------------------------------------------------------------- Adam ----
// optax.adam: m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2; p -= lr * mhat / (sqrt(vhat) + eps)
// first_bad (nullable): atomicMin(first_bad, count) where an updated parameter is not finite (a
// vector-memory atomic on the rare failing lanes; the common path adds one compare)
__global__ void adam_kernel(float *__restrict__ p, const float *__restrict__ g, float *__restrict__ m,
                            float *__restrict__ v, size_t n, float lr, float b1, float b2, float eps, float bc1,
                            float bc2, float gscale, int *__restrict__ first_bad, int count) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float gi = g[i] * gscale;
    const float mi = b1 * m[i] + (1.0f - b1) * gi;
    const float vi = b2 * v[i] + (1.0f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float mh = mi / bc1, vh = vi / bc2;
    const float pn = p[i] + (-lr) * (mh / (sqrtf(vh) + eps));
    p[i] = pn;
    if (first_bad && !isfinite(pn)) atomicMin(first_bad, count);
}

}  // namespace msat

using namespace msat;

static GraphRef make_gr(const int32_t *vbase, const int32_t *nv, const int32_t *cbase, const int32_t *nc, int G) {
    GraphRef g;
    g.vbase = vbase;
    g.nv = nv;
    g.cbase = cbase;
    g.nc = nc;
    g.G = G;
    return g;
}

static unsigned blocks_for(size_t n, int t = 256) { return (unsigned)((n + t - 1) / t); }

extern "C" int msat_critic_pool(const float *Hp, const float *Hn, const float *Hc, int32_t H, const int32_t *vbase,
                                const int32_t *nv, const int32_t *cbase, const int32_t *nc, int32_t G, int32_t S,
                                float *pooled, void *stream) {
    MSAT_REQUIRE(Hp && Hn && Hc && vbase && nv && cbase && nc && pooled && S >= 0 && G >= 1, "bad critic_pool args");
    if (!S) return MSAT_OK;
    hipLaunchKernelGGL(critic_pool_kernel, dim3(S), dim3(256), 0, (hipStream_t)stream, Hp, Hn, Hc, H,
                       make_gr(vbase, nv, cbase, nc, G), pooled);
    return check_launch("critic_pool_kernel");
}

extern "C" int msat_critic_pool_bwd(const float *Hp, const float *Hn, const float *Hc, int32_t H, const int32_t *vbase,
                                    const int32_t *nv, const int32_t *cbase, const int32_t *nc, int32_t G, int32_t S,
                                    const float *dpooled, float *dHp, float *dHn, float *dHc, void *stream) {
    MSAT_REQUIRE(Hp && Hn && Hc && dpooled && dHp && dHn && dHc, "bad critic_pool_bwd args");
    if (!S) return MSAT_OK;
    hipLaunchKernelGGL(critic_pool_bwd_kernel, dim3(S), dim3(256), 0, (hipStream_t)stream, Hp, Hn, Hc, H,
                       make_gr(vbase, nv, cbase, nc, G), dpooled, dHp, dHn, dHc);
    return check_launch("critic_pool_bwd_kernel");
}

extern "C" int msat_actor_pool(const float *Hp, const float *Hn, const float *Hc, int32_t H, const int32_t *vbase,
                               const int32_t *nv, const int32_t *cbase, const int32_t *nc, int32_t G, int32_t S,
                               int32_t A, int32_t M, int32_t base_sz, int32_t rem, const float *id_emb, int32_t E,
                               float *my_emb, float *ctx, void *stream) {
    MSAT_REQUIRE(Hp && Hn && Hc && id_emb && my_emb && ctx && G == A + 1, "bad actor_pool args");
    if (!S) return MSAT_OK;
    hipLaunchKernelGGL(actor_pool_kernel, dim3(S * A), dim3(256), 0, (hipStream_t)stream, Hp, Hn, Hc, H,
                       make_gr(vbase, nv, cbase, nc, G), A, M, base_sz, rem, id_emb, E, my_emb, ctx);
    return check_launch("actor_pool_kernel");
}

extern "C" int msat_actor_pool_bwd(int32_t H, const int32_t *vbase, const int32_t *nv, const int32_t *cbase,
                                   const int32_t *nc, int32_t G, int32_t S, int32_t A, int32_t M, int32_t base_sz,
                                   int32_t rem, int32_t E, const float *dmy, const float *dctx, float *dHp, float *dHn,
                                   float *dHc, float *did, void *stream) {
    MSAT_REQUIRE(dmy && dctx && dHp && dHn && dHc && did && G == A + 1, "bad actor_pool_bwd args");
    if (!S) return MSAT_OK;
    hipLaunchKernelGGL(actor_pool_bwd_kernel, dim3(S * A), dim3(256), 0, (hipStream_t)stream, H,
                       make_gr(vbase, nv, cbase, nc, G), A, M, base_sz, rem, E, dmy, dctx, dHp, dHn, dHc, did);
    return check_launch("actor_pool_bwd_kernel");
}

extern "C" int msat_bcast_add_relu(float *Q, const float *P, int32_t R, int32_t M, int32_t W, void *stream) {
    MSAT_REQUIRE(Q && P, "NULL pointer");
    const size_t n = (size_t)R * M * W;
    if (!n) return MSAT_OK;
    hipLaunchKernelGGL(bcast_add_relu_kernel, dim3(blocks_for(n)), dim3(256), 0, (hipStream_t)stream, Q, P, R, M, W);
    return check_launch("bcast_add_relu_kernel");
}

extern "C" int msat_group_sum(const float *dQ, int32_t R, int32_t M, int32_t W, float *dP, void *stream) {
    MSAT_REQUIRE(dQ && dP, "NULL pointer");
    const size_t n = (size_t)R * W;
    if (!n) return MSAT_OK;
    hipLaunchKernelGGL(group_sum_kernel, dim3(blocks_for(n)), dim3(256), 0, (hipStream_t)stream, dQ, R, M, W, dP);
    return check_launch("group_sum_kernel");
}

extern "C" int msat_assemble_logits(const float *flip, const float *noop, int32_t SA, int32_t A, int32_t M,
                                    int32_t base_sz, int32_t rem, float *logits, void *stream) {
    MSAT_REQUIRE(flip && noop && logits, "NULL pointer");
    const size_t n = (size_t)SA * (M + 1);
    if (!n) return MSAT_OK;
    hipLaunchKernelGGL(assemble_logits_kernel, dim3(blocks_for(n)), dim3(256), 0, (hipStream_t)stream, flip, noop, SA,
                       A, M, base_sz, rem, logits);
    return check_launch("assemble_logits_kernel");
}

extern "C" int msat_mask_var_logits(float *logits, int32_t SA, int32_t A, int32_t M, int32_t base_sz, int32_t rem,
                                    void *stream) {
    MSAT_REQUIRE(logits, "NULL pointer");
    const size_t n = (size_t)SA * M;
    if (!n) return MSAT_OK;
    hipLaunchKernelGGL(mask_var_logits_kernel, dim3(blocks_for(n)), dim3(256), 0, (hipStream_t)stream, logits, SA, A,
                       M, base_sz, rem);
    return check_launch("mask_var_logits_kernel");
}

extern "C" int msat_split_dlogits(const float *dlogits, int32_t SA, int32_t M, float *dflip, float *dnoop,
                                  void *stream) {
    MSAT_REQUIRE(dlogits && dflip && dnoop, "NULL pointer");
    const size_t n = (size_t)SA * (M + 1);
    if (!n) return MSAT_OK;
    hipLaunchKernelGGL(split_dlogits_kernel, dim3(blocks_for(n)), dim3(256), 0, (hipStream_t)stream, dlogits, SA, M,
                       dflip, dnoop);
    return check_launch("split_dlogits_kernel");
}

extern "C" int msat_sample_actions(const float *logits, int32_t R, int32_t W, int32_t greedy, uint64_t seed,
                                   uint64_t counter, int32_t *action, float *logp, void *stream) {
    MSAT_REQUIRE(logits && action && logp && W >= 1, "bad sample args");
    if (!R) return MSAT_OK;
    hipLaunchKernelGGL(sample_kernel, dim3(std::min(8192, (R + 3) / 4)), dim3(256), 0, (hipStream_t)stream, logits, R,
                       W, greedy, seed, counter, action, logp);
    return check_launch("sample_kernel");
}

extern "C" int msat_ppo_loss(const float *logits, int32_t S, int32_t A, int32_t M, int32_t action_mode,
                             int32_t base_sz, int32_t rem, const int32_t *action, const float *old_logp,
                             const float *gae, const float *value, const float *old_value, const float *targets,
                             float clip_eps, float vf_clip, float ent_coef, float vf_coef, int32_t minibatch,
                             float *dlogits, float *dvalue, float *row_terms, double *loss_sums, void *stream) {
    MSAT_REQUIRE(logits && action && old_logp && gae && value && old_value && targets && dlogits && dvalue &&
                     row_terms && loss_sums && minibatch >= 1,
                 "bad ppo_loss args");
    if (!S) return MSAT_OK;
    PpoCfg c;
    c.clip_eps = clip_eps;
    c.vf_clip = vf_clip;
    c.ent_coef = ent_coef;
    c.vf_coef = vf_coef;
    c.inv_n_actor = 1.0f / ((float)minibatch * (float)A);
    c.inv_n_ent = action_mode == 0 ? 1.0f / ((float)minibatch * (float)A) : 1.0f / ((float)minibatch * A * M);
    c.inv_n_value = 1.0f / (float)minibatch;
    c.mode = action_mode;
    const int R = S * A;
    hipStream_t s = (hipStream_t)stream;
    if (action_mode == 0)
        hipLaunchKernelGGL(ppo_loss_kernel, dim3(std::min(8192, (R + 3) / 4)), dim3(256), 0, s, logits, R, A, M + 1,
                           action, old_logp, gae, value, old_value, targets, c, dlogits, dvalue, row_terms);
    else
        hipLaunchKernelGGL(ppo_loss_multi_kernel, dim3((R + 255) / 256), dim3(256), 0, s, logits, R, A, M, base_sz,
                           rem, action, old_logp, gae, value, old_value, targets, c, dlogits, dvalue, row_terms);
    int rc = check_launch("ppo_loss_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(loss_sums_kernel, dim3(1), dim3(256), 0, s, row_terms, R, S, loss_sums);
    return check_launch("loss_sums_kernel");
}

extern "C" int msat_adam_checked(float *params, const float *grads, float *m, float *v, size_t n, float lr, float b1,
                                 float b2, float eps, int32_t count, float grad_scale, int32_t *first_bad,
                                 void *stream) {
    MSAT_REQUIRE(params && grads && m && v && count >= 1, "bad adam args");
    if (!n) return MSAT_OK;
    const float bc1 = (float)(1.0 - pow((double)b1, (double)count));
    const float bc2 = (float)(1.0 - pow((double)b2, (double)count));
    hipLaunchKernelGGL(adam_kernel, dim3(blocks_for(n)), dim3(256), 0, (hipStream_t)stream, params, grads, m, v, n, lr,
                       b1, b2, eps, bc1, bc2, grad_scale, first_bad, count);
    return check_launch("adam_kernel");
}

extern "C" int msat_adam(float *params, const float *grads, float *m, float *v, size_t n, float lr, float b1, float b2,
                         float eps, int32_t count, float grad_scale, void *stream) {
    return msat_adam_checked(params, grads, m, v, n, lr, b1, b2, eps, count, grad_scale, nullptr, stream);
}
