/*
 * marlsat_net.h — C-ABI of the MAPPO network / update kernels in libmarlsat.so
 * (gfx950).  Same conventions as marlsat.h: device pointers owned by the caller,
 * explicit dims, stream last, 0 on success / negative + msat_last_error().
 *
 * Reference computations replaced (kongqg/marl-sat):
 *   msat_gemm / msat_gemm_wgrad  <- every flax nn.Dense / nn.GRUCell matmul of
 *        GNN_ActorCritic (src/learners/mappo_gnn_sat_learner.py:44-80, :213-240,
 *        :311-349) and their jax.value_and_grad transposes (:647-649)
 */
#ifndef MARLSAT_NET_H
#define MARLSAT_NET_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* C[M,N] (+)= A[M,K] @ op(B) (+ bias[N]); op(B) = B[K,N] (transB=0) or B[N,K]^T (transB=1).
 * Row-major with leading dims; fp32 in / fp32 accumulate on the matrix cores. */
int msat_gemm(const float *A, int32_t lda, const float *B, int32_t ldb, int32_t transB, float *C,
              int32_t ldc, const float *bias, int32_t M, int32_t N, int32_t K, int32_t accumulate,
              void *stream);

/* C[M,N] (+)= op(A)[M,K] @ op(B)[K,N], fp32 operands, fp64 accumulation, one rounding per
 * element; op(A) = A[M,K] (transA=0) or A[K,M]^T, op(B) = B[K,N] (transB=0) or B[N,K]^T.
 * For the small folded-weight products of the phi folding (F = W Wi per forward, dW = dF Wi^T and
 * dWi = W^T dF per backward) that stand in for the reference's separate Dense layers
 * (src/learners/mappo_gnn_sat_learner.py:66-79). */
int msat_gemm_f64acc(const float *A, int32_t lda, int32_t transA, const float *B, int32_t ldb, int32_t transB,
                     float *C, int32_t ldc, int32_t M, int32_t N, int32_t K, int32_t accumulate, void *stream);

/* fp32 GEMM on the bf16 matrix cores (gemm_x3.hip): operands split exactly into three bf16
 * parts, six bf16 MFMAs per 16-deep k step keep every product term above fp32 rounding.
 * msat_split_bf16x3: planes (3 x rows x cols bf16, contiguous) of W (rows x cols, ldw).
 * msat_gemm_x3: C[M,N] (+)= A[M,K] @ W^T (+ bias), W [N][K] given as its split planes;
 *   K % 16 == 0, lda % 4 == 0, 16-byte aligned A / planes. */
int msat_split_bf16x3(const float *W, int32_t rows, int32_t cols, int32_t ldw, void *planes, void *stream);
/* the same with the columns rotated: planes[q][r][c] = part q of W[r][(c + rot) % cols] */
int msat_split_bf16x3_rot(const float *W, int32_t rows, int32_t cols, int32_t ldw, int32_t rot, void *planes,
                          void *stream);
int msat_gemm_x3(const float *A, int32_t lda, const void *Wplanes, float *C, int32_t ldc, const float *bias,
                 int32_t M, int32_t N, int32_t K, int32_t accumulate, void *stream);
/* fp16x2 form of msat_gemm_x3 for A = a GRU backward's packed rows with their row scale exponents
 * (rexp, msat_gru_ln_bwd_g4fe): three fp16 MFMAs per product.  Wplanes_h2 = msat_split_f16x2_rot of W
 * (fp16x2 planes of 2^10 W, *wbad = 1 if that overflowed), Wplanes_x3 = msat_split_bf16x3_rot of the
 * same W: with *wbad set the kernel runs the bf16x3 product instead.  K % 32 == 0. */
int msat_split_f16x2_rot(const float *W, int32_t rows, int32_t cols, int32_t ldw, int32_t rot, void *planes,
                         int32_t *wbad, void *stream);
/* Both data gradients of a GRU cell's packed backward rows in one launch: C0 (+)= A0 @ W0^T (N0 columns)
 * and C1 (+)= A1 @ W1^T (N1) over the same M rows (row exponents rexp), each as msat_gemm_h2. */
int msat_gemm_h2_dual(const float *A0, int32_t lda0, const void *W0_h2, const void *W0_x3, const int32_t *wbad0,
                      float *C0, int32_t ldc0, int32_t N0, int32_t acc0, const float *A1, int32_t lda1,
                      const void *W1_h2, const void *W1_x3, const int32_t *wbad1, float *C1, int32_t ldc1, int32_t N1,
                      int32_t acc1, const int32_t *rexp, int32_t M, int32_t K, void *stream);
/* The same with A0 / A1 the packed rows as fp16x2 planes (msat_gru_ln_bwd_g4fe with flags bit 3): lda in
 * fp16 elements (% 8), the lo plane plo elements after the hi plane (% 8); the rows are taken as split.
 * Bitwise the result of msat_gemm_h2_dual on the fp32 rows (the planes are the split it would make). */
int msat_gemm_h2_dual_planes(const void *A0, int32_t lda0, const void *W0_h2, const void *W0_x3,
                             const int32_t *wbad0, float *C0, int32_t ldc0, int32_t N0, int32_t acc0, const void *A1,
                             int32_t lda1, const void *W1_h2, const void *W1_x3, const int32_t *wbad1, float *C1,
                             int32_t ldc1, int32_t N1, int32_t acc1, int32_t plo, const int32_t *rexp, int32_t M,
                             int32_t K, void *stream);
int msat_gemm_h2(const float *A, int32_t lda, const int32_t *rexp, const void *Wplanes_h2, const void *Wplanes_x3,
                 const int32_t *wbad, float *C, int32_t ldc, const float *bias, int32_t M, int32_t N, int32_t K,
                 int32_t accumulate, void *stream);

/* W[K,N] (+)= A[M,K]^T @ G[M,N]: split over M, partial slabs reduced in a fixed order.
 * K <= 8 (feature / degree columns) streams G once instead of running 128-row MFMA tiles. */
size_t msat_gemm_wgrad_workspace_bytes(int32_t M, int32_t K, int32_t N);
int msat_gemm_wgrad(const float *A, int32_t lda, const float *G, int32_t ldg, float *W, int32_t ldw,
                    int32_t M, int32_t K, int32_t N, int32_t accumulate, void *workspace, void *stream);
/* W[:, (n + rot) % N] (+)= (A^T G)[:, n], 0 <= rot < N: the packed GRU backward rows' gate blocks
 * (n | r | z) into a weight stored (r | z | n) in one pass (learner:62-80 update cells' input rows). */
/* The same in fp16x2 (three fp16 MFMAs per product) for G = a GRU backward's packed rows with their
 * row scale exponents rexp (msat_gru_ln_bwd_g4fe): K > 8, N <= 384, rot % 4 == 0. */
int msat_gemm_wgrad_h2(const float *A, int32_t lda, const float *G, int32_t ldg, const int32_t *rexp, float *W,
                       int32_t ldw, int32_t M, int32_t K, int32_t N, int32_t rot, int32_t accumulate, void *workspace,
                       void *stream);
/* Both weight gradients of a GRU cell's packed backward rows in one fp16x2 launch: W0 (+)= A0^T G0 and
 * W1 (+)= A1^T G1 (columns rotated by rot0 / rot1) over the same M rows, row exponents rexp. */
size_t msat_gemm_wgrad_dual_workspace_bytes(int32_t M, int32_t K0, int32_t N0, int32_t K1, int32_t N1);
int msat_gemm_wgrad_h2_dual(const float *A0, int32_t lda0, const float *G0, int32_t ldg0, float *W0, int32_t ldw0,
                            int32_t K0, int32_t N0, int32_t rot0, const float *A1, int32_t lda1, const float *G1,
                            int32_t ldg1, float *W1, int32_t ldw1, int32_t K1, int32_t N1, int32_t rot1,
                            const int32_t *rexp, int32_t M, int32_t accumulate, void *workspace, void *stream);
/* The same with G0 / G1 the packed rows as fp16x2 planes (msat_gru_ln_bwd_g4fe, flags bit 3): ldg in fp16
 * elements (% 8), the lo plane plo elements after the hi plane (% 8, >= N), N % 8 == 0.  G is staged by
 * LDS-DMA with no split; the split-wide scale moves to A (a 2^(ge - e_r)). */
int msat_gemm_wgrad_h2_dual_planes(const float *A0, int32_t lda0, const void *G0, int32_t ldg0, float *W0,
                                   int32_t ldw0, int32_t K0, int32_t N0, int32_t rot0, const float *A1, int32_t lda1,
                                   const void *G1, int32_t ldg1, float *W1, int32_t ldw1, int32_t K1, int32_t N1,
                                   int32_t rot1, int32_t plo, const int32_t *rexp, int32_t M, int32_t accumulate,
                                   void *workspace, void *stream);
int msat_gemm_wgrad_rot(const float *A, int32_t lda, const float *G, int32_t ldg, float *W, int32_t ldw,
                        int32_t M, int32_t K, int32_t N, int32_t rot, int32_t accumulate, void *workspace,
                        void *stream);
/* Arithmetic path of msat_gemm_wgrad / msat_gemm_wgrad_rot: MSAT_PRECISION_FP16X2 (default) and
 * MSAT_PRECISION_BF16X3 run the fp32-accurate split kernels, MSAT_PRECISION_FP32 the fp32 MFMA tiles.
 * Set once per process (the Python host calls it at import with its validated MARLSAT_PRECISION);
 * until then the library reads MARLSAT_PRECISION once, and an unknown value there makes every weight
 * gradient fail with MSAT_EBADARG instead of picking a path.  Unknown `mode`: MSAT_EBADARG. */
#define MSAT_PRECISION_FP16X2 0
#define MSAT_PRECISION_BF16X3 1
#define MSAT_PRECISION_FP32 2
int msat_set_precision(int32_t mode);
int msat_get_precision(void); /* the mode in force, or MSAT_EBADARG if MARLSAT_PRECISION is unknown */

/* ---- graph batch assembly (learner:148-195 features + the agents' local graphs) ----
 * Block per sample: instantiate the per-instance templates (marlsat/learners/graphs.py) at the
 * sample's row bases (sample_bases (S,3) = var row, clause row, incidence starts) and compute the
 * node features from the sample's assignment x (S,V): vfeat (Nv,8) = [x, deg+/C, deg-/C, 0, n+, n-, 0, 0]
 * (static var features, then the var row's positive / negative incidence counts in its graph),
 * cfeat (Nc,3) = [is_sat, ntrue/3, 1], cdeg (Nc,4, nullable) = [n+, n-, 0, 0] positive / negative
 * literal slots of the clause row.  The counts carry the phi biases through the gather-first
 * message passing (sum_{edges} (h W + b) = (sum h) W + n b).  G = 1 (critic graph only) or A+1. */
int msat_assemble_graph_batch(
    int32_t S, int32_t G, int32_t A, int32_t V, int32_t C, const int32_t *inst, const uint8_t *x, const float *svf,
    const uint16_t *pool, const int32_t *sample_bases, const int32_t *t_vgid, const int32_t *t_cgid,
    const int32_t *t_slots, const int32_t *t_ptr, const int32_t *t_inc, const int32_t *voff, const int32_t *coff,
    const int32_t *eoff, const int32_t *poff, const int32_t *gv, const int32_t *gc, float *vfeat, float *cfeat,
    float *cdeg, int32_t *slots, int32_t *ptr, int32_t *inc, int32_t *g_vbase, int32_t *g_nv, int32_t *g_cbase, int32_t *g_nc,
    int32_t Nv, int32_t nnz, void *stream);

/* ---- message passing: signed literal gathers (the encoder's A^T M and A M, learner:66-74) ----
 * clause_gather: dst[c] (+)= [sum_{pos slots} src[v][0:H] | sum_{neg slots} src[v][H:2H]],
 *                slots (Nc,3) = (var_row << 1) | neg, or -1.
 * var_gather:    dst[v] (+)= [sum_{pos entries} src[c][0:H] | sum_{neg entries} src[c][H:2H]],
 *                CSR ptr (Nv+1), entries (clause_row << 1) | neg.  Each is the other's transpose. */
int msat_clause_gather(const float *src, int32_t ld_src, const int32_t *slots, float *dst, int32_t ld_dst,
                       int32_t num_clause_rows, int32_t H, int32_t accumulate, void *stream);
int msat_var_gather(const float *src, int32_t ld_src, const int32_t *ptr, const int32_t *inc, float *dst,
                    int32_t ld_dst, int32_t num_var_rows, int32_t H, int32_t accumulate, void *stream);
/* General forms (16-byte aligned rows, H % 32 == 0):
 * clause_gather2: positive slots read src_pos rows, negative slots src_neg rows (H wide each);
 *   merged = 0: dst[c] (+)= [sum_pos src_pos[v] | sum_neg src_neg[v]] (2H wide);
 *   merged = 1: dst[c] (+)= sum_pos src_pos[v] + sum_neg src_neg[v] (H wide; the transpose of
 *   var_gather2 with src_pos == src_neg).
 * var_gather2: dst_pos[v] (+)= sum_pos src_pos[c], dst_neg[v] (+)= sum_neg src_neg[c]. */
int msat_clause_gather2(const float *src_pos, const float *src_neg, int32_t ld_src, const int32_t *slots, float *dst,
                        int32_t ld_dst, int32_t num_clause_rows, int32_t H, int32_t merged, int32_t accumulate,
                        void *stream);
int msat_var_gather2(const float *src_pos, const float *src_neg, int32_t ld_src, const int32_t *ptr,
                     const int32_t *inc, float *dst_pos, float *dst_neg, int32_t ld_dst, int32_t num_var_rows,
                     int32_t H, int32_t accumulate, void *stream);

/* ---- fused flax GRUCell + LayerNorm (learner:69-80) ----
 * Gi = x Wi + bi, Gh = h Wh + [0,0,b_hn] (gates [r|z|n]); out = LN(GRU(h, x)).
 * Backward: dGi, dGh, dhprev (+=), LN scale/bias grads ([scale|bias] contiguous, (+)=). */
int msat_gru_ln_fwd(const float *Gi, int32_t ldi, const float *Gh, int32_t ldh, const float *hprev,
                    int32_t ldp, const float *ln_scale, const float *ln_bias, float *out, int32_t ldo,
                    int32_t R, int32_t H, void *stream);
size_t msat_gru_ln_bwd_partial_floats(int32_t R, int32_t H);
int msat_gru_ln_bwd(const float *dy, int32_t ldy, const float *Gi, int32_t ldi, const float *Gh, int32_t ldh,
                    const float *hprev, int32_t ldp, const float *ln_scale, float *dGi, int32_t lddi,
                    float *dGh, int32_t lddh, float *dhprev, int32_t lddp, float *dln_scale,
                    float *dln_bias, float *partial, int32_t R, int32_t H, int32_t accumulate_ln,
                    void *stream);
/* One kernel per GRU call on the fp32 matrix cores (gru_fused.hip): x = [x0 | x1 | x2]
 * (segment widths multiples of 4, 16-byte aligned rows; w1/w2 may be 0), Wi (Kx, 3H),
 * Wh (H, 3H), bi/bh (3H), out = LN(GRU(hprev, x)).  g4 (nullable, ldg >= 4H) receives the
 * pre-activations [r_pre | z_pre | gin | ghn] for msat_gru_ln_bwd_g4.
 * Replaces the two gate GEMMs + msat_gru_ln_fwd of update_c / update_v_pos / update_v_neg
 * + LayerNorm_k (learner:68-80). */
int msat_gru_ln_fused_fwd(const float *x0, int32_t ld0, int32_t w0, const float *x1, int32_t ld1, int32_t w1,
                          const float *x2, int32_t ld2, int32_t w2, const float *hprev, int32_t ldp,
                          const float *wi, const float *bi, const float *wh, const float *bh,
                          const float *ln_scale, const float *ln_bias, float *out, int32_t ldo, float *g4,
                          int32_t ldg, int32_t R, int32_t H, void *stream);
/* Same cell on the bf16 matrix cores (exact bf16x3 split, fp32-accurate; H = 128; register-A on
 * 16x16x32 bf16 MFMAs: activations read straight into registers, only the weights staged): weights given as msat_split_bf16x3_t planes of Wi^T zero-padded
 * to kxp columns (kxp >= Kx, multiple of 32) and of Wh^T (kxp = H).  g4 rows 16-byte aligned. */
int msat_gru_ln_fused_fwd_x3r(const float *x0, int32_t ld0, int32_t w0, const float *x1, int32_t ld1, int32_t w1,
                              const float *x2, int32_t ld2, int32_t w2, const float *hprev, int32_t ldp,
                              const void *wiT_planes, int32_t kxp, const float *bi, const void *whT_planes,
                              const float *bh, const float *ln_scale, const float *ln_bias, float *out, int32_t ldo,
                              float *g4, int32_t ldg, int32_t R, int32_t H, void *stream);
/* planes[q][n][k] = bf16x3 part q of (k < K ? W[k][n] : 0) for n < N, k < Kp: the transposed,
 * zero-padded split of a (K, N) weight (row stride ldw) for msat_gru_ln_fused_fwd_x3r. */
int msat_split_bf16x3_t(const float *W, int32_t K, int32_t N, int32_t ldw, int32_t Kp, void *planes, void *stream);
/* The same GRU cell with fp16x2 operands (x = x1 + x2, three fp16 MFMAs per product instead of six
 * bf16 ones; weights from msat_split_f16x2_t, scaled by 2^10; activations scaled by 2^7 before their split so
 * that small ones keep 22 bits).  fp16's range is checked per 128-row tile: a tile whose activations reach
 * |a| >= 256 (2^15 after the scale), or every tile when a weight split flagged wbad[0]
 * (wi) or wbad[1] (wh), is recomputed by the bf16x3 kernel from wiT_x3 / whT_x3 (msat_split_bf16x3_t
 * planes) in a second launch on the same stream.  tile_flags: >= ceil(R / 128) ints of workspace. */
int msat_gru_ln_fused_fwd_h2r(const float *x0, int32_t ld0, int32_t w0, const float *x1, int32_t ld1, int32_t w1,
                              const float *x2, int32_t ld2, int32_t w2, const float *hprev, int32_t ldp,
                              const void *wiT_h2, const void *whT_h2, const void *wiT_x3, const void *whT_x3,
                              int32_t kxp, const float *bi, const float *bh, const float *ln_scale,
                              const float *ln_bias, float *out, int32_t ldo, float *g4, int32_t ldg, int32_t R,
                              int32_t H, int32_t *tile_flags, const int32_t *wbad, void *stream);
/* planes[q][n][k] = fp16x2 part q of 2^10 (k < K ? W[k][n] : 0) (n < N, k < Kp) for
 * msat_gru_ln_fused_fwd_h2r; *bad (device int, cleared first) = 1 if a scaled weight is not in
 * (-2^15, 2^15). */
int msat_split_f16x2_t(const float *W, int32_t K, int32_t N, int32_t ldw, int32_t Kp, void *planes, int32_t *bad,
                       void *stream);
/* msat_gru_ln_bwd from the fused forward's g4 tape (same outputs).  dbi (3H) / dbh_n (H), both
 * or neither, receive (+=) the gate-bias gradients sum_rows dGi and sum_rows dGh[:, 2H:3H]
 * (b_ir|b_iz|b_in and b_hn) from the same pass.  partial >= msat_gru_ln_bwd_partial_floats.
 * accumulate_ln: bit 0 accumulates the LN grads (else overwrites them); bit 1 overwrites dhprev
 * (its prior contents are never read) instead of accumulating into it; bit 2 packs each row as
 * [dan | dar | daz | dan*r] (4H, dGh = dGi + H, lddi = lddh >= 4H): dGi is then in gate order
 * (n, r, z) and the r / z columns are written once for both. */
/* msat_gru_ln_bwd_g4 plus (+=) the gradient of the input-matrix rows that multiply nfeat per-row
 * features (nfeat 0, 2 or 6; feat (R, ldf)): dfeat[k][g H + j] = sum_rows feat[r][k] dG_g[r][j]
 * (dfeat nfeat x 3H contiguous, gates r, z, n), reduced with the gate-bias partials in one pass. */
int msat_gru_ln_bwd_g4f(const float *dy, int32_t ldy, const float *g4, int32_t ldg, const float *hprev, int32_t ldp,
                        const float *ln_scale, float *dGi, int32_t lddi, float *dGh, int32_t lddh, float *dhprev,
                        int32_t lddp, float *dln_scale, float *dln_bias, float *dbi, float *dbh_n, const float *feat,
                        int32_t ldf, int32_t nfeat, float *dfeat, float *partial, int32_t R, int32_t H,
                        int32_t accumulate_ln, void *stream);
/* msat_gru_ln_bwd_g4f (packed rows) + rexp[r] = the fp16x2 scale exponent of row r's largest |dG|
 * (max |dG| 2^e in [2^14, 2^15); 0x3fff for an all-zero row) for msat_gemm_wgrad_h2 / msat_gemm_h2.
 * Flags bit 3 (with the bias outputs and nfeat 2 or 6): the packed row is stored as fp16x2 planes at that
 * exponent instead of fp32 -- the row's 4H floats at dGi + r lddi hold [hi (4H fp16) | lo (4H fp16)] with
 * hi = fp16(x 2^e), lo = fp16(x 2^e - hi) (e = 0 for an all-zero row), for the *_planes products. */
int msat_gru_ln_bwd_g4fe(const float *dy, int32_t ldy, const float *g4, int32_t ldg, const float *hprev, int32_t ldp,
                         const float *ln_scale, float *dGi, int32_t lddi, float *dGh, int32_t lddh, float *dhprev,
                         int32_t lddp, float *dln_scale, float *dln_bias, float *dbi, float *dbh_n, const float *feat,
                         int32_t ldf, int32_t nfeat, float *dfeat, float *partial, int32_t R, int32_t H,
                         int32_t accumulate_ln, int32_t *rexp, void *stream);
int msat_gru_ln_bwd_g4(const float *dy, int32_t ldy, const float *g4, int32_t ldg, const float *hprev,
                       int32_t ldp, const float *ln_scale, float *dGi, int32_t lddi, float *dGh, int32_t lddh,
                       float *dhprev, int32_t lddp, float *dln_scale, float *dln_bias, float *dbi, float *dbh_n,
                       float *partial, int32_t R, int32_t H, int32_t accumulate_ln, void *stream);
/* out[N] (+)= column sums of G (M x N) — bias gradients; workspace >= msat_colsum_workspace_floats. */
size_t msat_colsum_workspace_floats(int32_t M, int32_t N);
int msat_colsum(const float *G, int32_t ldg, int32_t M, int32_t N, float *out, int32_t accumulate,
                float *workspace, void *stream);
int msat_relu(float *x, size_t n, void *stream);
int msat_relu_bwd(float *dy, const float *y, size_t n, void *stream);

/* ---- heads (learner:264-350): graph batch = per sample G graphs (0 critic, 1+i agent i) ---- */
int msat_critic_pool(const float *Hp, const float *Hn, const float *Hc, int32_t H, const int32_t *vbase,
                     const int32_t *nv, const int32_t *cbase, const int32_t *nc, int32_t G, int32_t S,
                     float *pooled, void *stream);
int msat_critic_pool_bwd(const float *Hp, const float *Hn, const float *Hc, int32_t H, const int32_t *vbase,
                         const int32_t *nv, const int32_t *cbase, const int32_t *nc, int32_t G, int32_t S,
                         const float *dpooled, float *dHp, float *dHn, float *dHc, void *stream);
int msat_actor_pool(const float *Hp, const float *Hn, const float *Hc, int32_t H, const int32_t *vbase,
                    const int32_t *nv, const int32_t *cbase, const int32_t *nc, int32_t G, int32_t S,
                    int32_t A, int32_t M, int32_t base_sz, int32_t rem, const float *id_emb, int32_t E,
                    float *my_emb, float *ctx, void *stream);
int msat_actor_pool_bwd(int32_t H, const int32_t *vbase, const int32_t *nv, const int32_t *cbase,
                        const int32_t *nc, int32_t G, int32_t S, int32_t A, int32_t M, int32_t base_sz,
                        int32_t rem, int32_t E, const float *dmy, const float *dctx, float *dHp, float *dHn,
                        float *dHc, float *did, void *stream);
int msat_bcast_add_relu(float *Q, const float *P, int32_t R, int32_t M, int32_t W, void *stream);
int msat_group_sum(const float *dQ, int32_t R, int32_t M, int32_t W, float *dP, void *stream);
int msat_assemble_logits(const float *flip, const float *noop, int32_t SA, int32_t A, int32_t M,
                         int32_t base_sz, int32_t rem, float *logits, void *stream);
int msat_mask_var_logits(float *logits, int32_t SA, int32_t A, int32_t M, int32_t base_sz, int32_t rem,
                         void *stream);
int msat_split_dlogits(const float *dlogits, int32_t SA, int32_t M, float *dflip, float *dnoop, void *stream);

/* ---- policy / loss / optimiser (learner:397-403, :597-650; mappo_runner.py:198) ---- */
int msat_sample_actions(const float *logits, int32_t R, int32_t W, int32_t greedy, uint64_t seed,
                        uint64_t counter, int32_t *action, float *logp, void *stream);
int msat_ppo_loss(const float *logits, int32_t S, int32_t A, int32_t M, int32_t action_mode,
                  int32_t base_sz, int32_t rem, const int32_t *action, const float *old_logp,
                  const float *gae, const float *value, const float *old_value, const float *targets,
                  float clip_eps, float vf_clip, float ent_coef, float vf_coef, int32_t minibatch,
                  float *dlogits, float *dvalue, float *row_terms, double *loss_sums, void *stream);
int msat_adam(float *params, const float *grads, float *m, float *v, size_t n, float lr, float b1, float b2,
              float eps, int32_t count, float grad_scale, void *stream);
/* msat_adam + a fail-loud guard: if an updated parameter is not finite, *first_bad = min(*first_bad,
 * count) (device int32, the caller initialises it to INT32_MAX).  No host sync: the runner reads the
 * flag once per train cycle (mappo_runner.py:313-317's loop) and raises, instead of carrying NaN
 * parameters forward -- the hazard of an instance with a variable in no clause at zero-initialised
 * biases (tests/test_isolated_variable.py). */
int msat_adam_checked(float *params, const float *grads, float *m, float *v, size_t n, float lr, float b1, float b2,
                      float eps, int32_t count, float grad_scale, int32_t *first_bad, void *stream);
/* ---- collectives (RCCL over xGMI, one communicator per process) ----
 * The gradient is ONE flat fp32 buffer (the grads of every parameter, 16-B aligned tensors): before
 * msat_adam(..., grad_scale = 1 / world) every rank SUM-all-reduces it in place (learner:647-650 is the
 * single-device update this replaces).  The Python learner reaches RCCL either through torch.distributed
 * (whose "nccl" backend is RCCL on ROCm; the default) or through these entry points
 * (marlsat/learners/collectives.py CapiComm, MARLSAT_COLLECTIVES=capi); a cgo / JNI host uses these.
 * Rank 0 draws the id, the host broadcasts its msat_comm_id_bytes() bytes, every rank calls
 * msat_comm_init.  Errors: MSAT_EBADARG, MSAT_ECOMM (message from RCCL). */
size_t msat_comm_id_bytes(void);
int msat_comm_unique_id(uint8_t *id_out);
int msat_comm_init(const uint8_t *id, int32_t rank, int32_t world, void **comm_out);
/* in place: buf[0..count) = sum over ranks; dtype 0 = fp32, 1 = fp64; enqueued on `stream` */
int msat_allreduce_sum(void *comm, void *buf, size_t count, int32_t dtype, void *stream);
int msat_comm_destroy(void *comm);

/* ---- learner glue (learner:562-592 minibatching, :661-719 metrics) ---- */
/* out[0..N) = a keyed pseudo-random permutation of [0, N) (4-round Feistel + cycle walking), for the
 * PPO epoch's minibatch rows (replaces jax.random.permutation, learner:576; deterministic in
 * (seed, counter)). */
int msat_permutation(int32_t N, uint64_t seed, uint64_t counter, int32_t *out, void *stream);
/* dst[f][s] = src[f][idx[s]] for nfields <= 8 fields of row_bytes[f] bytes per row (the micro-batch's
 * transition rows, learner:597-602); src / dst / row_bytes are host arrays of device pointers. */
int msat_gather_rows(const int32_t *idx, int32_t S, int32_t nfields, const void *const *src, void *const *dst,
                     const int32_t *row_bytes, void *stream);
/* Row bases of a graph batch (learner:148-195 batch assembly): per sample s of instance inst[s],
 * bases[s] = exclusive prefix sums of the instances' (var rows, clause rows, incidences) counts
 * nv / nc / ne, totals[3] = their sums (the batch's Nv, Nc, nnz), or -1 for a sum above INT32_MAX
 * (the batch cannot be indexed in int32; the caller must split it). */
int msat_graph_bases(int32_t S, const int32_t *inst, const int32_t *nv, const int32_t *nc, const int32_t *ne,
                     int32_t *bases, int32_t *totals, void *stream);
/* fp64 cycle sums over N transitions (learner:661-719): out[9] = sum reward, sum done, sum solved&done,
 * sum unsat*done, sum episode_step*(solved&done), sum tg, sum tg^2, sum d, sum d^2 (d = tg - vpred). */
int msat_cycle_metrics(int32_t N, const float *reward, const uint8_t *done, const uint8_t *solved,
                       const int32_t *num_unsatisfied, const int32_t *episode_step, const float *targets,
                       const float *vpred, double *out, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* MARLSAT_NET_H */
