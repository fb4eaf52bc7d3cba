/*
 * acmi.h — C-ABI of libacmi, the MI355X-native (gfx950) A2C/ACKTR hot path.
 *
 * Drop-in boundary for the reference's TF graph + kfac ops on the rollout and
 * update path of jrobine/actor-critic.  Every entry point
 *   - takes caller-owned DEVICE buffers (plain pointers, sizes, no torch types),
 *   - is stream-ordered on `stream` (a hipStream_t), asynchronous, never
 *     allocates and never synchronises (so a caller may capture it in a graph),
 *   - returns 0 (ACMI_OK) or a negative ACMI_ERR_* code; the message is in
 *     acmi_last_error() (thread-local).
 *
 * Reference interface each entry point replaces is cited as path:line into
 * /root/reference.  Layouts: NHWC u8 observations,
 * HWIO conv weights, [in,out] FC weights (reference nn.py:8-84), fp32 math.
 */
#ifndef ACMI_H_
#define ACMI_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ACMI_ABI_VERSION 4  /* 3: acmi_env_state_t.game, acmi_rollout_io_t step fusion fields;
                               4: ws_floats on acmi_backward / acmi_kfac_output_stats, per-net
                                  mode fields in acmi_net_t */

enum {
  ACMI_OK = 0,
  ACMI_ERR_ARG = -1,   /* bad shape / null pointer / unsupported size   */
  ACMI_ERR_HIP = -2,   /* a HIP launch failed                             */
  ACMI_ERR_WS = -3,    /* caller workspace too small                      */
};

typedef void* acmi_stream_t; /* hipStream_t */

const char* acmi_last_error(void);
int acmi_abi_version(void);
/* Host-only: sizeof of the ABI structs, in the order acmi_net_t, acmi_acts_t,
 * acmi_bwd_t, acmi_env_state_t, acmi_rollout_io_t (n <= 5 written), so a
 * binding can check its struct mirrors (returns the number written). */
int acmi_abi_struct_sizes(int64_t* sizes, int n);

/* Arithmetic of the fused weight-gradient + K-FAC A-factor reductions (conv2,
 * conv3, heads; the dominant K-FAC covariance work, kfac cov_update_thunks,
 * actorcritic/kfac_utils.py:39,44).  Both modes are fp32-accurate:
 *   ACMI_GEMM_X3  16-bit split operands on the 16-bit matrix cores (default):
 *                 f16x2 (two f16 parts, 3 MFMAs, power-of-two scales from
 *                 published maxima) for the conv tower, the dX chain, the band
 *                 and fc4 reductions; bf16x3 (6 MFMAs) for the small rest
 *   ACMI_GEMM_F32 v_mfma_f32_32x32x2_f32
 * Initial mode from the environment variable ACMI_GEMM ("x3" / "f32").
 * The acmi_set_*_mode functions set the PROCESS DEFAULT, which nets with a
 * zero mode field use; a net's own field overrides it (acmi_net_t).
 * Not stream-ordered: set it between launches. */
#define ACMI_GEMM_F32 0
#define ACMI_GEMM_X3 1
int acmi_set_gemm_mode(int mode);
int acmi_get_gemm_mode(void);

/* Precision of the forward's conv tower (rollout and update forward; BASELINE
 * configs[4] "bf16 forward / fp32 K-FAC factors" -- an extension, the
 * reference computes in fp32):
 *   ACMI_FWD_F32   f16x2 split operands (scaled f16 h + l, three MFMAs per
 *                  product), f32-accurate (default)
 *   ACMI_FWD_BF16  one 16-bit MFMA per product: weights and conv2/conv3 inputs
 *                  scaled by powers of two and rounded once to f16 (u8 pixels
 *                  exact), f32 accumulation.  The error bound is RELATIVE TO
 *                  EACH TENSOR'S RANGE: elements within 2^-14 of their tensor's
 *                  bound keep 11-bit significands (finer than bf16's 8), but
 *                  f16's exponent range is narrower than bf16's -- elements
 *                  below ~2^-28 of the bound become f16 subnormals and below
 *                  ~2^-38 flush to zero, where bf16 would keep them.  The
 *                  bounds are weight-derived (loose), which widens that margin;
 *                  the tests check error against each tensor's range
 * The backward, the K-FAC statistics and the optimizers stay f32-accurate; they
 * read the activations the forward produced.  Initial mode from ACMI_FORWARD
 * ("bf16" / "f32").  Not stream-ordered: set it between launches.
 * The 16-bit arithmetic lives in the fused conv tower only: setting
 * ACMI_FWD_BF16 fails (ACMI_ERR_ARG) in ACMI_GEMM_F32 mode, and a forward in
 * that mode fails without net->conv_prep or on observations / an image stride
 * that are not 16-byte aligned -- the mode is never silently ignored. */
#define ACMI_FWD_F32 0
#define ACMI_FWD_BF16 1
int acmi_set_forward_mode(int mode);
int acmi_get_forward_mode(void);

/* How conv2 / conv3 form their weight gradient + A factor in ACMI_GEMM_X3 mode
 * (both fp32-accurate, same sums reassociated):
 *   ACMI_CONV_STATS_BAND    pixel-pair band reduction (default): each pair of
 *                           input pixels sharing a patch is multiplied once over
 *                           the images' dense activation rows, the patch sums
 *                           folded afterwards (2.5x / 1.6x fewer MACs for conv3 /
 *                           conv2 than patch rows, no im2col gather)
 *   ACMI_CONV_STATS_PATCHES [P;1]^T [P | dY] over the im2col patch rows
 * Initial mode from ACMI_BAND ("0" = patches).  The band plans (sub-tile
 * groups, fold tables) are built on the first backward of each device and
 * kept for the process: that first acmi_backward allocates and synchronises
 * once (do not capture it in a graph).  Not stream-ordered. */
#define ACMI_CONV_STATS_PATCHES 0
#define ACMI_CONV_STATS_BAND 1
int acmi_set_conv_stats_mode(int mode);
int acmi_get_conv_stats_mode(void);
/* plan facts of the band reduction of conv2 (layer 1) or conv3 (layer 2) at
 * `rows` images: info[0] sub-tiles, [1] groups (blocks per chunk), [2] chunks,
 * [3] rows per chunk, [4] sum over groups of the busiest SIMD's sub-tiles */
int acmi_band_info(int layer, int C3, int64_t rows, int64_t* info);

/* ------------------------------------------------------------------------
 * Model layout.  Replaces AtariModel._build_params
 * (actorcritic/envs/atari/model.py:129-170, nn.py:8-84).
 * The flat fp32 parameter vector holds, in order:
 *   conv1.W[8][8][4][32] conv1.b[32] conv2.W[4][4][32][64] conv2.b[64]
 *   conv3.W[3][3][64][C3] conv3.b[C3] fc4.W[49*C3][512] fc4.b[512]
 *   pi.W[512][A] pi.b[A] v.W[512][1] v.b[1]
 * so each layer's homogeneous weight matrix [W; b] ((K+1) x Cout, the K-FAC
 * block of envs/atari/model.py:219-246) is one contiguous row-major slice.
 * ---------------------------------------------------------------------- */
#define ACMI_NUM_LAYERS 6   /* conv1 conv2 conv3 fc4 fc_policy fc_baseline */
#define ACMI_NUM_AFACT 5    /* fc_policy and fc_baseline share one A factor */
#define ACMI_NUM_GFACT 6

typedef struct acmi_net {
  int num_actions;     /* A  (Breakout 4, full Atari 18); 1 <= A <= 64    */
  int conv3_filters;   /* C3 (32 ACKTR, 64 A2C: a2c_acktr.py:51-53)       */
  const float* params; /* device, acmi_param_count() floats               */
  const void* conv_prep; /* nullable: device, acmi_conv_prep_bytes(C3) bytes,
                            filled by acmi_conv_prepare from THESE params (the
                            caller re-prepares after every parameter change) */
  /* This net's arithmetic, each the mode + 1 (ACMI_GEMM_*, ACMI_FWD_*,
   * ACMI_CONV_STATS_*); 0 = the process default (acmi_set_*_mode).  Every
   * entry point taking a net runs in its net's modes (held per calling thread
   * for the call), so two nets in one process, or two threads, never see each
   * other's settings; an invalid combination fails with ACMI_ERR_ARG. */
  int gemm_mode;
  int forward_mode;
  int conv_stats_mode;
} acmi_net_t;

/* The forward's fused conv tower (x3 gemm mode), fc4 at rollout batches
 * (split-K slabs with a forward workspace) and the backward's conv2 input
 * gradient (acmi_backward, acmi_kfac_output_stats) read their weights as
 * pre-split f16x2 MFMA fragments -- scaled f16 (h, l) pairs, with a header of
 * power-of-two scale bounds (max |W| per layer, weight-derived activation
 * bounds) -- when net->conv_prep is set: acmi_conv_prepare writes them
 * (stream-ordered, a few small kernels) -- once per parameter version, not per
 * rollout step or update.  With conv_prep == NULL the forward runs the
 * per-layer conv kernels and fc4 / the conv2 input gradient the generic
 * split-per-block bf16x3 GEMM: f32-class like the prepared path, not
 * bit-identical to it (the sampled-loss chain then stores its conv1-output
 * gradient and reduces its G factor separately); the 16-bit forward
 * (ACMI_FWD_BF16) needs conv_prep. */
int64_t acmi_conv_prep_bytes(int conv3_filters);
int acmi_conv_prepare(const acmi_net_t* net, void* conv_prep, acmi_stream_t stream);

int64_t acmi_param_count(int num_actions, int conv3_filters);
/* off[2*l] = W offset, off[2*l+1] = b offset of layer l (12 entries)       */
int acmi_param_offsets(int num_actions, int conv3_filters, int64_t* off12);

/* K-FAC block geometry: din[l] = K_l + 1 (homogeneous), dout[l] = Cout_l.
 * stat_off[0..4] = offsets of A factors (din^2 each, A4 shared by l=4,5),
 * stat_off[5..10] = offsets of G factors (dout^2), *total = floats overall. */
int acmi_kfac_layout(int num_actions, int conv3_filters, int64_t* din6,
                     int64_t* dout6, int64_t* stat_off11, int64_t* total);

/* ------------------------------------------------------------------------
 * Forward.  Replaces the TF graph of AtariModel.__init__/_build_layers
 * (envs/atari/model.py:77-217): u8/255 normalise (:92-95), conv1 8x8 s4,
 * conv2 4x4 s2, conv3 3x3 s1 (VALID, +bias, ReLU), NHWC flatten, fc4 512
 * ReLU, policy logits and value heads.  `obs` holds B NHWC u8 images
 * [84][84][4]; image b starts at obs + b*img_stride (bytes), which lets the
 * rollout read step t of a [N][T][84][84][4] buffer in place.
 * ---------------------------------------------------------------------- */
typedef struct acmi_acts {
  float* a1;     /* [B][20][20][32] post-ReLU                               */
  float* a2;     /* [B][9][9][64]                                           */
  float* a3;     /* [B][7][7][C3]  (= the NHWC-flattened fc4 input)         */
  float* a4;     /* [B][512]                                                */
  float* logits; /* [B][ld_logits]                                          */
  float* value;  /* [B]  (may be NULL when want_value == 0)                 */
  int ld_logits;
  float* ws;     /* optional split-K workspace (NULL: no split), floats:  */
  int64_t ws_floats; /* >= acmi_forward_ws_floats(B) enables it            */
  /* optional ReLU' bit masks of a1..a3 (all three or none; NULL: none): bit e
   * of word e / 32 = (a[e] > 0), i.e. one word per 32 channels of a pixel --
   * m1 [B][400], m2 [B][81][2], m3 [B][49][C3/32] uint32.  acmi_forward writes
   * them beside the activations (same image stride); acmi_backward and
   * acmi_kfac_output_stats then mask the input gradients from them instead of
   * re-reading the f32 activations (1/32 of the bytes; results bit-identical). */
  uint32_t* m1;
  uint32_t* m2;
  uint32_t* m3;
} acmi_acts_t;

int64_t acmi_forward_ws_floats(int B);

int acmi_forward(const acmi_net_t* net, const uint8_t* obs, int64_t img_stride,
                 int B, const acmi_acts_t* acts, int want_value,
                 acmi_stream_t stream);

/* ------------------------------------------------------------------------
 * Categorical sampling.  Replaces Categorical.sample (tf.multinomial) and
 * the squeeze of policies.py:86, model.py:135-151.  Counter-based RNG:
 * u = u01(key4(seed, stream_id, counter, row)); when `uniforms` is non-NULL
 * it supplies u[row] instead (parity tests).  Inverse-CDF over softmax in
 * f32.  A row with a NaN/inf logit yields action -1 and sets *bad_rows
 * (device int, accumulated) — the reference would instead emit index A and
 * fail later in sparse_softmax_cross_entropy (README.md:53-54).
 * mode != 0 -> argmax (Categorical.mode, model.py:153-169).
 * ---------------------------------------------------------------------- */
int acmi_sample_actions(const float* logits, int ld, int B, int A,
                        uint32_t seed, uint32_t stream_id, uint32_t counter,
                        const float* uniforms, int mode, int32_t* actions,
                        int32_t* bad_rows, acmi_stream_t stream);
/* The same for rows row_offset .. row_offset+B-1 of a larger batch (the RNG
 * key uses the global row): a batch sampled in pieces (the rollout's env
 * halves on two streams) draws exactly the actions of one launch. */
int acmi_sample_actions_at(const float* logits, int ld, int B, int A,
                           uint32_t seed, uint32_t stream_id, uint32_t counter,
                           int row_offset, const float* uniforms, int mode,
                           int32_t* actions, int32_t* bad_rows,
                           acmi_stream_t stream);
/* counter = *counter_dev + counter_add (counter_dev: device uint32, nullable):
 * a rollout captured once in a hipGraph and replayed reads its RNG counter
 * from device memory, the host refreshing it before each replay. */
int acmi_sample_actions_dev(const float* logits, int ld, int B, int A,
                            uint32_t seed, uint32_t stream_id,
                            const uint32_t* counter_dev, uint32_t counter_add,
                            int row_offset, const float* uniforms, int mode,
                            int32_t* actions, int32_t* bad_rows,
                            acmi_stream_t stream);

/* Per-row Categorical.entropy and log_prob(actions) (policies.py:87-89);
 * either output may be NULL (log_prob needs actions). */
int acmi_categorical(const float* logits, int ld, int B, int A,
                     const int32_t* actions, float* entropy, float* log_prob,
                     acmi_stream_t stream);

/* ------------------------------------------------------------------------
 * n-step targets and advantage.  Replaces objectives.py:123-130 with the
 * py_func closures _discount (:178-202) and _discount_bootstrap (:205-214).
 * Batch-major [N][T].  gamma_pow[k] = f32(gamma)**f32(k) (numpy float32
 * power, exactly the D-matrix entries of objectives.py:183-187), k < T;
 * boot_pow[k] = k-fold sequential f32 product of f32(gamma) (the float32
 * cumprod of objectives.py:211), k <= T.  Both tables are host-computed.
 * target[n,t] = sum_{i=t..stop} r[n,i]*gamma_pow[i-t] (ascending i, no FMA,
 *              stop = first terminal >= t)  +  boot_pow[T-t]*v_boot[n] (if no
 *              terminal in t..T-1);   adv = target - value.
 * ---------------------------------------------------------------------- */
int acmi_returns(const float* rewards, const uint8_t* terminals,
                 const float* values, const float* v_boot, int N, int T,
                 const float* gamma_pow, const float* boot_pow, float* targets,
                 float* adv, acmi_stream_t stream);

/* GAE(lambda) targets and advantages -- an option BEYOND the reference (whose
 * A2CObjective uses the n-step targets of acmi_returns, objectives.py:123-130;
 * BASELINE.json north_star names the GAE scan).  Batch-major [N][T], v_boot[N]
 * = V(s_T).  delta_t = r_t + gamma*V_{t+1}*(1-d_t) - V_t (V_T = v_boot),
 * A_t = delta_t + gamma*lambda*(1-d_t)*A_{t+1}, target_t = A_t + V_t; float32,
 * no contraction, in exactly that order.  lambda = 1 gives the n-step targets
 * in exact arithmetic.  0 <= lambda <= 1. */
int acmi_gae(const float* rewards, const uint8_t* terminals, const float* values,
             const float* v_boot, int N, int T, float gamma, float lambda,
             float* targets, float* adv, acmi_stream_t stream);

/* Advantage normalisation (an option beyond the reference, which has none,
 * objectives.py:128-130): moments[0..1] = (sum, sum of squares) of adv[0..M)
 * in double, fixed order (ws: acmi_adv_moments_ws_doubles(M) doubles).  A
 * data-parallel caller sums the moments over ranks, then
 * acmi_adv_normalize: adv = (adv - mean) / (std + eps), mean/std (population)
 * from moments over `count` rows (the global batch). */
int64_t acmi_adv_moments_ws_doubles(int64_t M);
int acmi_adv_moments(const float* adv, int64_t M, double* ws, double* moments,
                     acmi_stream_t stream);
int acmi_adv_normalize(float* adv, int64_t M, const double* moments, double count,
                       double eps, acmi_stream_t stream);

/* ------------------------------------------------------------------------
 * A2C losses and their gradient w.r.t. the head outputs.  Replaces
 * objectives.py:132-154 and the head part of tf.gradients of
 * L = L_pi + vcoef*L_v (objectives.py:78).  M = N*T rows.
 *   L_pi = -(mean(adv*logpi(a)) + beta*mean(H)),  L_v = mean((target-V)^2/2)
 * dhead[m][0..A-1] = dL/dlogits, dhead[m][A] = dL/dV, row stride ldh >= A+1,
 * each scaled by grad_scale (1/world_size for data-parallel means).
 * loss_out[0..2] = grad_scale * (L_pi, L_v, mean entropy) — deterministic
 * two-pass sums; scaled like dhead so that a SUM all-reduce over the ranks
 * (the update buffer's loss slots) yields the global means.
 * ws: >= acmi_a2c_loss_ws_floats(M) floats.
 * ---------------------------------------------------------------------- */
int64_t acmi_a2c_loss_ws_floats(int M);
int acmi_a2c_loss(const float* logits, int ld, const float* values,
                  const int32_t* actions, const float* targets,
                  const float* adv, int M, int A, float beta, float vcoef,
                  float grad_scale, float* dhead, int ldh, float* ws,
                  float* loss_out, acmi_stream_t stream);

/* ------------------------------------------------------------------------
 * Backward through the tower (the rest of tf.gradients, objectives.py:78)
 * fused with the K-FAC input-factor statistics (kfac cov_update_thunks,
 * kfac_utils.py:39,44; registration envs/atari/model.py:219-246):
 *   grads  <- dL/dparams in the param layout (overwritten)
 *   a_stats (nullable) <- for l = 0..4: A_l = mean over rows of [x;1][x;1]^T
 *           (conv: x = the (kh,kw,cin) input patch at every output location,
 *            rows = B*locations; fc: x = the input row; A_4 = fc4 output).
 * dhead: [B][ldh] from acmi_a2c_loss.  d1..d4 are [B]x(layer output) scratch.
 * ws: ws_floats >= acmi_backward_ws_floats(B, A, C3) floats; a smaller
 * ws_floats fails with ACMI_ERR_WS before anything is enqueued (nothing is
 * written).  Layout: [operand-scale scratch | conv1 A-factor integers |
 * split-K partials]; the partial region is everything past the fixed prefix, so
 * a larger workspace only lets more of the small layers' finalizes share one
 * launch (results bit-identical for every legal size).
 * net->conv_prep (when non-null) must have been prepared (acmi_conv_prepare)
 * from the same parameters as net->params: its header supplies the a1 / a2 /
 * a3 bounds that scale the f16x2 operands of the conv2 / conv3 / fc4
 * reductions, and the pre-split weights of the input-gradient chain.  Callers
 * re-prepare after every parameter update (NetEngine does, keyed by its
 * parameter version); a stale prep gives wrong scales, not an error.
 * ---------------------------------------------------------------------- */
typedef struct acmi_bwd {
  float* d1; /* [B][20][20][32] */
  float* d2; /* [B][9][9][64]   */
  float* d3; /* [B][7][7][C3]   */
  float* d4; /* [B][512]        */
  const float* dhead;
  int ldh;
} acmi_bwd_t;

int64_t acmi_backward_ws_floats(int B, int num_actions, int conv3_filters);
int acmi_backward(const acmi_net_t* net, const uint8_t* obs,
                  int64_t img_stride, int B, const acmi_acts_t* acts,
                  const acmi_bwd_t* bwd, float* grads, float* a_stats,
                  float* ws, int64_t ws_floats, acmi_stream_t stream);

/* ------------------------------------------------------------------------
 * K-FAC output-factor statistics (kfac "gradients" estimation mode over the
 * predictive distributions registered at policies.py:146-158 and
 * baselines.py:55-69): y_pi ~ Categorical(logits) and y_v ~ N(V, 1) are
 * sampled with the counter RNG keyed (seed, 0, counter, row_offset + b) --
 * row_offset = the global row of batch row 0 (rank * B for an env shard), so
 * a data-parallel shard draws exactly the full batch's samples; the per-example
 * gradients of -log p(y) w.r.t. each registered layer output are
 * back-propagated (dX only) and G_l = mean over rows of g g^T is written to
 * g_stats (layout of acmi_kfac_layout, G part).  Reuses bwd->d1..d4 and ws
 * (ws_floats >= acmi_backward_ws_floats(B, A, C3), else ACMI_ERR_WS before
 * anything is enqueued; layout [scratch | sampled head gradients | partials]).
 * ---------------------------------------------------------------------- */
int acmi_kfac_output_stats(const acmi_net_t* net, int B,
                           const acmi_acts_t* acts, const acmi_bwd_t* bwd,
                           uint32_t seed, uint32_t row_offset, uint32_t counter,
                           float* g_stats, float* ws, int64_t ws_floats,
                           acmi_stream_t stream);
/* acmi_backward + the input-gradient half of acmi_kfac_output_stats in one
 * call, with conv2's input gradient of BOTH chains as one launch (one W2^T
 * stream over the loss chain's and the sampled chain's image rows, the
 * epilogue chosen per tile: the masked d1 store, or conv1's G-factor Gram).
 * bwd / ws: the loss chain's (as acmi_backward); bwd_s / ws_s: the sampled
 * chain's own d1..d4 and workspace (ws_floats, ws_s_floats >=
 * acmi_backward_ws_floats), on which acmi_kfac_output_stats_finish then forms
 * the G factors.  The pair is bit-identical to acmi_backward followed by
 * acmi_kfac_output_stats(bwd_s, ws_s) with the same seed / row_offset /
 * counter, and records the same dX event.  Without net->conv_prep or in
 * ACMI_GEMM_F32 mode the two conv2 launches run one after the other.
 * Reference: the same graphs as acmi_backward / acmi_kfac_output_stats
 * (objectives.py:78-79, policies.py:157-158). */
int acmi_backward_stacked(const acmi_net_t* net, const uint8_t* obs, int64_t img_stride,
                          int B, const acmi_acts_t* acts, const acmi_bwd_t* bwd,
                          float* grads, float* a_stats, float* ws, int64_t ws_floats,
                          const acmi_bwd_t* bwd_s, uint32_t seed, uint32_t row_offset,
                          uint32_t counter, float* ws_s, int64_t ws_s_floats,
                          acmi_stream_t stream);
int acmi_kfac_output_stats_finish(const acmi_net_t* net, int B, const acmi_acts_t* acts,
                                  const acmi_bwd_t* bwd_s, float* g_stats, float* ws_s,
                                  int64_t ws_s_floats, acmi_stream_t stream);
/* Makes `stream` wait (stream-ordered, no host sync) for the point right after
 * the input-gradient chain of the most recent acmi_backward on this device, so
 * a sampled-loss chain (acmi_kfac_output_stats on its own buffers) enqueued on
 * `stream` afterwards runs next to that backward's weight-gradient reductions. */
int acmi_stream_wait_backward_dx(acmi_stream_t stream);

/* ------------------------------------------------------------------------
 * K-FAC running factors: zero-initialised EMA with zero-debias (kfac
 * FisherFactor cov update with cov_ema_decay, a2c_acktr.py:245):
 *   biased = decay*biased + (1-decay)*stats;  factors = biased * debias
 * (debias = 1/(1-decay^t), host-computed).  n floats.
 * ---------------------------------------------------------------------- */
int acmi_kfac_ema(float* biased, float* factors, const float* stats,
                  int64_t n, float decay, float debias, float stats_scale,
                  acmi_stream_t stream);

/* Factor statistics as upper triangles, for the data-parallel all-reduce of the
 * A / G statistics (the symmetric half only, 40 % fewer
 * bytes on the wire): which = 1 the A factors, 2 the G factors, 3 both; the
 * selected factors of the acmi_kfac_layout stats area packed back to back,
 * factor f (n x n) as n(n+1)/2 floats, row r's columns r .. n-1.  Unpack writes
 * both halves (the factors come back exactly symmetric).  Stream-ordered. */
int64_t acmi_kfac_packed_floats(int num_actions, int conv3_filters, int which);
int acmi_kfac_pack(int num_actions, int conv3_filters, int which, const float* stats, float* packed,
                   acmi_stream_t stream);
int acmi_kfac_unpack(int num_actions, int conv3_filters, int which, const float* packed, float* stats,
                     acmi_stream_t stream);

/* ------------------------------------------------------------------------
 * Damped inverses (kfac inv_update_thunks, kfac_utils.py:46-50): per layer
 *   lambda_l = damping / (conv_normalize && l<3 ? locations_l : 1)
 *   pi_l = sqrt((tr A_l / din_l) / (tr G_l / dout_l))
 *   Ainv_l = (A_l + pi_l*sqrt(lambda_l) I)^-1,  Ginv_l = (G_l + sqrt(lambda_l)/pi_l I)^-1
 * computed in fp64 (block Gauss-Jordan, SPD, no pivoting) and stored f32.
 * inv layout: 12 blocks, m = 2l (Ainv_l, n = din_l) and 2l+1 (Ginv_l,
 * n = dout_l); block m is n rows of stride ld_m = n rounded up to 4 at
 * offsets[m] (acmi_kfac_inverse_layout), padding columns zero, so the
 * preconditioning GEMMs read aligned float4 runs.
 * ws: >= acmi_kfac_inverse_ws_doubles(...) doubles.
 * ---------------------------------------------------------------------- */
int acmi_kfac_inverse_layout(int num_actions, int conv3_filters, int64_t* offsets,
                             int64_t* lds);
int64_t acmi_kfac_inverse_floats(int num_actions, int conv3_filters);
int64_t acmi_kfac_inverse_ws_doubles(int num_actions, int conv3_filters);
int acmi_kfac_inverse(int num_actions, int conv3_filters,
                      const float* factors, float damping, int conv_normalize,
                      float* inv, double* ws, acmi_stream_t stream);

/* Eigendecomposition of every damped-factor input (fp64 cyclic Jacobi):
 * eigenvalues (ascending) of A_l / G_l written to `eigvals` in the factor
 * layout order (diagnostic and parity path; north_star "KFAC eigenvalues"). */
int64_t acmi_kfac_eig_ws_doubles(int num_actions, int conv3_filters);
int acmi_kfac_eigvals(int num_actions, int conv3_filters, const float* factors,
                      double* eigvals, double* ws, acmi_stream_t stream);

/* ------------------------------------------------------------------------
 * Natural-gradient step (KfacOptimizer.apply_gradients, kfac_utils.py:53,
 * a2c_acktr.py:243-246):  Delta_l = Ainv_l [dW_l; db_l] Ginv_l;
 *   coeff = min(1, sqrt(norm_constraint / (lr^2 * sum_l <g_l, Delta_l>)));
 *   v = momentum*v + coeff*Delta;   params -= lr*v.
 * coeff is computed on the device (no host round trip); *coeff_out gets it.
 * ws: >= acmi_kfac_step_ws_floats() floats.
 * ---------------------------------------------------------------------- */
int64_t acmi_kfac_step_ws_floats(int num_actions, int conv3_filters);
int acmi_kfac_step(int num_actions, int conv3_filters, float* params,
                   float* velocity, const float* grads, const float* inv,
                   float lr, float momentum, float norm_constraint,
                   float* precon, float* ws, float* coeff_out,
                   acmi_stream_t stream);

/* ------------------------------------------------------------------------
 * First-order optimizers.  ClipGlobalNormOptimizer (nn.py:159-189) + TF1
 * MomentumOptimizer (cold start, a2c_acktr.py:240-241) / RMSPropOptimizer
 * (a2c_acktr.py:250-251, decay .9, momentum 0, eps 1e-10, ms init 1).
 * clip_norm <= 0 disables clipping.  norm_out (nullable) <- global norm.
 * ---------------------------------------------------------------------- */
int64_t acmi_opt_ws_floats(int64_t n);
int acmi_momentum_apply(float* params, float* accum, const float* grads,
                        int64_t n, float lr, float momentum, float clip_norm,
                        float* ws, float* norm_out, acmi_stream_t stream);
int acmi_rmsprop_apply(float* params, float* ms, float* mom,
                       const float* grads, int64_t n, float lr, float decay,
                       float momentum, float eps, float clip_norm, float* ws,
                       float* norm_out, acmi_stream_t stream);

/* ------------------------------------------------------------------------
 * Batched synthetic Atari stepper — replaces MultiEnv.step/reset over
 * SubprocessEnv (multi_env.py:49-81, 121-137, 140-362) with the semantics
 * of FrameStackWrapper (wrappers.py:201-235) and EpisodeInfoWrapper
 * (wrappers.py:263-323).  Frames are 84x84 u8 from mix32 of
 * (seed, env, episode, step, action); rewards in {-1,0,1} w.p. .05/.9/.05;
 * episode length 50 + (hash % 451).  State arrays are per env ([N]).
 * Stacks are NHWC [84][84][4] u8; env n reads obs_in + n*in_stride and
 * writes obs_out + n*out_stride (in-place allowed).
 * Mixed games (Atari-57, BASELINE configs[4] -- an extension: the
 * reference's MultiEnv holds one game, multi_env.py:36-47): with `game`
 * set, env n plays game[n] (0..56, the order of wrappers.ATARI57), whose
 * own salt, episode-length range, reward rates and legal-action count
 * (actions past it step as NOOP) replace the defaults above; game 12
 * (Breakout) keeps them.  game == NULL: every env the default game.
 * ---------------------------------------------------------------------- */
typedef struct acmi_env_state {
  int32_t* episode;   /* episode index                                    */
  int32_t* step;      /* steps taken in the current episode               */
  int32_t* length;    /* terminal step of the current episode             */
  float* total;       /* EpisodeInfoWrapper.total_reward                   */
  uint8_t* done;      /* _AutoResetWrapper._terminated                     */
  const uint8_t* game; /* game index per env, or NULL (read only)          */
} acmi_env_state_t;

int acmi_env_reset(const acmi_env_state_t* st, int N, int env_offset,
                   uint32_t seed, uint8_t* obs_out, int64_t out_stride,
                   acmi_stream_t stream);
/* rewards/terminals/episode_rewards: element n at [n*ld]; episode_rewards
 * gets the episode total at a terminal step and NaN otherwise.           */
int acmi_env_step(const acmi_env_state_t* st, int N, int env_offset,
                  uint32_t seed, const int32_t* actions, const uint8_t* obs_in,
                  int64_t in_stride, uint8_t* obs_out, int64_t out_stride,
                  float* rewards, uint8_t* terminals, float* episode_rewards,
                  int64_t ld, acmi_stream_t stream);

/* ------------------------------------------------------------------------
 * Atari frame preprocessing for real (raw RGB) frames, batched over envs:
 * replaces the frame half of the reference's per-env wrapper chain
 *   AtariFrameskipWrapper  (envs/atari/wrappers.py:54-67: np.amax of the last
 *                           two raw frames),
 *   AtariPreprocessFrameWrapper (wrappers.py:30-33: cv2 RGB2GRAY + INTER_AREA
 *                           resize to 84x84),
 *   FrameStackWrapper      (wrappers.py:224-235: roll, zero on terminal,
 *                           insert; reset repeats the frame 4 times).
 * Env n's frames: raw + n*env_stride is its LAST frame [H][W][3] u8, and, when
 * frame_stride != 0 and (nframes null or nframes[n] >= 2), the frame before
 * it is at + frame_stride (max-pooled with it).  H, W in [84, 504],
 * H*W <= 40960, W a multiple of 4, not both multiples of 84 (cv2's
 * integer-ratio fast path is not restated); raw/strides 4-byte aligned.
 * ---------------------------------------------------------------------- */
/* gray [84][84] u8 of env n at gray_out + n*out_stride */
int acmi_atari_preprocess(const uint8_t* raw, int64_t env_stride,
                          int64_t frame_stride, const uint8_t* nframes, int N,
                          int H, int W, uint8_t* gray_out, int64_t out_stride,
                          acmi_stream_t stream);
/* 4-frame stacks [84][84][4] u8 at stack + n*stack_stride: reset != 0 ->
 * [f,f,f,f]; else [s1,s2,s3,f], or [0,0,0,f] where terminals[n] != 0
 * (terminals nullable).  stack_in == stack_out is allowed. */
int acmi_atari_stack(const uint8_t* raw, int64_t env_stride, int64_t frame_stride,
                     const uint8_t* nframes, int N, int H, int W,
                     const uint8_t* terminals, int reset, const uint8_t* stack_in,
                     uint8_t* stack_out, int64_t stack_stride, acmi_stream_t stream);

/* Rollout variant of acmi_forward: batch row b reads image b of `obs` and
 * writes activation row b*act_img_stride (env-major [N][T] buffers, the
 * pointers in *acts pre-offset by step t), so step t of a T-step rollout
 * lands where the update expects it and the update re-uses it. */
int acmi_forward_strided(const acmi_net_t* net, const uint8_t* obs,
                         int64_t img_stride, int B, const acmi_acts_t* acts,
                         int want_value, int64_t act_img_stride,
                         acmi_stream_t stream);

/* One whole rollout step (MultiEnvAgent.interact's loop body, agents.py:
 * 199-219: sample_actions + MultiEnv.step) in two launch groups: the tower
 * of acmi_forward_strided up to fc4, then ONE fused kernel per env (one
 * workgroup each) that finalises a4, computes the heads, samples the action
 * (acmi_sample_actions_dev semantics, row = io->row_offset + b) and steps the
 * env (acmi_env_step semantics, reading the same frames `obs`).  Bit-identical
 * to acmi_forward_strided + acmi_sample_actions_dev + acmi_env_step. */
typedef struct acmi_rollout_io {
  uint32_t seed, stream_id, counter; /* sampler RNG key                      */
  const uint32_t* counter_dev;       /* nullable: counter += *counter_dev     */
  int row_offset;                    /* global row of batch row 0            */
  int32_t* actions;                  /* out, element b at [b*ld] (ld below)  */
  int32_t* bad_rows;                 /* device counter of non-finite rows    */
  acmi_env_state_t state;            /* env state of batch row 0's env       */
  int env_offset;                    /* global env id of batch row 0         */
  uint32_t env_seed;
  uint8_t* obs_out;                  /* next stacked frames, env b at b*out_stride */
  int64_t out_stride;
  float* rewards;                    /* element b at [b*ld]                  */
  uint8_t* terminals;
  float* episode_rewards;
  int64_t ld;
  /* Step fusion (zero / NULL: off).  next_acts: after its env step, each
   * env's workgroup runs the NEXT step's conv tower on the stack it just
   * wrote (obs_out, image stride out_stride), from LDS, into next_acts'
   * a1..a3 / m1..m3 rows (image stride next_act_stride) -- the tower launch
   * of the next step is then skipped by passing tower_done = 1 with it.
   * Needs the fused tower (x3 gemm mode, prepared weights, 16-byte aligned
   * obs_out / out_stride).  Bit-identical to the unfused steps.
   * At B <= 64 the fused step splits each image's tower over 7 workgroups;
   * their env step then leaves the post-step env states pending in acts->ws
   * (after the fc4 slabs; acmi_forward_ws_floats(B) reserves them) and the
   * NEXT step's fc4 launch commits them into `state`: consecutive fused steps
   * of a rollout must pass the same acts->ws, and a rollout must end with an
   * unfused step (next_acts = NULL, tower_done = 1), whose launch commits the
   * last pending states before its own env step.  Every step at B <= 64 commits
   * the entries still flagged there first, so a rollout abandoned between
   * fused steps is committed by the next rollout's step 0 on the same
   * acts->ws; the pending area must start zeroed (zero-fill the forward
   * workspace once before its first rollout step). */
  int tower_done;
  const struct acmi_acts* next_acts;
  int64_t next_act_stride;
  /* nullable: the stacks this step reads (obs) are also copied to
   * obs_copy + b*out_stride (step 0 reads the previous rollout's final
   * stacks in place and files them into the batch's step-0 rows) */
  uint8_t* obs_copy;
} acmi_rollout_io_t;
int acmi_rollout_step(const acmi_net_t* net, const uint8_t* obs,
                      int64_t img_stride, int B, const acmi_acts_t* acts,
                      int64_t act_img_stride, const acmi_rollout_io_t* io,
                      acmi_stream_t stream);

/* ------------------------------------------------------------------------
 * Building blocks exposed for parity tests and the bench (not needed by a
 * reference-shaped caller).
 * ---------------------------------------------------------------------- */
/* Host-only self-check of the GEMM launch planners (no GPU needed): the
 * slab groups of the fused wgrad/A-factor reduction cover every needed
 * sub-tile and column sum for K = 64..max_k, split-K chunks cover the rows.
 * Returns 0, or the first failing K (-1: chunk plan). */
int acmi_selftest_plans(int max_k);
/* Host-only diagnostic: the number of times acmi_backward / acmi_kfac_output_stats
 * finalized their deferred small-layer set early because the next layer's
 * split-K partials did not fit in the rest of the workspace (a legal size near
 * the minimum), since the previous call of this function (which resets it). */
int acmi_debug_ws_flushes(void);
/* Diagnostic (same-lease A/B of conv2's input gradient in the two K-FAC chains):
 * mode 0 = the two launches of acmi_backward / acmi_kfac_output_stats (the
 * loss chain's d2a -> masked d1 with max |d1| into d1max; the sampled chain's
 * d2b -> conv1's G-factor Gram partials); mode 1 = the same products stacked in
 * one launch (one W2^T stream, the epilogue chosen per tile).  d2max_*: the
 * published max |d2| slots; m1: the ReLU' mask words; needs net->conv_prep. */
int acmi_debug_convt2(const acmi_net_t* net, int mode, const float* d2a, const float* d2b,
                      const uint32_t* m1, float* d1, int B, float* gram_part,
                      const uint32_t* d2max_a, const uint32_t* d2max_b, uint32_t* d1max,
                      acmi_stream_t stream);

/* C[M][N] = A[M][K] @ B[K][N], row-major fp32, f32-input MFMA */
int acmi_gemm_f32(const float* A, const float* B, float* C, int M, int N,
                  int K, acmi_stream_t stream);

/* Launch-site timing for the bench: while enabled, HIP events are recorded on
 * the launch stream around every launch of `site` (up to `capacity`);
 * acmi_prof_collect synchronises them and returns the summed milliseconds
 * and the count, then rearms.  site 0 disables.  Not graph-capture safe. */
#define ACMI_PROF_CONV1_WGRAD 1 /* conv1 [P;1]^T [dY] reduction GEMM */
#define ACMI_PROF_CONV2_WGRAD 2
#define ACMI_PROF_CONV1_FWD 3
#define ACMI_PROF_CONV1_AFACTOR 4 /* exact-integer i8-MFMA conv1 A factor */
#define ACMI_PROF_CONV2_DX 5      /* conv2 input gradient (all stride phases) */
#define ACMI_PROF_FC4_DX 6        /* fc4 input gradient d4 W4^T (+ ReLU') */
#define ACMI_PROF_CONV3_DX 7      /* conv3 input gradient */
int acmi_prof_enable(int site, int capacity);
int acmi_prof_collect(double* total_ms, int* count);

#ifdef __cplusplus
}
#endif
#endif /* ACMI_H_ */
