// Rollout-side and loss-side kernels: categorical sampling, n-step targets,
// A2C loss + head gradients, first-order optimizers, batched synthetic Atari
// stepper with the reference's frame-stack / auto-reset / episode-info
// semantics.  Contracts and reference citations: include/acmi.h.
#include <math.h>

#include "common.hpp"
#include "stepper.hpp"

namespace acmi {

// ---------------------------------------------------------------------------
// sampling (policies.py:86 Categorical.sample / :87 mode)
// ---------------------------------------------------------------------------
// row_offset: global row index of local row 0 (a batch sampled in pieces draws
// the same uniforms as in one launch)
// ctr_dev (nullable): device counter base added to ctr (graph-replayed rollouts)
__global__ void sample_kernel(const float* logits, int ld, int B, int A, uint32_t seed,
                              uint32_t sid, uint32_t ctr, const uint32_t* ctr_dev,
                              uint32_t row_offset, const float* uniforms, int mode,
                              int32_t* actions, int32_t* bad) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= B) return;
  if (ctr_dev) ctr += *ctr_dev;
  bool bad_row;
  const int y = sample_row(logits + (long long)m * ld, A, seed, sid, ctr, (uint32_t)m + row_offset,
                           uniforms ? uniforms + m : nullptr, mode, &bad_row);
  if (bad_row) atomicAdd(bad, 1);
  actions[m] = y;
}

// per-row entropy and log pi(a) (Categorical.entropy / log_prob, policies.py:87-89)
__global__ void categorical_kernel(const float* logits, int ld, int B, int A, const int32_t* actions,
                                   float* ent, float* lpa) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= B) return;
  const float* z = logits + (long long)m * ld;
  float mx = -INFINITY;
  for (int a = 0; a < A; ++a) mx = fmaxf(mx, z[a]);
  float se = 0.f;
  for (int a = 0; a < A; ++a) se += expf(z[a] - mx);
  const float lse = mx + logf(se);
  if (ent) {
    float H = 0.f;
    for (int a = 0; a < A; ++a) {
      const float lp = z[a] - lse;
      H -= expf(lp) * lp;
    }
    ent[m] = H;
  }
  if (lpa && actions) lpa[m] = z[actions[m]] - lse;
}

// ---------------------------------------------------------------------------
// n-step targets (objectives.py:178-214), one thread per env, reverse-free:
// target[t] = sum_{i=t..stop} r_i * gp[i-t]  (ascending i, mul+add, no FMA)
// ---------------------------------------------------------------------------
__global__ void returns_kernel(const float* r, const uint8_t* d, const float* v,
                               const float* vb, int N, int T, const float* gp,
                               const float* bp, float* tgt, float* adv) {
  // one thread per (env, step): the first terminal at or after t ends the sum
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long long)N * T) return;
  const int n = (int)(idx / T), t = (int)(idx - (long long)n * T);
  const float* rn = r + (long long)n * T;
  const uint8_t* dn = d + (long long)n * T;
  int next_term = T;  // index of the first terminal >= t (T = none)
  for (int i = T - 1; i >= t; --i)
    if (dn[i]) next_term = i;
  const int stop = next_term < T ? next_term : T - 1;
  float acc = 0.f;
  for (int i = t; i <= stop; ++i) acc = __fadd_rn(acc, __fmul_rn(rn[i], gp[i - t]));
  const float boot = next_term < T ? 0.f : __fmul_rn(bp[T - t], vb[n]);
  const float target = __fadd_rn(acc, boot);
  tgt[idx] = target;
  adv[idx] = __fsub_rn(target, v[idx]);
}

// ---------------------------------------------------------------------------
// GAE(lambda) targets (Schulman et al. 2016; an option beyond the reference,
// whose targets are the n-step returns above): one thread per env, reverse scan
//   delta_t = r_t + gamma V_{t+1} (1 - d_t) - V_t,   V_T = V_boot
//   A_t = delta_t + gamma lambda (1 - d_t) A_{t+1},  target_t = A_t + V_t
// with the operation order fixed (__f*_rn: no contraction) so the numpy float32
// restatement (oracle.gae_f32) is bit-exact.  lambda = 1 equals the n-step
// target in exact arithmetic.
// ---------------------------------------------------------------------------
__global__ void gae_kernel(const float* r, const uint8_t* d, const float* v, const float* vb, int N,
                           int T, float gamma, float gl, float* tgt, float* adv) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float next_v = vb[n], last = 0.f;
  for (int t = T - 1; t >= 0; --t) {
    const long long i = (long long)n * T + t;
    const bool live = d[i] == 0;
    const float vi = v[i];
    const float delta = __fsub_rn(__fadd_rn(r[i], live ? __fmul_rn(gamma, next_v) : 0.f), vi);
    last = __fadd_rn(delta, live ? __fmul_rn(gl, last) : 0.f);
    adv[i] = last;
    tgt[i] = __fadd_rn(last, vi);
    next_v = vi;
  }
}

// ---------------------------------------------------------------------------
// advantage normalisation (an option beyond the reference): batch moments in
// double, two fixed-order passes; normalise with the (all-reduced) moments
// ---------------------------------------------------------------------------
constexpr int MOM_BLOCKS = 256;

__global__ void adv_moments_partial_kernel(const float* a, long long M, double* part) {
  __shared__ double red[2][4];
  double s = 0.0, q = 0.0;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < M;
       i += (long long)gridDim.x * blockDim.x) {
    const double x = a[i];
    s += x;
    q += x * x;
  }
  s = wave_sum_d(s);
  q = wave_sum_d(q);
  if ((threadIdx.x & 63) == 0) red[0][threadIdx.x >> 6] = s, red[1][threadIdx.x >> 6] = q;
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    part[2 * blockIdx.x + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

__global__ void adv_moments_final_kernel(const double* part, int nb, double* out) {
  double s = 0.0, q = 0.0;  // one wave, lane-strided then butterfly
  for (int i = threadIdx.x; i < nb; i += 64) s += part[2 * i], q += part[2 * i + 1];
  s = wave_sum_d(s);
  q = wave_sum_d(q);
  if (threadIdx.x == 0) out[0] = s, out[1] = q;
}

__global__ void adv_normalize_kernel(float* a, long long M, const double* mom, double count, double eps) {
  const double mean = mom[0] / count;
  const double var = fmax(mom[1] / count - mean * mean, 0.0);
  const double inv = 1.0 / (sqrt(var) + eps);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < M;
       i += (long long)gridDim.x * blockDim.x)
    a[i] = (float)(((double)a[i] - mean) * inv);
}

// ---------------------------------------------------------------------------
// A2C loss + head gradients (objectives.py:123-154, :78)
// ---------------------------------------------------------------------------
constexpr int LOSS_BLOCK = 256;

__global__ void a2c_loss_kernel(const float* logits, int ld, const float* values,
                                const int32_t* actions, const float* targets,
                                const float* adv, int M, int A, float beta, float vcoef,
                                float gscale, float* dhead, int ldh, float* part) {
  __shared__ float red[3][LOSS_BLOCK / 64];
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  float s_pl = 0.f, s_h = 0.f, s_v = 0.f;
  if (m < M) {
    const float* z = logits + (long long)m * ld;
    float mx = -INFINITY;
    for (int a = 0; a < A; ++a) mx = fmaxf(mx, z[a]);
    float se = 0.f;
    for (int a = 0; a < A; ++a) se += expf(z[a] - mx);
    const float lse = mx + logf(se);
    float H = 0.f;
    for (int a = 0; a < A; ++a) {
      const float lp = z[a] - lse;
      H -= expf(lp) * lp;
    }
    const int act = actions[m];
    const float lpa = z[act] - lse;
    const float ad = adv[m];
    const float diff = targets[m] - values[m];
    s_pl = ad * lpa;
    s_h = H;
    s_v = 0.5f * diff * diff;
    // dL/dz_k = -(1/M)[adv (onehot_k - p_k) - beta p_k (log p_k + H)]
    const float inv = gscale / (float)M;
    float* g = dhead + (long long)m * ldh;
    for (int a = 0; a < A; ++a) {
      const float lp = z[a] - lse;
      const float p = expf(lp);
      const float oh = a == act ? 1.f : 0.f;
      g[a] = -inv * (ad * (oh - p) - beta * p * (lp + H));
    }
    // d(vcoef * L_v)/dV = vcoef * (V - target) / M
    g[A] = vcoef * inv * (values[m] - targets[m]);
    for (int a = A + 1; a < ldh; ++a) g[a] = 0.f;
  }
  s_pl = wave_sum(s_pl);
  s_h = wave_sum(s_h);
  s_v = wave_sum(s_v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = s_pl;
    red[1][w] = s_h;
    red[2][w] = s_v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, b = 0.f, c = 0.f;
    for (int i = 0; i < LOSS_BLOCK / 64; ++i) {
      a += red[0][i];
      b += red[1][i];
      c += red[2][i];
    }
    part[blockIdx.x * 3 + 0] = a;
    part[blockIdx.x * 3 + 1] = b;
    part[blockIdx.x * 3 + 2] = c;
  }
}

__global__ void a2c_loss_final_kernel(const float* part, int nb, int M, float beta,
                                      float scale, float* out) {
  // one wave: deterministic fixed-order sums
  float a = 0.f, b = 0.f, c = 0.f;
  for (int i = threadIdx.x; i < nb; i += 64) {
    a += part[i * 3 + 0];
    b += part[i * 3 + 1];
    c += part[i * 3 + 2];
  }
  a = wave_sum(a);
  b = wave_sum(b);
  c = wave_sum(c);
  if (threadIdx.x == 0) {
    // scale = 1/world_size: the SUM all-reduce of the update buffer then leaves
    // the global means (every rank holds M rows)
    const float mean_pl = a / (float)M;
    const float mean_h = b / (float)M;
    out[0] = scale * -(mean_pl + beta * mean_h);
    out[1] = scale * (c / (float)M);
    out[2] = scale * mean_h;
  }
}

// ---------------------------------------------------------------------------
// deterministic global sum of squares / dot product (two passes)
// ---------------------------------------------------------------------------
constexpr int RED_BLOCKS = 512;

__global__ void dot_partial_kernel(const float* x, const float* y, long long n, float* part) {
  __shared__ float red[4];
  float s = 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    s += x[i] * y[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__device__ float block_final_sum(const float* part, int nb) {
  // called by one full block of 256: fixed-order reduction
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) s += part[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  const float tot = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return tot;
}

// scale[0] = clip factor (TF clip_by_global_norm), scale[1] = global norm
__global__ void clip_scale_kernel(const float* part, int nb, float clip_norm, float* scale,
                                  float* norm_out) {
  const float ss = block_final_sum(part, nb);
  if (threadIdx.x == 0) {
    const float gn = sqrtf(ss);
    float sc = 1.f;
    if (clip_norm > 0.f) sc = clip_norm * fminf(1.f / gn, 1.f / clip_norm);
    scale[0] = sc;
    scale[1] = gn;
    if (norm_out) norm_out[0] = gn;
  }
}

__global__ void momentum_kernel(float* p, float* acc, const float* g, long long n, float lr,
                                float mom, const float* scale) {
  const float sc = scale[0];
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const float a = mom * acc[i] + g[i] * sc;
    acc[i] = a;
    p[i] -= lr * a;
  }
}

__global__ void rmsprop_kernel(float* p, float* ms, float* mom, const float* g, long long n,
                               float lr, float decay, float momentum, float eps,
                               const float* scale) {
  const float sc = scale[0];
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const float gi = g[i] * sc;
    const float m2 = decay * ms[i] + (1.f - decay) * gi * gi;
    ms[i] = m2;
    const float mo = momentum * mom[i] + lr * gi / sqrtf(m2 + eps);
    mom[i] = mo;
    p[i] -= mo;
  }
}

// ---------------------------------------------------------------------------
// batched synthetic Atari stepper (multi_env.py:121-137 + wrappers.py:201-235
// + wrappers.py:263-323).  One workgroup per env; 1764 words of 4 pixels.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void env_reset_kernel(acmi_env_state_t st, int env_offset,
                                                        uint32_t seed, uint8_t* obs,
                                                        long long stride) {
  const int n = blockIdx.x;
  const uint32_t e = (uint32_t)(env_offset + n);
  const GameParams gp = game_params(env_game(st, n));
  const uint32_t base = key4(seed ^ gp.salt, e, 0u, RESET_TAG);
  uint4* out = reinterpret_cast<uint4*>(obs + (long long)n * stride);
  for (int g = threadIdx.x; g < FRAME_WORDS; g += blockDim.x) {
    const uint32_t w = word_hash(base, (uint32_t)g);
    uint4 o;
    o.x = (w & 255u) * 0x01010101u;
    o.y = ((w >> 8) & 255u) * 0x01010101u;
    o.z = ((w >> 16) & 255u) * 0x01010101u;
    o.w = (w >> 24) * 0x01010101u;
    out[g] = o;
  }
  if (threadIdx.x == 0) {
    st.episode[n] = 0;
    st.step[n] = 0;
    st.length[n] = episode_length(seed, e, 0u, gp);
    st.total[n] = 0.f;
    st.done[n] = 0;
  }
}

__global__ __launch_bounds__(256) void env_step_kernel(
    acmi_env_state_t st, int env_offset, uint32_t seed, const int32_t* actions,
    const uint8_t* obs_in, long long in_stride, uint8_t* obs_out, long long out_stride,
    float* rewards, uint8_t* terminals, float* ep_rewards, long long ld) {
  const int n = blockIdx.x;
  env_step_block(st, n, (uint32_t)(env_offset + n), seed, (uint32_t)actions[n],
                 obs_in + (long long)n * in_stride, obs_out + (long long)n * out_stride, rewards,
                 terminals, ep_rewards, ld);
}

}  // namespace acmi

using namespace acmi;

extern "C" {

int acmi_sample_actions(const float* logits, int ld, int B, int A, uint32_t seed,
                        uint32_t stream_id, uint32_t counter, const float* uniforms, int mode,
                        int32_t* actions, int32_t* bad_rows, acmi_stream_t stream) {
  return acmi_sample_actions_at(logits, ld, B, A, seed, stream_id, counter, 0, uniforms, mode,
                                actions, bad_rows, stream);
}

int acmi_sample_actions_at(const float* logits, int ld, int B, int A, uint32_t seed,
                           uint32_t stream_id, uint32_t counter, int row_offset,
                           const float* uniforms, int mode, int32_t* actions, int32_t* bad_rows,
                           acmi_stream_t stream) {
  return acmi_sample_actions_dev(logits, ld, B, A, seed, stream_id, nullptr, counter, row_offset,
                                 uniforms, mode, actions, bad_rows, stream);
}

int acmi_sample_actions_dev(const float* logits, int ld, int B, int A, uint32_t seed,
                            uint32_t stream_id, const uint32_t* counter_dev, uint32_t counter_add,
                            int row_offset, const float* uniforms, int mode, int32_t* actions,
                            int32_t* bad_rows, acmi_stream_t stream) {
  ACMI_REQUIRE(logits && actions && bad_rows && B >= 0 && A >= 1 && ld >= A && row_offset >= 0,
               ACMI_ERR_ARG, "acmi_sample_actions: bad arguments");
  if (B == 0) return ACMI_OK;
  hipLaunchKernelGGL(sample_kernel, dim3(cdiv(B, 256)), dim3(256), 0, (hipStream_t)stream,
                     logits, ld, B, A, seed, stream_id, counter_add, counter_dev,
                     (uint32_t)row_offset, uniforms, mode, actions, bad_rows);
  ACMI_LAUNCH_CHECK("acmi_sample_actions");
  return ACMI_OK;
}

int acmi_categorical(const float* logits, int ld, int B, int A, const int32_t* actions,
                     float* entropy, float* log_prob, acmi_stream_t stream) {
  ACMI_REQUIRE(logits && B >= 0 && A >= 1 && ld >= A && (entropy || log_prob) && (!log_prob || actions),
               ACMI_ERR_ARG, "acmi_categorical: bad arguments");
  if (B == 0) return ACMI_OK;
  hipLaunchKernelGGL(categorical_kernel, dim3(cdiv(B, 256)), dim3(256), 0, (hipStream_t)stream, logits, ld,
                     B, A, actions, entropy, log_prob);
  ACMI_LAUNCH_CHECK("acmi_categorical");
  return ACMI_OK;
}

int acmi_returns(const float* rewards, const uint8_t* terminals, const float* values,
                 const float* v_boot, int N, int T, const float* gamma_pow,
                 const float* boot_pow, float* targets, float* adv, acmi_stream_t stream) {
  ACMI_REQUIRE(rewards && terminals && values && v_boot && gamma_pow && boot_pow && targets &&
                   adv && N >= 0 && T >= 1,
               ACMI_ERR_ARG, "acmi_returns: bad arguments");
  if (N == 0) return ACMI_OK;
  hipLaunchKernelGGL(returns_kernel, dim3(cdiv((long long)N * T, 256)), dim3(256), 0, (hipStream_t)stream,
                     rewards, terminals, values, v_boot, N, T, gamma_pow, boot_pow, targets,
                     adv);
  ACMI_LAUNCH_CHECK("acmi_returns");
  return ACMI_OK;
}

int acmi_gae(const float* rewards, const uint8_t* terminals, const float* values, const float* v_boot,
             int N, int T, float gamma, float lambda, float* targets, float* adv, acmi_stream_t stream) {
  ACMI_REQUIRE(rewards && terminals && values && v_boot && targets && adv && N >= 0 && T >= 1 &&
                   lambda >= 0.f && lambda <= 1.f,
               ACMI_ERR_ARG, "acmi_gae: bad arguments");
  if (N == 0) return ACMI_OK;
  hipLaunchKernelGGL(gae_kernel, dim3(cdiv(N, 64)), dim3(64), 0, (hipStream_t)stream, rewards, terminals,
                     values, v_boot, N, T, gamma, gamma * lambda, targets, adv);
  ACMI_LAUNCH_CHECK("acmi_gae");
  return ACMI_OK;
}

int64_t acmi_adv_moments_ws_doubles(int64_t M) { (void)M; return 2LL * MOM_BLOCKS; }

int acmi_adv_moments(const float* adv, int64_t M, double* ws, double* moments, acmi_stream_t stream) {
  ACMI_REQUIRE(adv && ws && moments && M >= 1, ACMI_ERR_ARG, "acmi_adv_moments: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(adv_moments_partial_kernel, dim3(MOM_BLOCKS), dim3(256), 0, s, adv, (long long)M, ws);
  hipLaunchKernelGGL(adv_moments_final_kernel, dim3(1), dim3(64), 0, s, ws, MOM_BLOCKS, moments);
  ACMI_LAUNCH_CHECK("acmi_adv_moments");
  return ACMI_OK;
}

int acmi_adv_normalize(float* adv, int64_t M, const double* moments, double count, double eps,
                       acmi_stream_t stream) {
  ACMI_REQUIRE(adv && moments && M >= 1 && count >= 1.0 && eps >= 0.0, ACMI_ERR_ARG,
               "acmi_adv_normalize: bad arguments");
  hipLaunchKernelGGL(adv_normalize_kernel, dim3(std::min<long long>(cdiv(M, 256), 1024)), dim3(256), 0,
                     (hipStream_t)stream, adv, (long long)M, moments, count, eps);
  ACMI_LAUNCH_CHECK("acmi_adv_normalize");
  return ACMI_OK;
}

int64_t acmi_a2c_loss_ws_floats(int M) { return 3LL * cdiv(M, LOSS_BLOCK) + 16; }

int acmi_a2c_loss(const float* logits, int ld, const float* values, const int32_t* actions,
                  const float* targets, const float* adv, int M, int A, float beta, float vcoef,
                  float grad_scale, float* dhead, int ldh, float* ws, float* loss_out,
                  acmi_stream_t stream) {
  ACMI_REQUIRE(logits && values && actions && targets && adv && dhead && ws && loss_out &&
                   M > 0 && A >= 1 && ld >= A && ldh >= A + 1,
               ACMI_ERR_ARG, "acmi_a2c_loss: bad arguments");
  const int nb = cdiv(M, LOSS_BLOCK);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(a2c_loss_kernel, dim3(nb), dim3(LOSS_BLOCK), 0, s, logits, ld, values,
                     actions, targets, adv, M, A, beta, vcoef, grad_scale, dhead, ldh, ws);
  hipLaunchKernelGGL(a2c_loss_final_kernel, dim3(1), dim3(64), 0, s, ws, nb, M, beta,
                     grad_scale, loss_out);
  ACMI_LAUNCH_CHECK("acmi_a2c_loss");
  return ACMI_OK;
}

int64_t acmi_opt_ws_floats(int64_t n) { (void)n; return RED_BLOCKS + 16; }

static int clip_prologue(const float* g, long long n, float clip_norm, float* ws,
                         float* norm_out, hipStream_t s) {
  hipLaunchKernelGGL(dot_partial_kernel, dim3(RED_BLOCKS), dim3(256), 0, s, g, g, n, ws);
  hipLaunchKernelGGL(clip_scale_kernel, dim3(1), dim3(256), 0, s, ws, RED_BLOCKS, clip_norm,
                     ws + RED_BLOCKS, norm_out);
  ACMI_LAUNCH_CHECK("clip_by_global_norm");
  return ACMI_OK;
}

int acmi_momentum_apply(float* params, float* accum, const float* grads, int64_t n, float lr,
                        float momentum, float clip_norm, float* ws, float* norm_out,
                        acmi_stream_t stream) {
  ACMI_REQUIRE(params && accum && grads && ws && n > 0, ACMI_ERR_ARG,
               "acmi_momentum_apply: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  int rc = clip_prologue(grads, n, clip_norm, ws, norm_out, s);
  if (rc) return rc;
  hipLaunchKernelGGL(momentum_kernel, dim3(std::min<long long>(cdiv(n, 256), 2048)), dim3(256),
                     0, s, params, accum, grads, (long long)n, lr, momentum, ws + RED_BLOCKS);
  ACMI_LAUNCH_CHECK("acmi_momentum_apply");
  return ACMI_OK;
}

int acmi_rmsprop_apply(float* params, float* ms, float* mom, const float* grads, int64_t n,
                       float lr, float decay, float momentum, float eps, float clip_norm,
                       float* ws, float* norm_out, acmi_stream_t stream) {
  ACMI_REQUIRE(params && ms && mom && grads && ws && n > 0, ACMI_ERR_ARG,
               "acmi_rmsprop_apply: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  int rc = clip_prologue(grads, n, clip_norm, ws, norm_out, s);
  if (rc) return rc;
  hipLaunchKernelGGL(rmsprop_kernel, dim3(std::min<long long>(cdiv(n, 256), 2048)), dim3(256),
                     0, s, params, ms, mom, grads, (long long)n, lr, decay, momentum, eps,
                     ws + RED_BLOCKS);
  ACMI_LAUNCH_CHECK("acmi_rmsprop_apply");
  return ACMI_OK;
}

int acmi_env_reset(const acmi_env_state_t* st, int N, int env_offset, uint32_t seed,
                   uint8_t* obs_out, int64_t out_stride, acmi_stream_t stream) {
  ACMI_REQUIRE(st && obs_out && N >= 0 && out_stride >= 84 * 84 * 4 && out_stride % 16 == 0,
               ACMI_ERR_ARG, "acmi_env_reset: bad arguments");
  if (N == 0) return ACMI_OK;
  hipLaunchKernelGGL(env_reset_kernel, dim3(N), dim3(256), 0, (hipStream_t)stream, *st,
                     env_offset, seed, obs_out, (long long)out_stride);
  ACMI_LAUNCH_CHECK("acmi_env_reset");
  return ACMI_OK;
}

int acmi_env_step(const acmi_env_state_t* st, int N, int env_offset, uint32_t seed,
                  const int32_t* actions, const uint8_t* obs_in, int64_t in_stride,
                  uint8_t* obs_out, int64_t out_stride, float* rewards, uint8_t* terminals,
                  float* episode_rewards, int64_t ld, acmi_stream_t stream) {
  ACMI_REQUIRE(st && actions && obs_in && obs_out && rewards && terminals && episode_rewards &&
                   N >= 0 && in_stride % 16 == 0 && out_stride % 16 == 0 && ld >= 1,
               ACMI_ERR_ARG, "acmi_env_step: bad arguments");
  if (N == 0) return ACMI_OK;
  hipLaunchKernelGGL(env_step_kernel, dim3(N), dim3(256), 0, (hipStream_t)stream, *st,
                     env_offset, seed, actions, obs_in, (long long)in_stride, obs_out,
                     (long long)out_stride, rewards, terminals, episode_rewards,
                     (long long)ld);
  ACMI_LAUNCH_CHECK("acmi_env_step");
  return ACMI_OK;
}

}  // extern "C"
