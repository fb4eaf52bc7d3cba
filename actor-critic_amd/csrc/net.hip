// Nature-CNN policy/value tower on gfx950: forward, backward fused with the
// K-FAC input-factor statistics, and the sampled-loss output statistics.
//
// Reference: envs/atari/model.py:77-217 (graph), :219-246 (K-FAC layer
// registration), nn.py:37-126 (layer math), policies.py:146-158 and
// baselines.py:55-69 (predictive distributions), objectives.py:78 (the
// tf.gradients of the shared loss).  See include/acmi.h for the contract.
#include <math.h>
#include <stdlib.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "gemm.hpp"
#include "gemm3.hpp"
#include "conv1u8.hpp"
#include "convt3.hpp"
#include "convfwd3.hpp"
#include "band.hpp"
#include "tower.hpp"
#include "fc4roll.hpp"
#include "convt2.hpp"
#include "stepper.hpp"
#include "towersplit.hpp"

namespace acmi {

// Arithmetic modes.  Process-wide defaults (acmi_set_*_mode; initial values from
// the environment) and the modes in effect for the calling thread's current
// entry point: a net's own (acmi_net_t gemm_mode / forward_mode /
// conv_stats_mode, each mode + 1) or the defaults (ModeScope).
//   gemm:  ACMI_GEMM_X3 = 16-bit split operands (f16x2 / bf16x3, f32-accurate),
//          ACMI_GEMM_F32 = v_mfma_f32_32x32x2_f32; ACMI_GEMM ("f32" / "x3"), default x3
//   conv stats: pixel-pair band reduction (band.hpp, x3 only) or patch rows; ACMI_BAND ("0": patches)
//   forward: the conv tower's precision; ACMI_FORWARD ("bf16" / "f32")
static int s_gemm_mode = [] {
  const char* e = getenv("ACMI_GEMM");
  return (e && e[0] == 'f') ? ACMI_GEMM_F32 : ACMI_GEMM_X3;
}();
static int s_conv_stats_mode = [] {
  const char* e = getenv("ACMI_BAND");
  return (e && e[0] == '0') ? ACMI_CONV_STATS_PATCHES : ACMI_CONV_STATS_BAND;
}();
static int s_forward_mode = [] {
  const char* e = getenv("ACMI_FORWARD");
  return (e && e[0] == 'b') ? ACMI_FWD_BF16 : ACMI_FWD_F32;
}();
thread_local int g_gemm_mode = s_gemm_mode;
thread_local int g_conv_stats_mode = s_conv_stats_mode;
thread_local int g_forward_mode = s_forward_mode;

// a net's mode fields (0: the process default) are valid
static bool net_modes_ok(const acmi_net_t* n) {
  if (!n) return true;
  const int g = n->gemm_mode ? n->gemm_mode - 1 : s_gemm_mode;
  const int f = n->forward_mode ? n->forward_mode - 1 : s_forward_mode;
  const int c = n->conv_stats_mode ? n->conv_stats_mode - 1 : s_conv_stats_mode;
  return (g == ACMI_GEMM_F32 || g == ACMI_GEMM_X3) && (f == ACMI_FWD_F32 || f == ACMI_FWD_BF16) &&
         (c == ACMI_CONV_STATS_PATCHES || c == ACMI_CONV_STATS_BAND) && (f == ACMI_FWD_F32 || g == ACMI_GEMM_X3);
}
// the modes of one entry point's call, restored when it returns (thread-local:
// calls on different threads with different nets do not interfere)
struct ModeScope {
  int g, f, c;
  explicit ModeScope(const acmi_net_t* n) : g(g_gemm_mode), f(g_forward_mode), c(g_conv_stats_mode) {
    g_gemm_mode = n && n->gemm_mode ? n->gemm_mode - 1 : s_gemm_mode;
    g_forward_mode = n && n->forward_mode ? n->forward_mode - 1 : s_forward_mode;
    g_conv_stats_mode = n && n->conv_stats_mode ? n->conv_stats_mode - 1 : s_conv_stats_mode;
  }
  ~ModeScope() {
    g_gemm_mode = g;
    g_forward_mode = f;
    g_conv_stats_mode = c;
  }
};

static thread_local char g_err[512];
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// ---------------------------------------------------------------------------
// launch-site profiling: HIP events recorded on the launch stream around one
// chosen kernel (acmi_prof_enable), summed by acmi_prof_collect.
// ---------------------------------------------------------------------------
static int g_prof_site = 0;
static int g_prof_cap = 0;
static int g_prof_n = 0;
static hipEvent_t* g_prof_ev = nullptr;  // 2 * cap events

static void prof_begin(int site, hipStream_t s) {
  if (site != g_prof_site || g_prof_n >= g_prof_cap) return;
  (void)hipEventRecord(g_prof_ev[2 * g_prof_n], s);
}
static void prof_end(int site, hipStream_t s) {
  if (site != g_prof_site || g_prof_n >= g_prof_cap) return;
  (void)hipEventRecord(g_prof_ev[2 * g_prof_n + 1], s);
  ++g_prof_n;
}

// ---------------------------------------------------------------------------
// layout
// ---------------------------------------------------------------------------
struct Layout {
  int A, C3;
  long long off[12];  // W, b per layer
  long long total;
  long long K[6], N[6];
  long long din[6], dout[6];
  long long stat_off[11], stat_total;
  long long rows_per_img[6];  // output locations per image (conv L, fc 1)
};

static bool make_layout(int A, int C3, Layout* L) {
  if (A < 1 || A > 64 || (C3 != 32 && C3 != 64)) return false;
  L->A = A;
  L->C3 = C3;
  const long long K[6] = {8 * 8 * 4, 4 * 4 * 32, 3 * 3 * 64, 49LL * C3, 512, 512};
  const long long N[6] = {32, 64, C3, 512, A, 1};
  const long long R[6] = {400, 81, 49, 1, 1, 1};
  long long o = 0;
  for (int l = 0; l < 6; ++l) {
    L->K[l] = K[l];
    L->N[l] = N[l];
    L->din[l] = K[l] + 1;
    L->dout[l] = N[l];
    L->rows_per_img[l] = R[l];
    L->off[2 * l] = o;
    o += K[l] * N[l];
    L->off[2 * l + 1] = o;
    o += N[l];
  }
  L->total = o;
  long long s = 0;
  for (int f = 0; f < 5; ++f) {
    L->stat_off[f] = s;
    s += L->din[f] * L->din[f];
  }
  for (int l = 0; l < 6; ++l) {
    L->stat_off[5 + l] = s;
    s += L->dout[l] * L->dout[l];
  }
  L->stat_total = s;
  return true;
}

bool get_layout(int A, int C3, Layout* L) { return make_layout(A, C3, L); }

// ---------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------
// d4 = (dhead [W_pi | w_v]^T) * relu'(a4): A+1 MACs per output, elementwise
// over [B][512] (memory-bound); the k-ordered fmaf chain is the f32 MFMA's.
// amax (nullable): max |d4| published for fc4's f16x2 input gradient, once per
// block (common.hpp amax_update; every thread reaches the block reduction,
// out-of-range ones contribute 0)
__device__ __forceinline__ void block_amax256(unsigned* amax, float m) {
  __shared__ float red[4];
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) amax_update(amax, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
}
__device__ __forceinline__ float absmax4f(float4 r) {
  return fmaxf(fmaxf(fabsf(r.x), fabsf(r.y)), fmaxf(fabsf(r.z), fabsf(r.w)));
}

__global__ __launch_bounds__(256) void heads_dx_kernel(const float* dhead, int ldh, int B, const float* wpi,
                                                       const float* wv, int A, const float* a4, float* d4,
                                                       unsigned* amax) {
  // 4 consecutive outputs per thread (float4 a4 / d4)
  const long long q0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool ok = q0 < (long long)B * 128;
  const long long q = ok ? q0 : 0;
  const int m = (int)(q >> 7), j0 = (int)(q & 127) * 4;
  const float* g = dhead + (long long)m * ldh;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int a = 0; a < A; ++a) {
    const float ga = g[a];
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[e] = __builtin_fmaf(ga, wpi[(j0 + e) * A + a], acc[e]);
  }
  const float gv = g[A];  // (wv is not 16-byte aligned for every A: scalar loads)
#pragma unroll
  for (int e = 0; e < 4; ++e) acc[e] = __builtin_fmaf(gv, wv[j0 + e], acc[e]);
  const float4 x = *reinterpret_cast<const float4*>(a4 + q * 4);
  // masks as multiplies by 0/1 of the computed sums (a select with a load
  // operand would be turned into a branch around the load)
  float4 o;
  o.x = acc[0] * (float)(x.x > 0.f);
  o.y = acc[1] * (float)(x.y > 0.f);
  o.z = acc[2] * (float)(x.z > 0.f);
  o.w = acc[3] * (float)(x.w > 0.f);
  if (ok) *reinterpret_cast<float4*>(d4 + q * 4) = o;
  if (amax) block_amax256(amax, ok ? absmax4f(o) : 0.f);
}

// Breakout's A = 4 (16-byte aligned W_pi rows, dhead rows of ldh % 4 == 0): the
// four W_pi rows and the dhead row as float4 loads (7 loads a thread instead of 26),
// the same k-ordered fmaf chain per output
__global__ __launch_bounds__(256) void heads_dx4_kernel(const float* dhead, int ldh, int B, const float* wpi,
                                                        const float* wv, const float* a4, float* d4,
                                                        unsigned* amax) {
  const long long q0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool ok = q0 < (long long)B * 128;
  const long long q = ok ? q0 : 0;
  const int m = (int)(q >> 7), j0 = (int)(q & 127) * 4;
  const float* g = dhead + (long long)m * ldh;
  const float4 g4 = *reinterpret_cast<const float4*>(g);
  const float gv = g[4];
  const float4* w4 = reinterpret_cast<const float4*>(wpi + j0 * 4);
  const float4 x = *reinterpret_cast<const float4*>(a4 + q * 4);
  float o[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float4 w = w4[e];
    float acc = __builtin_fmaf(g4.x, w.x, 0.f);
    acc = __builtin_fmaf(g4.y, w.y, acc);
    acc = __builtin_fmaf(g4.z, w.z, acc);
    acc = __builtin_fmaf(g4.w, w.w, acc);
    o[e] = __builtin_fmaf(gv, wv[j0 + e], acc);
  }
  float4 r;
  r.x = o[0] * (float)(x.x > 0.f);
  r.y = o[1] * (float)(x.y > 0.f);
  r.z = o[2] * (float)(x.z > 0.f);
  r.w = o[3] * (float)(x.w > 0.f);
  if (ok) *reinterpret_cast<float4*>(d4 + q * 4) = r;
  if (amax) block_amax256(amax, ok ? absmax4f(r) : 0.f);
}

// acmi_acts_t's masks: all three or none
static bool masks_ok(const acmi_acts_t* a) { return (a->m1 && a->m2 && a->m3) || (!a->m1 && !a->m2 && !a->m3); }

// ReLU' bit masks from the f32 activations, for the per-layer forward (the tower
// writes them itself): word k of image b (wpi words per image, one per 32
// channels) = bits (act > 0) of its 32 floats; images st apart in both buffers
__global__ void act_mask_kernel(const float* act, int B, int wpi, long long st, uint32_t* mask) {
  const long long w = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= (long long)B * wpi) return;
  const long long b = w / wpi, k = w - b * wpi;
  const float4* src = reinterpret_cast<const float4*>(act + (b * st * wpi + k) * 32);
  uint32_t bits = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float4 v = src[q];
    bits |= (uint32_t)(v.x > 0.f) << (4 * q) | (uint32_t)(v.y > 0.f) << (4 * q + 1) |
            (uint32_t)(v.z > 0.f) << (4 * q + 2) | (uint32_t)(v.w > 0.f) << (4 * q + 3);
  }
  mask[b * st * wpi + k] = bits;
}

// conv/fc epilogue with an image remap so the rollout can write step t of an
// env-major [N][T][rows] activation buffer in place.
struct EpiAct {
  float* out;
  const float* bias;
  int cols;         // output channels (row length)
  int L;            // output rows per image
  long long img_stride;  // floats between consecutive images in `out`
  float scale = 1.f;     // conv1: 1/255 (its A operand is the raw u8 pixels)
  __device__ __forceinline__ float aux(int, int j) const { return bias[j]; }
  __device__ __forceinline__ void store(int i, int j, float v, float b) const {
    const uint32_t img = (uint32_t)i / (uint32_t)L;
    const uint32_t p = (uint32_t)i - img * (uint32_t)L;
    out[(long long)img * img_stride + (long long)p * cols + j] = fmaxf(__builtin_fmaf(v, scale, b), 0.f);
  }
};


// Fused rollout tail (acmi_rollout_step): one workgroup per env b -- a4 from
// fc4's split-K slabs (or as stored), the A+1 heads, the categorical draw and
// the env step, with the arithmetic of heads_kernel / sample_kernel /
// env_step_kernel (same per-element orders), so the fused step is bit-identical
// to the three launches it replaces.
struct TailArgs {
  acmi_rollout_io_t io;
  const uint8_t* obs;
  long long img_stride;
};
constexpr int kMaxHeads = 32;
// sx [512], sl [kMaxHeads], s_action: the block's scratch in LDS; mirror
// (nullable): the new stack also goes there (the fused next-step tower's image)
// SPLIT (towersplit.hpp): one of kSplitParts workgroups of env `row` (part `spart`):
// the heads and the draw are computed by every part (the same arithmetic, so the
// same action), only part 0 stores them; the env step builds the stack words the
// part's tower needs (env_step_part) and the post-step state goes to pend.
template <int NZ, bool SPLIT = false>
__device__ __forceinline__ void rollout_tail_body(
    const float* part, int nz, const float* b4, float* a4, long long a4_stride, int B,
    const float* wpi, const float* bpi, const float* wv, const float* bv, int A, float* logits,
    long long l_stride, float* value, long long v_stride, const TailArgs& ta, float* sx, float* sl,
    int& s_action, uint4* mirror, int row = -1, int spart = 0, PendState* pend = nullptr) {
  if (row < 0) row = blockIdx.x;
  const bool writer = spart == 0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  EnvPre pre;  // the env's state and current stack: in flight during the heads
  if constexpr (!SPLIT) env_prefetch(ta.io.state, row, ta.obs + (long long)row * ta.img_stride, pre);
  if (!SPLIT && ta.io.obs_copy) {  // the stacks this step read, filed where the batch keeps them
    uint4* cp = reinterpret_cast<uint4*>(ta.io.obs_copy + (long long)row * ta.io.out_stride);
#pragma unroll
    for (int i = 0; i < kEnvWords; ++i) {
      const int g = threadIdx.x + kEnvThreads * i;
      if (g < FRAME_WORDS) cp[g] = pre.old[i];
    }
  }
  // head a's weight for a4 element lane + 64 e (a == A: the value head); the
  // wave's first two heads are loaded now, beside the slab and stack loads
  auto head_w = [&](int a, int e) {
    const int ai = a < A ? a : 0;
    return a < A ? wpi[(lane + 64 * e) * A + ai] : wv[lane + 64 * e];
  };
  float hw[2][8];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int e = 0; e < 8; ++e) hw[h][e] = head_w(min(wave + 4 * h, A), e);  // (unused past A)
  float* x = a4 + (long long)row * a4_stride;
  if (NZ > 0) {
    // both columns' NZ slab loads issued before the (fixed-order) sums
    const long long zs = (long long)(B + 1) * 512;
    float pv[2][NZ > 0 ? NZ : 1];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int z = 0; z < NZ; ++z) pv[h][z] = part[z * zs + (long long)row * 512 + threadIdx.x + 256 * h];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = threadIdx.x + 256 * h;
      float acc = 0.f;
#pragma unroll
      for (int z = 0; z < NZ; ++z) acc += pv[h][z];
      const float v = fmaxf(acc + b4[j], 0.f);
      if (writer) x[j] = v;
      sx[j] = v;
    }
  } else {
    for (int j = threadIdx.x; j < 512; j += 256) sx[j] = x[j];
  }
  __syncthreads();
  float xv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) xv[e] = sx[lane + 64 * e];
  auto head = [&](int a, const float (&w)[8]) {  // head a (a == A: the value head)
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) s += xv[e] * w[e];
    s = wave_sum(s);
    if (lane == 0) sl[a] = s + (a < A ? bpi[a] : bv[0]);
  };
  if (wave <= A) head(wave, hw[0]);
  if (wave + 4 <= A) head(wave + 4, hw[1]);
  for (int a = wave + 8; a <= A; a += 4) {
    float w[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) w[e] = head_w(a, e);
    head(a, w);
  }
  __syncthreads();
  const acmi_rollout_io_t& io = ta.io;
  if (threadIdx.x == 0) {
    if (writer) {
      for (int a = 0; a < A; ++a) logits[(long long)row * l_stride + a] = sl[a];
      if (value) value[(long long)row * v_stride] = sl[A];
    }
    const uint32_t ctr = io.counter + (io.counter_dev ? *io.counter_dev : 0u);
    bool bad;
    const int y = sample_row(sl, A, io.seed, io.stream_id, ctr, (uint32_t)(row + io.row_offset),
                             nullptr, 0, &bad);
    if (writer) {
      if (bad) atomicAdd(io.bad_rows, 1);
      io.actions[(long long)row * io.ld] = y;
    }
    s_action = y;
  }
  __syncthreads();
  if constexpr (SPLIT) {
    env_step_part(io.state, row, (uint32_t)(io.env_offset + row), io.env_seed, (uint32_t)s_action,
                  ta.obs + (long long)row * ta.img_stride, split_word_lo(spart), split_word_hi(spart),
                  split_own_lo(spart), split_own_hi(spart), io.obs_out + (long long)row * io.out_stride,
                  io.obs_copy ? io.obs_copy + (long long)row * io.out_stride : nullptr, mirror, writer, io.rewards,
                  io.terminals, io.episode_rewards, io.ld, pend);
  } else {
    env_step_block_pre(io.state, row, (uint32_t)(io.env_offset + row), io.env_seed, (uint32_t)s_action, pre,
                       io.obs_out + (long long)row * io.out_stride, io.rewards, io.terminals,
                       io.episode_rewards, io.ld, mirror);
  }
}

template <int NZ>
__global__ __launch_bounds__(256) void rollout_tail_kernel(
    const float* part, int nz, const float* b4, float* a4, long long a4_stride, int B,
    const float* wpi, const float* bpi, const float* wv, const float* bv, int A, float* logits,
    long long l_stride, float* value, long long v_stride, TailArgs ta) {
  __shared__ float sx[512];
  __shared__ float sl[kMaxHeads];
  __shared__ int s_action;
  rollout_tail_body<NZ>(part, nz, b4, a4, a4_stride, B, wpi, bpi, wv, bv, A, logits, l_stride, value, v_stride,
                        ta, sx, sl, s_action, nullptr);
}

// The rollout tail of step t fused with the conv tower of step t + 1 (the
// acmi_rollout_io_t next_acts contract): the env step leaves the new stack in
// the tower's LDS image as well as in obs_out, the tower then runs on it --
// one launch and one image round trip fewer per step, the same arithmetic.
// The tail's scratch sits in the tower's a1 region (unused until conv1's
// epilogue).  Two blocks per CU, like the tower.
struct NextTower {
  const float *b1, *b2, *b3;
  float *a1, *a2, *a3;
  long long st;
  const char* prep;
  uint32_t *m1, *m2, *m3;
};
template <int NZ, int C3, bool H16>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void rollout_tail_tower_kernel(
    const float* part, int nz, const float* b4, float* a4, long long a4_stride, int B,
    const float* wpi, const float* bpi, const float* wv, const float* bv, int A, float* logits,
    long long l_stride, float* value, long long v_stride, TailArgs ta, NextTower nt) {
  __shared__ __attribute__((aligned(16))) char lds[kTowLds + kTowScr];
  float* sx = reinterpret_cast<float*>(lds + kTowObs);
  int* s_action = reinterpret_cast<int*>(sx + 512 + kMaxHeads);
  rollout_tail_body<NZ>(part, nz, b4, a4, a4_stride, B, wpi, bpi, wv, bv, A, logits, l_stride, value, v_stride,
                        ta, sx, sx + 512, *s_action, reinterpret_cast<uint4*>(lds));
  __syncthreads();  // the image in LDS; the tail's scratch free again
  tower_body<C3, H16, true>(nullptr, 0, nt.b1, nt.b2, nt.b3, nt.a1, nt.a2, nt.a3, nt.st, nt.prep, nt.m1, nt.m2,
                            nt.m3, lds, blockIdx.x);
}

// The split rollout step (small batches, towersplit.hpp): kSplitParts workgroups
// per env -- the tail (redundant heads / draw, the env step's words each part's
// tower needs, the post-step state into pend) and then part j of the next
// step's conv tower.  The pending states are committed by the next step's fc4
// launch (fc4_roll_kernel: env_commit_pending), the first launch after this one.
template <int NZ, int C3, bool H16>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void rollout_tail_split_kernel(
    const float* part, int nz, const float* b4, float* a4, long long a4_stride, int B,
    const float* wpi, const float* bpi, const float* wv, const float* bv, int A, float* logits,
    long long l_stride, float* value, long long v_stride, TailArgs ta, NextTower nt, PendState* pend) {
  __shared__ __attribute__((aligned(16))) char lds[kSpLds];
  const int n = blockIdx.x / kSplitParts, j = blockIdx.x - n * kSplitParts;
  float* sx = reinterpret_cast<float*>(lds + kSpImg);  // the tail's scratch in the a1 image
  int* s_action = reinterpret_cast<int*>(sx + 512 + kMaxHeads);
  rollout_tail_body<NZ, true>(part, nz, b4, a4, a4_stride, B, wpi, bpi, wv, bv, A, logits, l_stride, value,
                              v_stride, ta, sx, sx + 512, *s_action, reinterpret_cast<uint4*>(lds), n, j, pend);
  __syncthreads();  // the image rows in LDS; the tail's scratch free again
  tower_part_body<C3, H16>(j, nt.b1, nt.b2, nt.b3, nt.a1, nt.a2, nt.a3, nt.st, nt.prep, nt.m1, nt.m2, nt.m3, lds, n);
}
// the split tower alone (small batches without a fused tail: step 0, the bootstrap
// forward): part j loads the input rows 8j .. 8j+35 of image n
template <int C3, bool H16>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void tower_split_kernel(
    const uint8_t* obs, long long img_stride, NextTower nt) {
  __shared__ __attribute__((aligned(16))) char lds[kSpLds];
  const int n = blockIdx.x / kSplitParts, j = blockIdx.x - n * kSplitParts;
  const uint4* src = reinterpret_cast<const uint4*>(obs + n * img_stride);
  uint4* dst = reinterpret_cast<uint4*>(lds);
  const int g0 = split_word_lo(j), g1 = split_word_hi(j);
  constexpr int NW = (36 * 21 + 255) / 256;
  uint4 v[NW];
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const int g = g0 + (int)threadIdx.x + 256 * i;
    v[i] = src[g < g1 ? g : g0];
  }
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const int g = g0 + (int)threadIdx.x + 256 * i;
    if (g < g1) dst[g] = v[i];
  }
  __syncthreads();
  tower_part_body<C3, H16>(j, nt.b1, nt.b2, nt.b3, nt.a1, nt.a2, nt.a3, nt.st, nt.prep, nt.m1, nt.m2, nt.m3, lds, n);
}

inline int roundup4(int x) { return (x + 3) & ~3; }

// policy/value heads, one wave per row: the 512-long dot products of a4 with
// the A+1 head columns, lane-strided partial sums + a butterfly (fixed order).
// With part != nullptr the row of a4 is first finalised from fc4's split-K
// partial slabs [nz][B+1][512] (relu(sum_z + b4), fixed z order) and stored.
template <int NZ>
__global__ __launch_bounds__(256) void heads_kernel(const float* part, int nz, const float* b4,
                                                    float* a4, long long a4_stride, int B,
                                                    const float* wpi, const float* bpi,
                                                    const float* wv, const float* bv, int A,
                                                    float* logits, long long l_stride,
                                                    float* value, long long v_stride) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= B) return;
  float* x = a4 + (long long)row * a4_stride;
  float xv[8];
  if (NZ > 0) {
    // all NZ x 8 slab loads are issued before the (fixed-order) sums
    const long long zs = (long long)(B + 1) * 512;
    float v[NZ > 0 ? NZ : 1][8];
#pragma unroll
    for (int z = 0; z < NZ; ++z)
#pragma unroll
      for (int e = 0; e < 8; ++e) v[z][e] = part[z * zs + (long long)row * 512 + lane + 64 * e];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int j = lane + 64 * e;
      float acc = 0.f;
#pragma unroll
      for (int z = 0; z < NZ; ++z) acc += v[z][e];
      xv[e] = fmaxf(acc + b4[j], 0.f);
      x[j] = xv[e];
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) xv[e] = x[lane + 64 * e];
  }
  for (int a = 0; a < A; ++a) {
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) s += xv[e] * wpi[(lane + 64 * e) * A + a];
    s = wave_sum(s);
    if (lane == 0) logits[(long long)row * l_stride + a] = s + bpi[a];
  }
  if (value) {
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) s += xv[e] * wv[lane + 64 * e];
    s = wave_sum(s);
    if (lane == 0) value[(long long)row * v_stride] = s + bv[0];
  }
}

// (Measured and removed: conv2's input gradient on the dY-im2col-in-LDS kernel
// of convt3.hpp, 939 / 620 us per launch at M = 10240 against 444 on gemm3 -- its
// f32 dY image leaves one block per CU; conv1 / conv2 forwards on convfwd3.hpp,
// 26.5 / 82 us at 512 images against 26.5 / 30.  conv3's input gradient and
// forward keep those kernels: 231 -> 186 us, 19.6 -> 18.7 us.)


// split factor for fc4 at small batch (64 x 128 tiles over 512 columns; 4 / 6 /
// 12 / 16 chunks measured no better than 8)
static void fc4_plan(int B, int K, int* nz, int* chunk) {
  // the split cap at batches <= 128 is 16: the chain of k-steps per chunk, not
  // the slab traffic, sets fc4's time there (14 / 16 measured best)
  const int maxsp = B <= 128 ? 16 : 8;
  const int blocks = cdiv(B, 64) * 4;
  int sp = blocks >= 256 ? 1 : std::min(maxsp, cdiv(256 * maxsp / 8, blocks));
  const int q = g_gemm_mode == ACMI_GEMM_X3 ? 16 : 32;  // the split GEMM's K-tile
  int ch = (cdiv(K, sp) + q - 1) / q * q;
  *chunk = ch;
  *nz = cdiv(K, ch);
}

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
template <int C3>
static int forward_impl(const Layout& L, const float* P, const uint8_t* obs,
                        long long img_stride, int B, const acmi_acts_t* a,
                        int want_value, long long act_img_stride,
                        hipStream_t s, const TailArgs* tail = nullptr, const void* prep = nullptr) {
  // act_img_stride: images between consecutive batch rows in the activation
  // buffers (1 = contiguous; T = rollout step t of an env-major buffer).
  const long long st = act_img_stride;
  // conv1 -> conv2 -> conv3 as one fused kernel per image (tower.hpp, f16x2 on
  // acmi_conv_prepare's fragments) in x3 mode; the per-layer kernels below in f32
  // mode, without prepared weights or for unaligned images
  const bool tower =
      g_gemm_mode == ACMI_GEMM_X3 && prep && (uintptr_t)obs % 16 == 0 && img_stride % 16 == 0;
  ACMI_REQUIRE(tower || g_forward_mode == ACMI_FWD_F32, ACMI_ERR_ARG,
               "16-bit forward needs the fused tower: net->conv_prep and 16-byte aligned observations / image "
               "stride");
  // step fusion (acmi_rollout_io_t): this step's tower ran in the previous
  // step's tail; the next step's tower runs in this step's tail
  const bool tower_done = tail && tail->io.tower_done;
  const acmi_acts_t* nxt = tail ? tail->io.next_acts : nullptr;
  ACMI_REQUIRE(tower || (!tower_done && !nxt), ACMI_ERR_ARG,
               "rollout step fusion needs the fused tower (x3 gemm mode, conv_prep, 16-byte aligned images)");
  ACMI_REQUIRE(!tail || !tail->io.obs_copy || ((uintptr_t)tail->io.obs_copy % 16 == 0 && tail->io.out_stride % 16 == 0),
               ACMI_ERR_ARG, "acmi_rollout_step: obs_copy must be 16-byte aligned");
  ACMI_REQUIRE(!nxt || (nxt->a1 && nxt->a2 && nxt->a3 && masks_ok(nxt) && tail->io.next_act_stride >= 1 &&
                        (uintptr_t)tail->io.obs_out % 16 == 0 && tail->io.out_stride % 16 == 0),
               ACMI_ERR_ARG, "acmi_rollout_step: bad next_acts / next_act_stride / obs_out alignment");
  // small batches: each image's tower over kSplitParts workgroups (towersplit.hpp)
  auto tower_any = [&](const uint8_t* o, long long ostride, float* a1, float* a2, float* a3, long long ast,
                       uint32_t* m1, uint32_t* m2, uint32_t* m3) {
    const bool h16 = g_forward_mode == ACMI_FWD_BF16;
    if (B <= kSplitMaxB) {
      const NextTower nt{P + L.off[1], P + L.off[3], P + L.off[5], a1, a2, a3, ast,
                         static_cast<const char*>(prep), m1, m2, m3};
      if (h16)
        hipLaunchKernelGGL((tower_split_kernel<C3, true>), dim3(B * kSplitParts), dim3(256), 0, s, o, ostride, nt);
      else
        hipLaunchKernelGGL((tower_split_kernel<C3, false>), dim3(B * kSplitParts), dim3(256), 0, s, o, ostride, nt);
    } else {
      launch_tower<C3>(o, ostride, B, P, L.off, a1, a2, a3, ast, prep, s, h16, m1, m2, m3);
    }
  };
  if (tower) {
    // the three convs fused per image (16-byte image loads)
    if (!tower_done) {
      prof_begin(ACMI_PROF_CONV1_FWD, s);
      tower_any(obs, img_stride, a->a1, a->a2, a->a3, st, a->m1, a->m2, a->m3);
      prof_end(ACMI_PROF_CONV1_FWD, s);
    }
  } else {
  {  // conv1: [B,84,84,4]u8 -> [B,20,20,32]; the u8 patches stay bytes in LDS
    using Src = ConvRows<uint8_t, 84, 84, 4, 8, 8, 4>;
    MatI<true> w{P + L.off[0], 32, 256, 32};
    EpiAct epi{a->a1, P + L.off[1], 32, 400, st * 400 * 32, 1.0f / 255.0f};
    prof_begin(ACMI_PROF_CONV1_FWD, s);
    launch_conv1_fwd_u8<32>(Src{obs, (uint32_t)img_stride, B * 400}, w, epi, B * 400, 256, s);
    prof_end(ACMI_PROF_CONV1_FWD, s);
  }
  {  // conv2: -> [B,9,9,64]
    using Src = ConvRows<float, 20, 20, 32, 4, 4, 2>;
    RowsAsK<Src> opA{Src{a->a1, (uint32_t)(st * 400 * 32), B * 81}};
    MatI<true> opB{P + L.off[2], 64, 512, 64};
    EpiAct epi{a->a2, P + L.off[3], 64, 81, st * 81 * 64};
    if (B <= 2048)
      launch_mm<64, 64, 32, 1, 1, false, false, 32>(opA, opB, epi, B * 81, 64, 512, 1, 0, s);
    else
      launch_mm<128, 64, 32, 2, 1, false, false, 16>(opA, opB, epi, B * 81, 64, 512, 1, 0, s);
  }
  {  // conv3: -> [B,7,7,C3]
    using Src = ConvRows<float, 9, 9, 64, 3, 3, 1>;
    RowsAsK<Src> opA{Src{a->a2, (uint32_t)(st * 81 * 64), B * 49}};
    MatI<true> opB{P + L.off[4], C3, 576, C3};
    EpiAct epi{a->a3, P + L.off[5], C3, 49, st * 49 * C3};
    if (g_gemm_mode == ACMI_GEMM_X3)
      launch_convf_x3<float, 9, 9, 64, 3, 3, 1, C3, 2, 64>(a->a2, st * 81 * 64, B, P + L.off[4], epi, s);
    else if constexpr (C3 == 32)
      // (f32 MFMA: the 128x32 bf16x3 tile needs BK = 32 and fits 2 blocks per CU;
      // measured slower than this at B = 512, 21.1 vs 19.6 us)
      launch_gemm<128, 32, 32, 1, 1, false, false>(opA, opB, epi, B * 49, C3, 576, 1, 0, s);
    else
      launch_mm<128, 64, 32, 2, 1, false, false, 16>(opA, opB, epi, B * 49, C3, 576, 1, 0, s);
  }
  if (a->m1) {  // the ReLU' masks the tower would have written
    hipLaunchKernelGGL(act_mask_kernel, dim3(cdiv((long long)B * 400, 256)), dim3(256), 0, s, a->a1, B, 400, st, a->m1);
    hipLaunchKernelGGL(act_mask_kernel, dim3(cdiv((long long)B * 162, 256)), dim3(256), 0, s, a->a2, B, 162, st, a->m2);
    hipLaunchKernelGGL(act_mask_kernel, dim3(cdiv((long long)B * 49 * C3 / 32, 256)), dim3(256), 0, s, a->a3, B,
                       49 * C3 / 32, st, a->m3);
  }
  }  // per-layer convs
  // fc4: [B,49*C3] -> [B,512]
  const int K4 = 49 * C3;
  // rows are images; with an image stride the dense row stride is st*K4
  RowsAsK<DenseRows> opA4{DenseRows{a->a3, (int)(st * K4), B, K4}};
  MatI<true> opB4{P + L.off[6], 512, K4, 512};
  int nz, chunk;
  fc4_plan(B, K4, &nz, &chunk);
  const bool split = nz > 1 && a->ws && a->ws_floats >= (long long)nz * (B + 1) * 512;
  const char* w4p = prep ? static_cast<const char*>(prep) + TowerPrep<C3>::BYTES + CT2::BYTES : nullptr;
  // the split rollout step's pending env states, after fc4's slabs in the forward
  // workspace (acmi_forward_ws_floats reserves them at B <= kSplitMaxB); only with
  // the rollout fc4 kernel, the one launch that commits them
  const bool fc4_roll = split && g_gemm_mode == ACMI_GEMM_X3 && w4p && fc4_roll_ok(a->a3, st * K4, K4, chunk);
  PendState* pend = fc4_roll && tail && B <= kSplitMaxB &&
                            a->ws_floats >= (long long)nz * (B + 1) * 512 + (long long)B * (sizeof(PendState) / 4)
                        ? reinterpret_cast<PendState*>(a->ws + (long long)nz * (B + 1) * 512)
                        : nullptr;
  if (split) {
    // small (rollout) batches: split K over chunks; the heads kernel reduces
    // the slabs in fixed order and applies bias + relu
    // every rollout step with a pending area commits the entries flagged there
    // (the previous fused step's; also, at step 0, those a rollout abandoned
    // between fused steps left behind -- the flag is cleared on commit)
    const Fc4Commit cm{pend, tail ? tail->io.state : acmi_env_state_t{}, pend ? B : 0};
    if (!(fc4_roll &&
          launch_fc4_roll(a->a3, st * K4, B, K4, w4p, nz, chunk, a->ws,
                          reinterpret_cast<const unsigned*>(static_cast<const char*>(prep) + TowerPrep<C3>::HDR),
                          s, cm))) {
      // (no fused tower without the rollout fc4: no split step, nothing pending)
      EpiPartial epi{a->ws, B, 512};
      launch_mm<64, 128, 32, 1, 2, true, false, 16>(opA4, opB4, epi, B, 512, K4, nz, chunk, s);
    }
  } else {
    EpiAct epi{a->a4, P + L.off[7], 512, 1, st * 512};
    launch_mm<64, 128, 32, 1, 2, false, false, 16>(opA4, opB4, epi, B, 512, K4, 1, 0, s);
  }
  // heads: [B,512] -> logits [B,A], value [B]
  const dim3 hg(cdiv(B, 4)), hb(256);
  const float* hp = split ? a->ws : nullptr;
  float* hv = want_value ? a->value : nullptr;
  NextTower ntw{};
  if (nxt) ntw = NextTower{P + L.off[1], P + L.off[3], P + L.off[5], nxt->a1, nxt->a2, nxt->a3,
                          tail->io.next_act_stride, static_cast<const char*>(prep), nxt->m1, nxt->m2, nxt->m3};
  const bool h16 = g_forward_mode == ACMI_FWD_BF16;
  // the fused tail + next tower at the rollout's split-K count; any other (or
  // no) split runs the tail and then the next step's tower as two launches
  // (small batches run the 16-wave tower, which the fused tail does not host)
  // (fused at the split counts the plan produces: 8 at the rollout batch; 14 / 16
  // below 128 images -- K = 1568 / 3136 in chunks of 7 / 13 k16-steps)
  const bool fuse_next = nxt && split && (nz == 8 || nz == 14 || nz == 16);
#define ACMI_HEADS(NZ)                                                                          \
  if (tail && fuse_next && pend && (NZ == 14 || NZ == 16)) {                                    \
    if (h16)                                                                                    \
      hipLaunchKernelGGL((rollout_tail_split_kernel<NZ == 16 ? 16 : 14, C3, true>), dim3(B * kSplitParts), hb, 0, s, \
                         hp, nz, P + L.off[7], a->a4, st * 512, B, P + L.off[8], P + L.off[9],  \
                         P + L.off[10], P + L.off[11], L.A, a->logits, st * a->ld_logits, hv, st, \
                         *tail, ntw, pend);                                                     \
    else                                                                                        \
      hipLaunchKernelGGL((rollout_tail_split_kernel<NZ == 16 ? 16 : 14, C3, false>), dim3(B * kSplitParts), hb, 0, s, \
                         hp, nz, P + L.off[7], a->a4, st * 512, B, P + L.off[8], P + L.off[9],  \
                         P + L.off[10], P + L.off[11], L.A, a->logits, st * a->ld_logits, hv, st, \
                         *tail, ntw, pend);                                                     \
  } else if (tail && fuse_next && (NZ == 8 || NZ == 14 || NZ == 16)) {                          \
    if (h16)                                                                                    \
      hipLaunchKernelGGL((rollout_tail_tower_kernel<NZ == 16 ? 16 : NZ == 14 ? 14 : 8, C3, true>), dim3(B), hb, 0, s, hp, nz, \
                         P + L.off[7], a->a4, st * 512, B, P + L.off[8], P + L.off[9],          \
                         P + L.off[10], P + L.off[11], L.A, a->logits, st * a->ld_logits, hv, st, \
                         *tail, ntw);                                                           \
    else                                                                                        \
      hipLaunchKernelGGL((rollout_tail_tower_kernel<NZ == 16 ? 16 : NZ == 14 ? 14 : 8, C3, false>), dim3(B), hb, 0, s, hp, nz, \
                         P + L.off[7], a->a4, st * 512, B, P + L.off[8], P + L.off[9],          \
                         P + L.off[10], P + L.off[11], L.A, a->logits, st * a->ld_logits, hv, st, \
                         *tail, ntw);                                                           \
  } else if (tail)                                                                              \
    hipLaunchKernelGGL(rollout_tail_kernel<NZ>, dim3(B), hb, 0, s, hp, nz, P + L.off[7], a->a4,  \
                       st * 512, B, P + L.off[8], P + L.off[9], P + L.off[10], P + L.off[11],    \
                       L.A, a->logits, st * a->ld_logits, hv, st, *tail);                        \
  else                                                                                          \
    hipLaunchKernelGGL(heads_kernel<NZ>, hg, hb, 0, s, hp, nz, P + L.off[7], a->a4, st * 512, B, \
                       P + L.off[8], P + L.off[9], P + L.off[10], P + L.off[11], L.A, a->logits, \
                       st * a->ld_logits, hv, st)
  switch (split ? nz : 0) {
    case 0: ACMI_HEADS(0); break;
    case 2: ACMI_HEADS(2); break;
    case 3: ACMI_HEADS(3); break;
    case 4: ACMI_HEADS(4); break;
    case 5: ACMI_HEADS(5); break;
    case 6: ACMI_HEADS(6); break;
    case 7: ACMI_HEADS(7); break;
    case 8: ACMI_HEADS(8); break;
    case 9: ACMI_HEADS(9); break;
    case 10: ACMI_HEADS(10); break;
    case 11: ACMI_HEADS(11); break;
    case 12: ACMI_HEADS(12); break;
    case 13: ACMI_HEADS(13); break;
    case 14: ACMI_HEADS(14); break;
    case 15: ACMI_HEADS(15); break;
    case 16: ACMI_HEADS(16); break;
    default: ACMI_REQUIRE(false, ACMI_ERR_ARG, "fc4 split factor %d out of range", nz);
  }
#undef ACMI_HEADS
  if (nxt && !fuse_next)  // the next step's tower on the stacks the tail just wrote
    tower_any(tail->io.obs_out, tail->io.out_stride, nxt->a1, nxt->a2, nxt->a3, tail->io.next_act_stride, nxt->m1,
              nxt->m2, nxt->m3);
  ACMI_LAUNCH_CHECK("acmi_forward");
  return ACMI_OK;
}

// ---------------------------------------------------------------------------
// split-K weight-gradient / factor reduction
// ---------------------------------------------------------------------------
// part: [nchunk][I+1][J] with J = kp + cout_pad + (kp ? 1 : 0).
// grad (layer [W;b], (K+1) x cout, optionally split into two column groups
// for the fused heads) and astat ((K+1)^2, symmetric, / rows).
struct WgradDesc {
  const float* part;
  int nchunk;
  int I;  // = K
  int J;
  int kp;       // 0 or K
  int cout;
  float* gradA;  // columns [0, nsplit)
  int nsplit;
  float* gradB;  // columns [nsplit, cout)
  float* astat;  // nullable
  int rows;
  float wscale;  // applied to the weight rows (a < K) of the gradient
};

// One block = 32 consecutive outputs x 8 chunk groups: group g sums chunks
// g, g+8, ... in order (4 loads in flight), then the 8 group sums are added in
// group order -- a fixed order (deterministic) with 8x the loads in flight of one
// thread per output.  Outputs: the gradient rows (K+1) x cout, then the upper
// triangle of the A factor (written to both halves).
constexpr int kFinGroups = 8;
__device__ __forceinline__ float chunk_sum_group(const float* p, int n, long long cs, int g) {
  float s = 0.f;
  for (int c0 = g; c0 < n; c0 += 4 * kFinGroups) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = c0 + u * kFinGroups;
      v[u] = p[(long long)(c < n ? c : g) * cs];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) s += (c0 + u * kFinGroups < n) ? v[u] : 0.f;
  }
  return s;
}

__device__ __forceinline__ void finalize_wgrad_body(const WgradDesc& d, int bx, float (*red)[32]) {
  const int K = d.I;
  const long long ngrad = (long long)(K + 1) * d.cout;
  const long long nstat = d.astat ? (long long)(K + 1) * (K + 1) : 0;
  const int el = threadIdx.x & 31, g = threadIdx.x >> 5;
  const long long idx = (long long)bx * 32 + el;
  const long long cs = (long long)(d.I + 1) * d.J;  // chunk stride
  // the partial this output sums (nullptr: nothing to sum)
  const float* p = nullptr;
  int a = 0, b = 0, n = 0;
  if (idx < ngrad) {
    a = (int)(idx / d.cout);
    n = (int)(idx - (long long)a * d.cout);
    const int row = a < K ? a : d.I;
    p = d.part + (long long)row * d.J + d.kp + n;
  } else if (idx < ngrad + nstat) {
    const long long e = idx - ngrad;
    a = (int)(e / (K + 1));
    b = (int)(e - (long long)a * (K + 1));
    // column K (the homogeneous coordinate) = sum of P = column-sum row
    if (a <= b && a != K) p = b < K ? d.part + (long long)a * d.J + b : d.part + (long long)d.I * d.J + a;
  }
  red[g][el] = p ? chunk_sum_group(p, d.nchunk, cs, g) : 0.f;
  __syncthreads();
  if (g != 0 || idx >= ngrad + nstat) return;
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < kFinGroups; ++q) s += red[q][el];
  if (idx < ngrad) {
    if (a < K) s *= d.wscale;
    if (n < d.nsplit) d.gradA[(long long)a * d.nsplit + n] = s;
    else d.gradB[(long long)a * (d.cout - d.nsplit) + (n - d.nsplit)] = s;
  } else {
    if (a > b) return;
    if (a == K) s = (float)d.rows;
    s *= 1.0f / (float)d.rows;
    d.astat[(long long)a * (K + 1) + b] = s;
    d.astat[(long long)b * (K + 1) + a] = s;
  }
}

// Gradient outputs (d.astat == nullptr) of a partial with few chunks (<= 8): one
// thread per output instead of 32 outputs x 8 chunk groups per block (7 of the 8
// groups idle at one chunk: the fc4 gradient's 803 K outputs were 25 K blocks).
// The same sums in the same order: group g holds chunk g alone (0 + p[g]), the
// groups added in order from 0.
__device__ __forceinline__ void finalize_grad_thread_body(const WgradDesc& d, int bx) {
  const int K = d.I;
  const long long idx = (long long)bx * 256 + threadIdx.x;
  if (idx >= (long long)(K + 1) * d.cout) return;
  const int a = (int)(idx / d.cout), n = (int)(idx - (long long)a * d.cout);
  const float* p = d.part + (long long)(a < K ? a : d.I) * d.J + d.kp + n;
  const long long cs = (long long)(d.I + 1) * d.J;
  float v[kFinGroups];
#pragma unroll
  for (int g = 0; g < kFinGroups; ++g) v[g] = p[(long long)(g < d.nchunk ? g : 0) * cs];
  float s = 0.f;
#pragma unroll
  for (int g = 0; g < kFinGroups; ++g) s += g < d.nchunk ? 0.f + v[g] : 0.f;
  if (a < K) s *= d.wscale;
  if (n < d.nsplit) d.gradA[(long long)a * d.nsplit + n] = s;
  else d.gradB[(long long)a * (d.cout - d.nsplit) + (n - d.nsplit)] = s;
}
__device__ __forceinline__ bool fin_thread_ok(const WgradDesc& d) { return !d.astat && d.nchunk <= kFinGroups; }
inline int fin_blocks(const WgradDesc& d) {
  const long long total = (long long)(d.I + 1) * d.cout + (d.astat ? (long long)(d.I + 1) * (d.I + 1) : 0);
  return (int)(!d.astat && d.nchunk <= kFinGroups ? cdiv(total, 256) : cdiv(total, 32));
}

__global__ __launch_bounds__(256) void finalize_wgrad_kernel(WgradDesc d) {
  __shared__ float red[kFinGroups][32];
  if (fin_thread_ok(d)) finalize_grad_thread_body(d, blockIdx.x);
  else finalize_wgrad_body(d, blockIdx.x, red);
}

// The A factor of a split-K wgrad partial ((K+1)^2, symmetric): one block per
// 32x32 tile of the upper triangle; each element sums its chunks in exactly
// finalize_wgrad_kernel's order (chunk group g = c mod 8 in chunk order, then
// the groups in order), is stored at (a, b) and, through an LDS transpose, at
// (b, a) -- both halves written by coalesced rows (the element-per-thread
// mirror store of finalize_wgrad_kernel is a 4-byte scatter with stride K+1).
__device__ __forceinline__ void finalize_afactor_body(const WgradDesc& d, int ntile, int bx, float (*tr)[33]) {
  const int K = d.I, K1 = K + 1;
  // upper-triangle tile (ta <= tb) of linear index bx
  int t = bx, ta = 0;
  while (t >= ntile - ta) t -= ntile - ta, ++ta;
  const int tb = ta + t;
  const long long cs = (long long)(d.I + 1) * d.J;
  const int c = threadIdx.x & 31, r0 = threadIdx.x >> 5;
  const float inv = 1.0f / (float)d.rows;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int r = r0 + 8 * it;
    const int a = 32 * ta + r, b = 32 * tb + c;
    float v = 0.f;
    if (a < K1 && b < K1 && a <= b) {
      if (a == K) {
        v = (float)d.rows * inv;  // rows * fl(1/rows), as finalize_wgrad_kernel (1 - 2^-24 for some rows)
      } else {
        const float* p = b < K ? d.part + (long long)a * d.J + b : d.part + (long long)d.I * d.J + a;
        float s = 0.f;
        for (int g = 0; g < kFinGroups; ++g) {
          float sg = 0.f;
          for (int ch = g; ch < d.nchunk; ch += kFinGroups) sg += p[(long long)ch * cs];
          s += sg;
        }
        v = s * inv;
      }
      d.astat[(long long)a * K1 + b] = v;
    }
    tr[r][c] = v;
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 4; ++it) {  // (b, a) for a < b: row b of the output reads column b of the tile
    const int r = r0 + 8 * it;     // row offset inside tile tb
    const int b = 32 * tb + r, a = 32 * ta + c;
    if (a < K1 && b < K1 && a < b) d.astat[(long long)b * K1 + a] = tr[c][r];
  }
}
__global__ __launch_bounds__(256) void finalize_afactor_kernel(WgradDesc d, int ntile) {
  __shared__ float tr[32][33];
  finalize_afactor_body(d, ntile, blockIdx.x, tr);
}

// Several layers' weight-gradient / A-factor finalizes as one launch (each
// layer's split-K partials in their own workspace range): task k owns blocks
// [blk0, blk0 of k+1) and runs finalize_wgrad_kernel's (kind 0) or
// finalize_afactor_kernel's (kind 1) body -- the same sums.
struct WgradTask {
  WgradDesc d;
  int kind, ntile, blk0;
};
constexpr int kWgradTasks = 6;
struct WgradSet {
  int n = 0;
  int blocks = 0;
  WgradTask t[kWgradTasks];
  void add(const WgradDesc& d, int kind, int ntile, int nblocks) {
    t[n++] = WgradTask{d, kind, ntile, blocks};
    blocks += nblocks;
  }
};
__global__ __launch_bounds__(256) void finalize_wgrad_multi_kernel(WgradSet S) {
  __shared__ float red[kFinGroups][32];
  __shared__ float tr[32][33];
  int k = 0;
  while (k + 1 < S.n && (int)blockIdx.x >= S.t[k + 1].blk0) ++k;
  const WgradTask& T = S.t[k];
  const int b = blockIdx.x - T.blk0;
  if (T.kind == 0) {
    if (fin_thread_ok(T.d)) finalize_grad_thread_body(T.d, b);
    else finalize_wgrad_body(T.d, b, red);
  } else {
    finalize_afactor_body(T.d, T.ntile, b, tr);
  }
}

// G factor: part [nchunk][I+1][J] (I == J == n, no colsum row used); one
// wave per output element sums the chunks in a fixed (lane-strided, then
// butterfly) order, so the result is deterministic.
// thread per upper-triangle element (few chunks): consecutive threads read
// consecutive partials, the value is written to both halves
__global__ void finalize_cov_thread_kernel(const float* part, int nchunk, int n, int sub,
                                           float* out, int rows) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= sub * sub) return;
  const int a = idx / sub, b = idx - a * sub;
  if (a > b) return;
  const long long cs = (long long)(n + 1) * n;
  const float v = chunk_sum(part + (long long)a * n + b, nchunk, cs) * (1.0f / (float)rows);
  out[a * sub + b] = v;
  out[b * sub + a] = v;
}

// wave per element (many chunks: the lanes split the chunks)
__global__ void finalize_cov_kernel(const float* part, int nchunk, int n,
                                    int sub, float* out, int rows) {
  // out is sub x sub, taken from the top-left of the n x n product
  const int idx = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (idx >= sub * sub) return;
  const int a = idx / sub, b = idx - a * sub;
  const int lo = a < b ? a : b, hi = a < b ? b : a;
  const long long cs = (long long)(n + 1) * n;
  const float* p = part + (long long)lo * n + hi;
  float s = 0.f;
  for (int c = lane; c < nchunk; c += 64) s += p[c * cs];
  s = wave_sum(s);
  if (lane == 0) out[idx] = s * (1.0f / (float)rows);
}

// G of the value head: element (A, A) of the heads product
__global__ void finalize_cov_elem_kernel(const float* part, int nchunk, int n,
                                         int a, float* out, int rows) {
  // one wave: lane-strided partial sums + a butterfly (fixed order)
  const int lane = threadIdx.x & 63;
  if (threadIdx.x >= 64 || blockIdx.x != 0) return;
  const long long cs = (long long)(n + 1) * n;
  const float* p = part + (long long)a * n + a;
  float s = 0.f;
  for (int c = lane; c < nchunk; c += 64) s += p[c * cs];
  s = wave_sum(s);
  if (lane == 0) out[0] = s * (1.0f / (float)rows);
}

// The sampled-loss chain's G-factor finalizes as ONE launch after all its Grams
// (each Gram's partials in its own workspace range): task k owns blocks
// [blk0, blk0 of k+1) and runs the body of finalize_cov_thread_kernel (kind 0),
// finalize_cov_kernel (1) or finalize_cov_elem_kernel (2) -- the same sums.
struct CovTask {
  const float* part;
  float* out;
  int nchunk, n, sub, rows, kind, a, blk0;
};
constexpr int kCovTasks = 8;
struct CovSet {
  int n = 0;
  int blocks = 0;
  CovTask t[kCovTasks];
  void add(const float* part, int nchunk, int n_, int sub, float* out, int rows, int kind, int a = 0) {
    const int nt = cdiv(sub, 32);
    const int nb = kind == 0 ? cdiv(sub * sub, 256) : kind == 1 ? cdiv(sub * sub, 4) : kind == 3 ? nt * (nt + 1) / 2 : 1;
    t[n++] = CovTask{part, out, nchunk, n_, sub, rows, kind, a, blocks};
    blocks += nb;
  }
};
__global__ __launch_bounds__(256) void finalize_cov_multi_kernel(CovSet S) {
  int k = 0;
  while (k + 1 < S.n && (int)blockIdx.x >= S.t[k + 1].blk0) ++k;
  const CovTask& T = S.t[k];
  const int b = blockIdx.x - T.blk0;
  const long long cs = (long long)(T.n + 1) * T.n;
  if (T.kind == 3) {
    // kind 0's sums on 32 x 32 upper-triangle tiles, both halves written by
    // coalesced rows through an LDS transpose (kind 0's mirror store is a 4-byte
    // scatter with stride sub: the 512-wide G factor's half)
    __shared__ float tr[32][33];
    const int ntile = (T.sub + 31) / 32;
    int t = b, ta = 0;
    while (t >= ntile - ta) t -= ntile - ta, ++ta;
    const int tb = ta + t;
    const int c = threadIdx.x & 31, r0 = threadIdx.x >> 5;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int r = r0 + 8 * it;
      const int a = 32 * ta + r, cc = 32 * tb + c;
      float v = 0.f;
      if (a < T.sub && cc < T.sub && a <= cc) {
        v = chunk_sum(T.part + (long long)a * T.n + cc, T.nchunk, cs) * (1.0f / (float)T.rows);
        T.out[a * T.sub + cc] = v;
      }
      tr[r][c] = v;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int r = r0 + 8 * it;
      const int bb = 32 * tb + r, a = 32 * ta + c;
      if (a < T.sub && bb < T.sub && a < bb) T.out[bb * T.sub + a] = tr[c][r];
    }
    return;
  }
  if (T.kind == 0) {
    const int idx = b * 256 + threadIdx.x;
    if (idx >= T.sub * T.sub) return;
    const int a = idx / T.sub, c = idx - a * T.sub;
    if (a > c) return;
    const float v = chunk_sum(T.part + (long long)a * T.n + c, T.nchunk, cs) * (1.0f / (float)T.rows);
    T.out[a * T.sub + c] = v;
    T.out[c * T.sub + a] = v;
  } else {
    const int idx = T.kind == 1 ? b * 4 + (threadIdx.x >> 6) : 0;
    const int lane = threadIdx.x & 63;
    if (idx >= T.sub * T.sub || (T.kind == 2 && threadIdx.x >= 64)) return;
    int lo, hi;
    if (T.kind == 1) {
      const int a = idx / T.sub, c = idx - a * T.sub;
      lo = a < c ? a : c, hi = a < c ? c : a;
    } else {
      lo = hi = T.a;
    }
    const float* p = T.part + (long long)lo * T.n + hi;
    float v = 0.f;
    for (int c = lane; c < T.nchunk; c += 64) v += p[c * cs];
    v = wave_sum(v);
    if (lane == 0) T.out[idx] = v * (1.0f / (float)T.rows);
  }
}

// G = D^T D for narrow D (n <= NP, NP in {32, 64}) straight from global memory:
// each wave streams row pairs (lane l: row 2q + (l>>5), column l&31 [+32]) as
// the A and B fragments of v_mfma_f32_32x32x2_f32 (the Gram tile is D^T D of
// the same registers).  Two register sets of UNR k-steps: the next group's
// loads are issued before this group's MFMAs.  The block's 4 waves are summed
// into one LDS image in wave order (deterministic) and stored as
// part[chunk][NP+1][NP] (finalize_cov_*).
template <int NP>
__global__ __launch_bounds__(256) void gram_small_kernel(const float* D, int ld, int n,
                                                        long long rows, long long chunk,
                                                        float* part) {
  constexpr int T = NP / 32;           // column tiles
  constexpr int NT = T * (T + 1) / 2;  // upper-triangle tile pairs
  constexpr int UNR = 8;
  __shared__ float red[NP * NP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, c = lane & 31;
  const long long r0 = (long long)blockIdx.x * chunk;
  const long long r1 = min(rows, r0 + chunk);
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  const float* zero = zero_run();
  auto load = [&](long long base, float (&v)[UNR][T]) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const long long row = base + 8 * u + h;
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const int col = c + 32 * t;
        const bool ok = row < r1 && col < n;
        v[u][t] = *(ok ? D + row * ld + col : zero);
      }
    }
  };
  auto mma = [&](const float (&v)[UNR][T]) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      int t = 0;
#pragma unroll
      for (int x = 0; x < T; ++x)
#pragma unroll
        for (int y = x; y < T; ++y, ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(v[u][x], v[u][y], acc[t], 0, 0, 0);
    }
  };
  float va[UNR][T], vb[UNR][T];
  long long base = r0 + 2 * wave;
  load(base, va);
  for (; base < r1; base += 16 * UNR) {
    load(base + 8 * UNR, vb);
    mma(va);
    if (base + 8 * UNR >= r1) break;
    load(base + 16 * UNR, va);
    mma(vb);
  }
  // acc[t][r]: tile (x, y), row 32x + (r&3) + 8(r>>2) + 4h, column 32y + c
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
      int t = 0;
#pragma unroll
      for (int x = 0; x < T; ++x)
#pragma unroll
        for (int y = x; y < T; ++y, ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int i = 32 * x + (r & 3) + 8 * (r >> 2) + 4 * h, j = 32 * y + c;
            const float prev_ij = w ? red[i * NP + j] : 0.f;
            red[i * NP + j] = prev_ij + acc[t][r];
            if (x != y) {
              const float prev_ji = w ? red[j * NP + i] : 0.f;
              red[j * NP + i] = prev_ji + acc[t][r];
            }
          }
    }
    __syncthreads();
  }
  float* out = part + (long long)blockIdx.x * (NP + 1) * NP;
  for (int e = threadIdx.x; e < NP * NP; e += 256) out[e] = red[e];
}

// split-K reductions fill whole rounds of resident blocks (plan_rounds):
// MI355X has 256 CUs; blocks per CU follow from each config's LDS image
constexpr int kCUs = 256;

static bool band_on(bool with_stats) {
  return with_stats && g_gemm_mode == ACMI_GEMM_X3 && g_conv_stats_mode == ACMI_CONV_STATS_BAND;
}

struct WgradPlan {
  int I, J, kp, cout_pad, nc, ch;
  bool slabs;  // symred_kernel (slab groups) instead of 128x128 live tiles
  bool six;    // bf16x3 six-slab groups (symred6_kernel)
  bool six_greedy = false;  // ... with the greedy plan for any K (fc4)
  SymPlan sp;
  SymPlan6 sp6;
  long long floats;
};

static WgradPlan wgrad_plan(int K, int cout, bool with_stats, long long rows, bool u8 = false,
                            int mode = g_gemm_mode) {
  WgradPlan p;
  p.cout_pad = roundup4(cout);
  p.kp = with_stats ? K : 0;
  p.I = K;
  // no homogeneous column: the A factor's last column (sum of P) is the
  // column-sum row's P part, by symmetry
  p.J = p.kp + p.cout_pad;
  p.slabs = with_stats && sym_plan(K, p.cout_pad, &p.sp);  // (f32 patch sources only)
  p.six = p.slabs && mode == ACMI_GEMM_X3 && sym_plan6(K, p.cout_pad, &p.sp6);
  // fc4 (K = 1568, no four-slab plan): greedy six-slab groups instead of 128x128 tiles
  p.six_greedy = !p.slabs && !u8 && with_stats && mode == ACMI_GEMM_X3 && K % 4 == 0 &&
                 sym_plan6_greedy(K, p.cout_pad, &p.sp6);
  if (p.six_greedy) p.six = true;
  if (u8)  // conv1 weight gradient: conv1_wgrad_u8/x3_kernel, one 256x32 block per chunk
    conv1_wgrad_u8_plan(rows, &p.nc, &p.ch, mode);
  else if (p.six_greedy)  // many groups: one round of blocks, few chunks (partials stay small)
    plan_rounds(rows, p.sp6.ngroups, kCUs, &p.nc, &p.ch, 2048);
  else if (p.six)  // one 512-thread block per CU (2 x 64 accumulators per wave)
    plan_rounds(rows, p.sp6.ngroups, kCUs, &p.nc, &p.ch);
  else if (p.slabs && mode == ACMI_GEMM_X3)
    plan_rounds(rows, p.sp.ngroups, kCUs * std::min(8, 160 * 1024 / symred3_lds_bytes()), &p.nc,
                &p.ch);
  else if (p.slabs)
    plan_rounds(rows, p.sp.ngroups, kCUs * std::min(8, 160 * 1024 / symred_lds_bytes<16>()), &p.nc,
                &p.ch);
  else if (with_stats)
    plan_rounds(rows, live_tiles<128, 128>(p.I, p.J, K),
                kCUs * gemm_blocks_per_cu<128, 128, 16, false, false>(), &p.nc, &p.ch);
  else
    plan_rounds(rows, live_tiles<128, 32>(p.I, p.J, 0),
                kCUs * gemm_blocks_per_cu<128, 32, 32, false, false>(), &p.nc, &p.ch);
  p.floats = (long long)p.nc * (p.I + 1) * p.J;
  return p;
}

struct GcovPlan {
  int np, nc, ch;
  long long floats;
};

// narrow Gram: chunks of >= 512 rows, at most 2048 blocks (8 per CU)
static void gram_plan(long long rows, int* nc, long long* chunk) {
  long long n = std::min<long long>(2048, std::max<long long>(1, rows / 512));
  long long ch = (rows + n - 1) / n;
  ch = (ch + 63) / 64 * 64;
  *chunk = ch;
  *nc = (int)((rows + ch - 1) / ch);
}

static GcovPlan gcov_plan(int n, long long rows) {
  GcovPlan p;
  p.np = roundup4(n);
  plan_rounds(rows, live_tiles<64, 64>(p.np, p.np, p.np),
              kCUs * gemm_blocks_per_cu<64, 64, 32, false, false>(), &p.nc, &p.ch);
  p.floats = (long long)p.nc * (p.np + 1) * p.np;
  return p;
}

// the partial floats gcov_layer will need (its two paths' plans)
static long long gcov_need(int n, long long rows) {
  if (n <= 32) {
    int nc;
    long long ch;
    gram_plan(rows, &nc, &ch);
    return (long long)nc * 33 * 32;
  }
  return gcov_plan(n, rows).floats;
}

// Launch [P;1]^T [P | dY] (with_stats; the 1 row is the column-sum row) or
// [P;1]^T [dY] over rows.
template <class Src>
static int wgrad_layer(const Src& src, int K, long long rows, const float* dy,
                       int ldy, int cout, bool with_stats, float* part,
                       long long part_cap, float* gradA, int nsplit,
                       float* gradB, float* astat, hipStream_t s, int site = 0,
                       float wscale = 1.f, const unsigned* pmax = nullptr, const unsigned* ymax = nullptr,
                       WgradSet* defer = nullptr, long long* used = nullptr) {
  constexpr bool kU8 = !std::is_same<typename Src::elem_t, float>::value;
  const int mode = g_gemm_mode;
  const WgradPlan pl = wgrad_plan(K, cout, with_stats, rows, kU8, mode);
  const int I = pl.I, J = pl.J, kp = pl.kp, nc = pl.nc, ch = pl.ch;
  RowsAsI<Src> opA{src};
  CatRowsI<Src> opB{src, kp, dy, ldy, cout, pl.cout_pad, (int)rows};
  if constexpr (!std::is_same<typename Src::elem_t, float>::value)
    ACMI_REQUIRE(!with_stats, ACMI_ERR_ARG, "u8 patch sources take the integer A-factor path");
  ACMI_REQUIRE(pl.floats <= part_cap, ACMI_ERR_WS, "wgrad workspace too small (%lld > %lld)",
               pl.floats, part_cap);
  EpiPartial epi{part, I, J};
  prof_begin(site, s);
  if constexpr (std::is_same<typename Src::elem_t, float>::value) {
    if (pl.six)  // six-slab groups, bf16x3 split operands (f16x2 with published bounds)
      launch_symred6(opB, epi, pl.sp6, I, J, (int)rows, nc, ch, s, pmax, ymax, kp);
    else if (pl.slabs && mode == ACMI_GEMM_X3)  // slab groups, bf16x3 split operands
      launch_symred3(opB, epi, pl.sp, I, J, (int)rows, nc, ch, s);
    else if (pl.slabs)  // slab groups over the upper triangle of P^T P and the dY columns
      launch_symred<16>(opB, epi, pl.sp, I, J, (int)rows, nc, ch, s);
    else if (with_stats)  // 128x128 live tiles (fc4: K not a multiple of 64)
      launch_mm<128, 128, 16, 2, 2, true, true, 16>(opA, opB, epi, I, J, (int)rows, nc, ch, s, K);
    else
      launch_mm<128, 32, 32, 1, 1, true, true, 32>(opA, opB, epi, I, J, (int)rows, nc, ch, s);
  } else {  // u8 patches (conv1): weight gradient only, bytes in LDS
    ACMI_REQUIRE(K == 256 && cout == 32 && ldy == 32, ACMI_ERR_ARG, "conv1 weight gradient shape");
    launch_conv1_wgrad_u8(src, dy, (int)rows, nc, ch, epi, s);
  }
  prof_end(site, s);
  // few chunks (fc4): the A factor on upper-triangle tiles mirrored through LDS;
  // many (the heads' 80): one output per 8 threads, chunk groups in parallel
  const bool tiles = astat && nc <= kFinGroups;
  WgradDesc d{part, nc, I, J, kp, cout, gradA, nsplit, gradB, tiles ? nullptr : astat, (int)rows, wscale};
  if (used) *used = pl.floats;
  if (defer) {
    defer->add(d, 0, 0, fin_blocks(d));
    if (tiles) {
      d.astat = astat;
      const int nt = cdiv(K + 1, 32);
      defer->add(d, 1, nt, nt * (nt + 1) / 2);
    }
    ACMI_LAUNCH_CHECK("wgrad_layer");
    return ACMI_OK;
  }
  hipLaunchKernelGGL(finalize_wgrad_kernel, dim3(fin_blocks(d)), dim3(256), 0, s, d);
  if (tiles) {
    d.astat = astat;
    const int nt = cdiv(K + 1, 32);
    hipLaunchKernelGGL(finalize_afactor_kernel, dim3(nt * (nt + 1) / 2), dim3(256), 0, s, d, nt);
  }
  ACMI_LAUNCH_CHECK("wgrad_layer");
  return ACMI_OK;
}

// G = g^T g / rows for g [rows][ld] (first n columns), via split-K; gmax: the
// published max |g| (bit pattern) -- the wide Grams then run on f16x2 split
// operands (three MFMAs per product instead of bf16x3's six)
// defer: append the finalize to this set instead of launching it (the caller
// launches the set once; *used: the partial floats this Gram wrote)
static int gcov_layer(const float* g, int ld, int n, long long rows, int sub,
                      float* part, long long part_cap, float* out,
                      hipStream_t s, float* out_v = nullptr, int v_index = -1,
                      const unsigned* gmax = nullptr, CovSet* defer = nullptr, long long* used = nullptr) {
  int np, nc;
  if (n <= 32) {  // narrow: streaming Gram kernel (f32 MFMA; 64 wide runs faster on the split-K
                  // bf16x3 GEMM below: conv2's G factor 82 + 25 -> 59 + 16 us)
    np = n <= 32 ? 32 : 64;
    long long ch;
    gram_plan(rows, &nc, &ch);
    ACMI_REQUIRE((long long)nc * (np + 1) * np <= part_cap, ACMI_ERR_WS, "gcov workspace too small");
    if (np == 32)
      hipLaunchKernelGGL(gram_small_kernel<32>, dim3(nc), dim3(256), 0, s, g, ld, n, rows, ch, part);
    else
      hipLaunchKernelGGL(gram_small_kernel<64>, dim3(nc), dim3(256), 0, s, g, ld, n, rows, ch, part);
  } else {
    const GcovPlan pl = gcov_plan(n, rows);
    np = pl.np;
    nc = pl.nc;
    DenseRows src{g, ld, (int)rows, np};
    RowsAsI<DenseRows> op{src};
    ACMI_REQUIRE(pl.floats <= part_cap, ACMI_ERR_WS, "gcov workspace too small");
    EpiPartial epi{part, np, np};
    if (gmax && g_gemm_mode == ACMI_GEMM_X3)
      launch_gemm3_f16_splitk<64, 64, 16, 1, 1>(op, op, epi, np, np, (int)rows, nc, (int)pl.ch, gmax, gmax, s, np);
    else
      launch_mm<64, 64, 32, 1, 1, true, false, 16>(op, op, epi, np, np, (int)rows, nc, pl.ch, s, np);
  }
  if (used) *used = (long long)nc * (np + 1) * np;
  if (defer) {
    defer->add(part, nc, np, sub, out, (int)rows, nc <= 64 ? (sub >= 64 ? 3 : 0) : 1);
    if (out_v) defer->add(part, nc, np, 1, out_v, (int)rows, 2, v_index);
    ACMI_LAUNCH_CHECK("gcov_layer");
    return ACMI_OK;
  }
  if (nc <= 64)
    hipLaunchKernelGGL(finalize_cov_thread_kernel, dim3(cdiv((long long)sub * sub, 256)), dim3(256), 0,
                       s, part, nc, np, sub, out, (int)rows);
  else
    hipLaunchKernelGGL(finalize_cov_kernel, dim3(cdiv((long long)sub * sub, 4)), dim3(256), 0,
                       s, part, nc, np, sub, out, (int)rows);
  if (out_v)
    hipLaunchKernelGGL(finalize_cov_elem_kernel, dim3(1), dim3(64), 0, s, part, nc, np,
                       v_index, out_v, (int)rows);
  ACMI_LAUNCH_CHECK("gcov_layer");
  return ACMI_OK;
}

// the split-K partial region's minimum: the largest partial over all layers (with
// stats, both gemm modes, both Gram paths, the band reductions)
static long long bwd_partial_floats(int B, int A, int C3) {
  long long m = 0;
  const long long rowsL[5] = {400LL * B, 81LL * B, 49LL * B, B, B};
  const int Ks[5] = {256, 512, 576, 49 * C3, 512};
  const int co[5] = {32, 64, C3, 512, A + 1};
  for (int l = 0; l < 5; ++l) {
    for (int mode : {ACMI_GEMM_F32, ACMI_GEMM_X3})
      m = std::max(m, wgrad_plan(Ks[l], co[l], true, rowsL[l], false, mode).floats);
    for (int mode : {ACMI_GEMM_F32, ACMI_GEMM_X3})
      m = std::max(m, wgrad_plan(Ks[l], co[l], false, rowsL[l], l == 0, mode).floats);
    // G factors of the same layer's output
    if (co[l] <= 64) {  // (both Gram paths sized: gcov_layer picks by width)
      int nc;
      long long ch;
      gram_plan(rowsL[l], &nc, &ch);
      const long long np = co[l] <= 32 ? 32 : 64;
      m = std::max(m, nc * (np + 1) * np);
    }
    m = std::max(m, gcov_plan(co[l], rowsL[l]).floats);
  }
  // band reductions of conv2 / conv3 (rows = images)
  m = std::max(m, band_ws_floats(band_host_plan(20, 20, 32, 4, 4, 2, 64), B));
  m = std::max(m, band_ws_floats(band_host_plan(9, 9, 64, 3, 3, 1, C3), B));
  return (m + 63) / 64 * 64;
}

static long long afactor_ws_floats(int B) { return conv1_afactor_ws_ints(400LL * B); }

// Workspace of acmi_backward / acmi_kfac_output_stats (one size for both):
//   backward:      [scratch kBandScratch | conv1 A-factor ints | partials ...]
//   output stats:  [scratch kBandScratch | sampled head gradients B x ldg | partials ...]
// (prefixes rounded to 256 B); the partial region is the rest of the caller's
// buffer, at least bwd_partial_floats
static long long head_grad_ldg(int A) { return roundup4(A + 1) < 8 ? 8 : roundup4(A + 1); }
static long long bwd_prefix_floats(int B) { return kBandScratch + (afactor_ws_floats(B) + 63) / 64 * 64; }
static long long stats_prefix_floats(int B, int A) { return kBandScratch + ((long long)B * head_grad_ldg(A) + 63) / 64 * 64; }
static int g_ws_flushes = 0;  // acmi_debug_ws_flushes

// Recorded on the backward's stream right after its input-gradient chain (per
// device): acmi_stream_wait_backward_dx lets the sampled-loss chain on another
// stream start there, next to the weight-gradient reductions instead of next to
// the (memory-bound) input gradients.
static hipEvent_t* dx_done_event() {
  static hipEvent_t ev[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!ev[dev] && hipEventCreateWithFlags(&ev[dev], hipEventDisableTiming) != hipSuccess) {
    ev[dev] = nullptr;
    return nullptr;
  }
  return &ev[dev];
}
// ---------------------------------------------------------------------------
// backward (dX chain) shared by the loss backward and the sampled backward
// ---------------------------------------------------------------------------
// the chain up to d2: heads -> d4, fc4 -> d3, conv3 -> d2
template <int C3>
static int dx_chain_pre(const Layout& L, const float* P, int B, const acmi_acts_t* a,
                        const acmi_bwd_t* bw, const float* dhead, int ldh,
                        hipStream_t s, const char* prep, unsigned* dxs) {
  // dxs: kBandScratch words of scratch (band.hpp layout): the dX epilogues publish
  // max |d3|, |d2| there, the f16x2 consumers (convt2, the band reductions) scale
  // by them
  ACMI_REQUIRE(dxs, ACMI_ERR_ARG, "dx_chain: no scratch");
  ACMI_REQUIRE(hipMemsetAsync(dxs, 0, kBandScratch * sizeof(unsigned), s) == hipSuccess, ACMI_ERR_HIP,
               "dx_chain: scratch reset failed");
  // heads -> d4 = (dhead W_h^T) * relu'(a4)
  if (L.A == 4 && ldh % 4 == 0 && (uintptr_t)(P + L.off[8]) % 16 == 0 && (uintptr_t)dhead % 16 == 0)
    hipLaunchKernelGGL(heads_dx4_kernel, dim3(cdiv((long long)B * 128, 256)), dim3(256), 0, s, dhead,
                       ldh, B, P + L.off[8], P + L.off[10], a->a4, bw->d4, dxs + kBsMaxD4);
  else
    hipLaunchKernelGGL(heads_dx_kernel, dim3(cdiv((long long)B * 128, 256)), dim3(256), 0, s, dhead,
                       ldh, B, P + L.off[8], P + L.off[10], L.A, a->a4, bw->d4, dxs + kBsMaxD4);
  // max |W3|, |W4| for the f16x2 operands below: from the prepared weights'
  // header, else computed here
  const unsigned* hdr = prep ? reinterpret_cast<const unsigned*>(prep + TowerPrep<C3>::HDR) : nullptr;
  const unsigned* w3max = hdr ? hdr + kTowMaxW3 : dxs + kBsMaxW3;
  const unsigned* w4max = hdr ? hdr + kTowMaxW4 : dxs + kBsMaxW4;
  if (!hdr && g_gemm_mode == ACMI_GEMM_X3) {
    hipLaunchKernelGGL(absmax_kernel, dim3(16), dim3(256), 0, s, P + L.off[4], (long long)576 * C3,
                       dxs + kBsMaxW3);
    hipLaunchKernelGGL(absmax_kernel, dim3(64), dim3(256), 0, s, P + L.off[6], (long long)49 * C3 * 512,
                       dxs + kBsMaxW4);
  }
  {  // fc4 -> d3 = (d4 W4^T) * relu'(a3)
    const int K3 = 49 * C3;
    RowsAsK<DenseRows> opA{DenseRows{bw->d4, 512, B, 512}};
    MatTK<true> opB{P + L.off[6], 512, 512, K3};
    // f16x2 on 128 x 64 tiles, BK = 32 (per launch at M = 10240: 89.8 us; 64 x 128
    // 107, 128 x 128 96.6, 64 x 128 / BK 32 97.1, 256 x 128 127.7; bf16x3 64 x 128 132)
    auto run = [&](auto epi) {
      if (g_gemm_mode == ACMI_GEMM_X3)
        launch_gemm3_f16<128, 64, 32, 2, 1>(opA, opB, epi, B, K3, 512, dxs + kBsMaxD4, w4max, s);
      else
        launch_mm<64, 128, 32, 1, 2, false, false, 16>(opA, opB, epi, B, K3, 512, 1, 0, s);
    };
    // ReLU'(a3) from the mask bits when the forward wrote them
    prof_begin(ACMI_PROF_FC4_DX, s);
    if (a->m3) run(EpiReluGrad<true>{bw->d3, reinterpret_cast<const float*>(a->m3), K3, dxs + kBsMaxD3});
    else run(EpiReluGrad<false>{bw->d3, a->a3, K3, dxs + kBsMaxD3});
    prof_end(ACMI_PROF_FC4_DX, s);
  }
  // conv input gradients as transposed products: rows = (phase, channel) of
  // the weights, columns = (super-)pixels gathering dY (EpiConvT, float4 rows)
  {  // conv3 -> d2 (stride 1: one phase)
    // its weights pre-split in the prepared buffer (after fc4's, acmi_conv_prep_bytes)
    const char* ct3p = prep ? prep + TowerPrep<C3>::BYTES + CT2::BYTES + fc4_prep_bytes(49 * C3) : nullptr;
    using Src = ConvTRows<9, 9, 3, 3, 1, C3>;
    using W = ConvTWeights<3, 3, 1, 64, C3>;
    W opA{P + L.off[4]};
    RowsAsK<Src> opB{Src{bw->d3, B * Src::L}};
    auto run = [&](auto epi) {
      if (g_gemm_mode == ACMI_GEMM_X3)
        // f16x2 operands: the scales of max |W3| and of max |d3| (the fc4 dX epilogue's)
        launch_convt_x3<9, 9, 3, 3, 1, 64, C3, 256>(P + L.off[4], ct3p, bw->d3, B, epi, w3max, dxs + kBsMaxD3, s);
      else
        launch_mm<64, 128, 16, 1, 2, false, false, 16>(opA, opB, epi, W::N, B * Src::L, Src::COLS, 1, 0, s);
    };
    prof_begin(ACMI_PROF_CONV3_DX, s);
    if (a->m2) run(EpiConvT<9, 9, 1, 64, true>{bw->d2, reinterpret_cast<const float*>(a->m2), dxs + kBsMaxD2});
    else run(EpiConvT<9, 9, 1, 64>{bw->d2, a->a2, dxs + kBsMaxD2});
    prof_end(ACMI_PROF_CONV3_DX, s);
  }
  ACMI_LAUNCH_CHECK("dx_chain");
  return ACMI_OK;
}

// conv2's input gradient, from d2 (max |d2| in dxs): the loss chain stores the
// masked d1 (gram_part null), the sampled chain reduces it to conv1's G-factor
// Gram partials (*gram_done set when it did)
template <int C3>
static int dx_conv2(const Layout& L, const float* P, int B, const acmi_acts_t* a, const acmi_bwd_t* bw,
                    hipStream_t s, const char* prep, float* gram_part, bool* gram_done, unsigned* dxs) {
  if (gram_done) *gram_done = false;
  {  // conv2 -> d1 (stride 2: the four phases of a 2x2 super-pixel are the
     // 4 x 32 rows of one product over the 10x10 super-pixels)
    using Src = ConvTRows<20, 20, 4, 4, 2, 64>;
    using W = ConvTWeights<4, 4, 2, 32, 64>;
    W opA{P + L.off[2]};
    RowsAsK<Src> opB{Src{bw->d2, B * Src::L}};
    // (max |d1|: conv1's f16x2 weight gradient; ReLU'(a1) from the mask bits when written)
    const float* act1 = a->m1 ? reinterpret_cast<const float*>(a->m1) : a->a1;
    prof_begin(ACMI_PROF_CONV2_DX, s);
    const char* p2 = prep ? prep + TowerPrep<C3>::BYTES : nullptr;
    if (p2 && g_gemm_mode == ACMI_GEMM_X3) {
      // pre-split weights, four phases per wave (convt2.hpp); the sampled-loss
      // chain reduces d1 to its Gram partials instead of storing it
      auto go = [&](auto GRAMc, auto MASKc) {
        constexpr bool GR = decltype(GRAMc)::value, MK = decltype(MASKc)::value;
        if (GR)
          hipLaunchKernelGGL((convt2_kernel<GR, MK>), dim3(convt2_gram_blocks(B)), dim3(256), 0, s, p2, bw->d2,
                             act1, nullptr, B, gram_part, dxs + kBsMaxD2, nullptr);
        else
          hipLaunchKernelGGL((convt2_kernel<GR, MK>), dim3(convt2_store_blocks(B)), dim3(256), 0, s, p2,
                             bw->d2, act1, bw->d1, B, nullptr, dxs + kBsMaxD2, dxs + kBsMaxD1);
      };
      using T = std::true_type;
      using F = std::false_type;
      if (gram_part) {
        if (a->m1) go(T{}, T{});
        else go(T{}, F{});
        if (gram_done) *gram_done = true;
      } else {
        if (a->m1) go(F{}, T{});
        else go(F{}, F{});
      }
    } else if (a->m1) {
      launch_mm<128, 128, 16, 2, 2, false, false, 16>(
          opA, opB, EpiConvT<20, 20, 2, 32, true>{bw->d1, act1, dxs + kBsMaxD1}, W::N, B * Src::L, Src::COLS, 1, 0, s);
    } else {
      launch_mm<128, 128, 16, 2, 2, false, false, 16>(opA, opB, EpiConvT<20, 20, 2, 32>{bw->d1, act1, dxs + kBsMaxD1},
                                                      W::N, B * Src::L, Src::COLS, 1, 0, s);
    }
    prof_end(ACMI_PROF_CONV2_DX, s);
  }
  ACMI_LAUNCH_CHECK("dx_conv2");
  return ACMI_OK;
}

template <int C3>
static int dx_chain(const Layout& L, const float* P, int B, const acmi_acts_t* a,
                    const acmi_bwd_t* bw, const float* dhead, int ldh,
                    hipStream_t s, const char* prep = nullptr, float* gram_part = nullptr,
                    bool* gram_done = nullptr, unsigned* dxs = nullptr) {
  const int rc = dx_chain_pre<C3>(L, P, B, a, bw, dhead, ldh, s, prep, dxs);
  if (rc) return rc;
  return dx_conv2<C3>(L, P, B, a, bw, s, prep, gram_part, gram_done, dxs);
}

template <int C3>
static int backward_impl(const Layout& L, const float* P, const uint8_t* obs,
                         long long img_stride, int B, const acmi_acts_t* a,
                         const acmi_bwd_t* bw, float* grads, float* astat,
                         float* ws, long long ws_cap, hipStream_t s, const char* prep,
                         bool dx_done = false) {
  // dx_done: the caller ran the dX chain into bw / the scratch (backward_stacked_impl)
  const bool st = astat != nullptr;
  // conv1's weight gradient is fused into the A-factor pass (bf16x3 mode; it needs
  // d1, so the pass follows the dX chain).  (Measured and removed: the A factor on a
  // library side stream next to the dX chain, 5.69 vs 5.64 ms per update -- the i8
  // gather competes with the symmetric reductions for L2 and LDS; the A factor
  // before the dX chain.)
  const bool fuse_c1 = st && g_gemm_mode == ACMI_GEMM_X3;
  // operand-scale scratch (band.hpp) first: the dX epilogues publish max |d3|,
  // |d2| into it; then the conv1 A-factor integers; the partial region is the rest
  unsigned* bscr = reinterpret_cast<unsigned*>(ws);
  const long long prefix = bwd_prefix_floats(B);
  float* part = ws + prefix;
  const long long avail = ws_cap - prefix;
  const bool band = band_on(st);
  int rc = ACMI_OK;
  if (!dx_done) {
    rc = dx_chain<C3>(L, P, B, a, bw, bw->dhead, bw->ldh, s, prep, nullptr, nullptr, bscr);
    if (rc) return rc;
    hipEvent_t* ev = dx_done_event();
    ACMI_REQUIRE(ev && hipEventRecord(*ev, s) == hipSuccess, ACMI_ERR_HIP, "acmi_backward: dX event record failed");
  }
  float* wpart_c1 = nullptr;  // conv1's fused weight-gradient partials (in the A-factor workspace)
  if (st) {
    prof_begin(ACMI_PROF_CONV1_AFACTOR, s);
    const int rc0 = conv1_afactor_u8(obs, img_stride, B, astat + L.stat_off[0],
                                     reinterpret_cast<int*>(ws + kBandScratch), afactor_ws_floats(B), s,
                                     fuse_c1 ? bw->d1 : nullptr, &wpart_c1, bscr + kBsMaxD1);
    prof_end(ACMI_PROF_CONV1_AFACTOR, s);
    if (rc0) return rc0;
  }
  // the conv1, heads and fc4 finalizes deferred into one launch: each layer's
  // partials in their own range of the partial region (a layer that does not fit
  // after the others finalizes the set so far first -- at workspaces near the
  // minimum, acmi_debug_ws_flushes counts it)
  WgradSet fin;
  long long off = 0;
  auto flush = [&]() {
    if (fin.n) hipLaunchKernelGGL(finalize_wgrad_multi_kernel, dim3(fin.blocks), dim3(256), 0, s, fin);
    fin = WgradSet();
    off = 0;
  };
  if (st && fuse_c1) {  // the conv1 weight gradient came with the A factor: reduce its chunks
    const long long rows = 400LL * B;
    WgradDesc d{wpart_c1, conv1_afactor_fused_chunks(rows), 256, 32, 0, 32, grads + L.off[0], 32,
                nullptr, nullptr, (int)rows, 1.0f / 255.0f};
    fin.add(d, 0, 0, fin_blocks(d));
  }
  // need: the layer's partial floats (its plan), checked here so that a layer
  // that does not fit after the others starts a new range instead of failing;
  // the layer then reports what it used, which must be that plan
  auto layer = [&](long long need, auto&& run) -> int {
    long long used = 0;
    if (off > 0 && need > avail - off) ++g_ws_flushes, flush();
    else if (fin.n + 2 > kWgradTasks) flush();
    const int r = run(part + off, avail - off, &used);
    ACMI_REQUIRE(r != ACMI_OK || used == need, ACMI_ERR_ARG,
                 "internal: a layer used %lld partial floats against its planned %lld", used, need);
    off += (used + 3) / 4 * 4;
    return r;
  };
  // heads: X = a4 (512), dY = dhead (A+1 columns: pi | v)
  rc = layer(wgrad_plan(512, L.A + 1, st, B).floats, [&](float* pt, long long cap, long long* used) {
    return wgrad_layer(DenseRows{a->a4, 512, B, 512}, 512, B, bw->dhead, bw->ldh, L.A + 1, st, pt, cap,
                       grads + L.off[8], L.A, grads + L.off[10], st ? astat + L.stat_off[4] : nullptr, s, 0, 1.f,
                       nullptr, nullptr, &fin, used);
  });
  if (rc) return rc;
  // fc4: X = a3 flat; f16x2 with the prepared weights' a3 bound and max |d4|
  // (published by the dX chain's heads kernel)
  const unsigned* a3b =
      prep ? reinterpret_cast<const unsigned*>(prep + TowerPrep<C3>::HDR) + kTowMaxA3 : nullptr;
  rc = layer(wgrad_plan(49 * C3, 512, st, B).floats, [&](float* pt, long long cap, long long* used) {
    return wgrad_layer(DenseRows{a->a3, 49 * C3, B, 49 * C3}, 49 * C3, B, bw->d4, 512, 512, st, pt, cap,
                       grads + L.off[6], 512, nullptr, st ? astat + L.stat_off[3] : nullptr, s, 0, 1.f, a3b,
                       a3b ? bscr + kBsMaxD4 : nullptr, &fin, used);
  });
  if (rc) return rc;
  flush();
  // conv3 / conv2: pixel-pair band reductions over the dense activation rows
  // (band.hpp), or the patches of a2 / a1
  const long long band_cap = avail;
  // a1 / a2 bounds from the weights (max |d2|, |d3| came with the dX chain): the
  // prepared weights' header holds them (tower_stats_body, the same sums as
  // band_bounds_kernel), else computed here
  const unsigned* xb = prep ? reinterpret_cast<const unsigned*>(prep + TowerPrep<C3>::HDR) : nullptr;
  const unsigned* a1b = xb ? xb + kTowMaxA1 : bscr + kBsMaxA1;
  const unsigned* a2b = xb ? xb + kTowMaxA2 : bscr + kBsMaxA2;
  if (band) {
    if (!xb)
      hipLaunchKernelGGL(band_bounds_kernel, dim3(64), dim3(256), 0, s, P + L.off[0], P + L.off[1], P + L.off[2],
                         P + L.off[3], bscr);
    rc = band_layer(a->a2, 9, 9, 64, 3, 3, 1, bw->d3, C3, B, part, band_cap, grads + L.off[4],
                    astat + L.stat_off[2], 1.f, a2b, bscr + kBsMaxD3, s);
  } else
    rc = wgrad_layer(ConvRows<float, 9, 9, 64, 3, 3, 1>{a->a2, 81 * 64, B * 49}, 576, 49LL * B,
                     bw->d3, C3, C3, st, part, avail, grads + L.off[4], C3, nullptr,
                     st ? astat + L.stat_off[2] : nullptr, s);
  if (rc) return rc;
  if (band)
    rc = band_layer(a->a1, 20, 20, 32, 4, 4, 2, bw->d2, 64, B, part, band_cap, grads + L.off[2],
                    astat + L.stat_off[1], 1.f, a1b, bscr + kBsMaxD2, s, ACMI_PROF_CONV2_WGRAD);
  else
    rc = wgrad_layer(ConvRows<float, 20, 20, 32, 4, 4, 2>{a->a1, 400 * 32, B * 81}, 512,
                     81LL * B, bw->d2, 64, 64, st, part, avail, grads + L.off[2], 64, nullptr,
                     st ? astat + L.stat_off[1] : nullptr, s, ACMI_PROF_CONV2_WGRAD);
  if (rc) return rc;
  // conv1: patches of the u8 observations
  // conv1: weight gradient on the f32 engine; its A factor from the u8 frames on
  // the i8 matrix cores (exact integer sums, afactor_u8.hip)
  if (!fuse_c1)
    rc = wgrad_layer(ConvRows<uint8_t, 84, 84, 4, 8, 8, 4>{obs, (uint32_t)img_stride, B * 400}, 256,
                     400LL * B, bw->d1, 32, 32, false, part, avail, grads + L.off[0], 32, nullptr,
                     nullptr, s, ACMI_PROF_CONV1_WGRAD, 1.0f / 255.0f);  // raw u8 patches
  return rc;
}

// sampled-loss output gradients at the heads (kfac "gradients" mode):
// g_pi = softmax(z) - onehot(y), y ~ Cat(z);  g_v = V - y_v = -eps, eps~N(0,1)
__global__ void sampled_head_grad_kernel(const float* logits, int ld, int B, int A,
                                         uint32_t seed, uint32_t row0, uint32_t ctr,
                                         float* g, int ldg) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= B) return;
  const float* z = logits + (long long)m * ld;
  float mx = -INFINITY;
  for (int a = 0; a < A; ++a) mx = fmaxf(mx, z[a]);
  float se = 0.f;
  for (int a = 0; a < A; ++a) se += expf(z[a] - mx);
  // keyed by the global row: a data-parallel shard draws what the full batch would
  const uint32_t h = key4(seed, 0u, ctr, row0 + (uint32_t)m);
  const float u = u01(h);
  // inverse CDF draw
  const float target = u * se;
  float c = 0.f;
  int y = A - 1;
  for (int a = 0; a < A; ++a) {
    c += expf(z[a] - mx);
    if (target < c) { y = a; break; }
  }
  float* gr = g + (long long)m * ldg;
  for (int a = 0; a < A; ++a) gr[a] = expf(z[a] - mx) / se - (a == y ? 1.f : 0.f);
  // Box-Muller from two further counters
  const float u1 = u01(mix32(h ^ 0x68e31da4U)) + (1.0f / 33554432.0f);
  const float u2 = u01(mix32(h ^ 0xb5297a4dU));
  const float eps = sqrtf(-2.f * logf(u1)) * cosf(6.2831853071795864f * u2);
  gr[A] = -eps;
  for (int a = A + 1; a < ldg; ++a) gr[a] = 0.f;
}

template <int C3>
static int output_stats_impl(const Layout& L, const float* P, int B,
                             const acmi_acts_t* a, const acmi_bwd_t* bw,
                             uint32_t seed, uint32_t row0, uint32_t ctr,
                             float* gstat, float* ws, long long ws_cap,
                             hipStream_t s, const char* prep, int stage = 0) {
  // stage: 0 the whole chain; 2 only the G factors, from what backward_stacked_impl
  // left in bw (d2..d4) and in this workspace (scratch maxima, conv1's Gram partials)
  const int ldg = (int)head_grad_ldg(L.A);
  // [the dX chain's scratch (operand-scale maxima) | ghead [B][ldg] | partials]
  unsigned* dxs = reinterpret_cast<unsigned*>(ws);
  float* ghead = ws + kBandScratch;
  const long long prefix = stats_prefix_floats(B, L.A);
  float* part = ws + prefix;
  const long long cap = ws_cap - prefix;
  bool g1_done = false;
  const bool g1_fits = (long long)convt2_gram_blocks(B) * 33 * 32 <= cap;
  int rc = ACMI_OK;
  if (stage == 0) {
    hipLaunchKernelGGL(sampled_head_grad_kernel, dim3(cdiv(B, 128)), dim3(128), 0, s,
                       a->logits, a->ld_logits, B, L.A, seed, row0, ctr, ghead, ldg);
    rc = dx_chain<C3>(L, P, B, a, bw, ghead, ldg, s, prep, g1_fits ? part : nullptr, &g1_done, dxs);
    if (rc) return rc;
  } else {
    g1_done = g1_fits && prep && g_gemm_mode == ACMI_GEMM_X3;  // (dx_conv2's Gram predicate)
  }
  // the G factors' finalizes deferred into one launch: every Gram's partials in
  // their own range of the workspace (while they fit; else the set so far is
  // finalized and the ranges start over)
  CovSet fin;
  long long off = 0;
  auto flush = [&]() {
    if (fin.n) hipLaunchKernelGGL(finalize_cov_multi_kernel, dim3(fin.blocks), dim3(256), 0, s, fin);
    fin = CovSet();
    off = 0;
  };
  if (g1_done) {  // G of conv1's output from the conv2 dX kernel's per-block Gram partials
    fin.add(part, convt2_gram_blocks(B), 32, 32, gstat + L.stat_off[5 + 0], (int)(400LL * B), 1);
    off = ((long long)convt2_gram_blocks(B) * 33 * 32 + 3) / 4 * 4;
  }
  // one Gram into the next free range, or -- when its plan's partials do not fit
  // after the others -- into a new range after the set so far is finalized
  auto gram = [&](const float* g, int ld, int n, long long rows, int sub, float* out, float* out_v, int vi,
                  const unsigned* gmax) -> int {
    long long used = 0;
    const long long need = gcov_need(n, rows);
    if (off > 0 && need > cap - off) ++g_ws_flushes, flush();
    else if (fin.n + 2 > kCovTasks) flush();
    const int r = gcov_layer(g, ld, n, rows, sub, part + off, cap - off, out, s, out_v, vi, gmax, &fin, &used);
    ACMI_REQUIRE(r != ACMI_OK || used == need, ACMI_ERR_ARG,
                 "internal: a Gram used %lld partial floats against its planned %lld", used, need);
    off += (used + 3) / 4 * 4;
    return r;
  };
  // heads: G_pi (A x A) from the first A columns, G_v = element (A, A)
  rc = gram(ghead, ldg, L.A + 1, B, L.A, gstat + L.stat_off[5 + 4], gstat + L.stat_off[5 + 5], L.A, nullptr);
  if (rc) return rc;
  // (the dX chain above published max |d4| and max |d2| into dxs)
  rc = gram(bw->d4, 512, 512, B, 512, gstat + L.stat_off[5 + 3], nullptr, -1, dxs + kBsMaxD4);
  if (rc) return rc;
  rc = gram(bw->d3, C3, C3, 49LL * B, C3, gstat + L.stat_off[5 + 2], nullptr, -1, nullptr);
  if (rc) return rc;
  rc = gram(bw->d2, 64, 64, 81LL * B, 64, gstat + L.stat_off[5 + 1], nullptr, -1, dxs + kBsMaxD2);
  if (rc) return rc;
  if (!g1_done) rc = gram(bw->d1, 32, 32, 400LL * B, 32, gstat + L.stat_off[5 + 0], nullptr, -1, nullptr);
  if (rc) return rc;
  flush();
  ACMI_LAUNCH_CHECK("G factor finalize");
  return ACMI_OK;
}

// acmi_backward + the input-gradient half of acmi_kfac_output_stats, with conv2's
// input gradient of both chains as ONE launch (convt2_kernel MIX: one W2^T
// stream, the loss chain's tiles storing d1, the sampled chain's reducing
// conv1's G-factor Gram); the G factors follow in output_stats_impl stage 2.
// Bit-identical to the two calls.
template <int C3>
static int backward_stacked_impl(const Layout& L, const float* P, const uint8_t* obs, long long img_stride, int B,
                                 const acmi_acts_t* a, const acmi_bwd_t* bw, float* grads, float* astat, float* ws,
                                 long long ws_cap, const acmi_bwd_t* bws, uint32_t seed, uint32_t row0, uint32_t ctr,
                                 float* wss, long long wss_cap, hipStream_t s, const char* prep) {
  unsigned* bscr = reinterpret_cast<unsigned*>(ws);
  int rc = dx_chain_pre<C3>(L, P, B, a, bw, bw->dhead, bw->ldh, s, prep, bscr);
  if (rc) return rc;
  // the sampled chain's head gradients and its chain up to d2 (output_stats_impl's layout)
  const int ldg = (int)head_grad_ldg(L.A);
  unsigned* dxs = reinterpret_cast<unsigned*>(wss);
  float* ghead = wss + kBandScratch;
  float* part_s = wss + stats_prefix_floats(B, L.A);
  const long long cap_s = wss_cap - stats_prefix_floats(B, L.A);
  hipLaunchKernelGGL(sampled_head_grad_kernel, dim3(cdiv(B, 128)), dim3(128), 0, s, a->logits, a->ld_logits, B, L.A,
                     seed, row0, ctr, ghead, ldg);
  rc = dx_chain_pre<C3>(L, P, B, a, bws, ghead, ldg, s, prep, dxs);
  if (rc) return rc;
  const bool g1_fits = (long long)convt2_gram_blocks(B) * 33 * 32 <= cap_s;
  if (prep && g_gemm_mode == ACMI_GEMM_X3 && g1_fits) {
    const char* p2 = prep + TowerPrep<C3>::BYTES;
    const float* act1 = a->m1 ? reinterpret_cast<const float*>(a->m1) : a->a1;
    prof_begin(ACMI_PROF_CONV2_DX, s);
    if (a->m1)
      hipLaunchKernelGGL((convt2_kernel<true, true, true>), dim3(convt2_gram_blocks(B)), dim3(256), 0, s, p2, bw->d2,
                         act1, bw->d1, B, part_s, bscr + kBsMaxD2, bscr + kBsMaxD1, bws->d2, dxs + kBsMaxD2);
    else
      hipLaunchKernelGGL((convt2_kernel<true, false, true>), dim3(convt2_gram_blocks(B)), dim3(256), 0, s, p2, bw->d2,
                         act1, bw->d1, B, part_s, bscr + kBsMaxD2, bscr + kBsMaxD1, bws->d2, dxs + kBsMaxD2);
    prof_end(ACMI_PROF_CONV2_DX, s);
    ACMI_LAUNCH_CHECK("stacked conv2 dX");
  } else {  // the two launches (no prepared weights / f32 mode / a workspace without room for the Gram)
    rc = dx_conv2<C3>(L, P, B, a, bw, s, prep, nullptr, nullptr, bscr);
    if (rc) return rc;
    bool g1_done = false;
    rc = dx_conv2<C3>(L, P, B, a, bws, s, prep, g1_fits ? part_s : nullptr, &g1_done, dxs);
    if (rc) return rc;
  }
  {
    hipEvent_t* ev = dx_done_event();
    ACMI_REQUIRE(ev && hipEventRecord(*ev, s) == hipSuccess, ACMI_ERR_HIP, "acmi_backward: dX event record failed");
  }
  return backward_impl<C3>(L, P, obs, img_stride, B, a, bw, grads, astat, ws, ws_cap, s, prep, true);
}

}  // namespace acmi

using namespace acmi;

extern "C" {

const char* acmi_last_error(void) { return g_err; }
int acmi_abi_version(void) { return ACMI_ABI_VERSION; }
int acmi_abi_struct_sizes(int64_t* sizes, int n) {
  const int64_t all[5] = {(int64_t)sizeof(acmi_net_t), (int64_t)sizeof(acmi_acts_t), (int64_t)sizeof(acmi_bwd_t),
                          (int64_t)sizeof(acmi_env_state_t), (int64_t)sizeof(acmi_rollout_io_t)};
  if (!sizes || n < 0) return 0;
  const int k = n < 5 ? n : 5;
  for (int i = 0; i < k; ++i) sizes[i] = all[i];
  return k;
}

int acmi_set_gemm_mode(int mode) {
  ACMI_REQUIRE(mode == ACMI_GEMM_F32 || mode == ACMI_GEMM_X3, ACMI_ERR_ARG,
               "acmi_set_gemm_mode: unknown mode %d", mode);
  ACMI_REQUIRE(mode == ACMI_GEMM_X3 || s_forward_mode == ACMI_FWD_F32, ACMI_ERR_ARG,
               "acmi_set_gemm_mode: f32 gemm mode has no bf16 forward (acmi_set_forward_mode(ACMI_FWD_F32) first)");
  s_gemm_mode = g_gemm_mode = mode;
  return ACMI_OK;
}
int acmi_get_gemm_mode(void) { return s_gemm_mode; }

int acmi_set_forward_mode(int mode) {
  ACMI_REQUIRE(mode == ACMI_FWD_F32 || mode == ACMI_FWD_BF16, ACMI_ERR_ARG, "acmi_set_forward_mode: bad mode %d",
               mode);
  // the bf16 arithmetic exists only in the fused tower (tower.hpp): refuse a mode
  // the forward could not honour instead of silently computing in f32
  ACMI_REQUIRE(mode == ACMI_FWD_F32 || s_gemm_mode == ACMI_GEMM_X3, ACMI_ERR_ARG,
               "acmi_set_forward_mode: bf16 forward needs the fused tower (x3 gemm mode)");
  s_forward_mode = g_forward_mode = mode;
  return ACMI_OK;
}
int acmi_get_forward_mode(void) { return s_forward_mode; }

int acmi_set_conv_stats_mode(int mode) {
  ACMI_REQUIRE(mode == ACMI_CONV_STATS_PATCHES || mode == ACMI_CONV_STATS_BAND, ACMI_ERR_ARG,
               "acmi_set_conv_stats_mode: unknown mode %d", mode);
  s_conv_stats_mode = g_conv_stats_mode = mode;
  return ACMI_OK;
}
int acmi_get_conv_stats_mode(void) { return s_conv_stats_mode; }


int acmi_band_info(int layer, int C3, int64_t rows, int64_t* info) {
  ACMI_REQUIRE(info && (layer == 1 || layer == 2) && (C3 == 32 || C3 == 64) && rows > 0, ACMI_ERR_ARG,
               "acmi_band_info: bad arguments");
  const BandPlan* p = layer == 1 ? band_host_plan(20, 20, 32, 4, 4, 2, 64) : band_host_plan(9, 9, 64, 3, 3, 1, C3);
  ACMI_REQUIRE(p, ACMI_ERR_ARG, "acmi_band_info: no plan");
  int nc, ch;
  band_chunks(rows, (int)p->groups.size(), &nc, &ch);
  info[0] = p->ntiles;
  info[1] = (int64_t)p->groups.size();
  info[2] = nc;
  info[3] = ch;
  int units = 0;
  for (const BandGroup& G : p->groups) {
    int t = 0;
    for (int w = 0; w < 8; ++w) t += (G.ra[w][0] >= 0) + (G.ra[w][1] >= 0);
    units += (t + 3) / 4;
  }
  info[4] = units;  // sum over groups of the busiest SIMD's sub-tiles
  return ACMI_OK;
}

int64_t acmi_param_count(int A, int C3) {
  Layout L;
  if (!make_layout(A, C3, &L)) return -1;
  return L.total;
}

int acmi_param_offsets(int A, int C3, int64_t* off) {
  Layout L;
  ACMI_REQUIRE(off && make_layout(A, C3, &L), ACMI_ERR_ARG, "bad A=%d/C3=%d", A, C3);
  for (int i = 0; i < 12; ++i) off[i] = L.off[i];
  return ACMI_OK;
}

int acmi_kfac_layout(int A, int C3, int64_t* din, int64_t* dout, int64_t* so, int64_t* total) {
  Layout L;
  ACMI_REQUIRE(make_layout(A, C3, &L), ACMI_ERR_ARG, "bad A=%d/C3=%d", A, C3);
  for (int l = 0; l < 6; ++l) {
    if (din) din[l] = L.din[l];
    if (dout) dout[l] = L.dout[l];
  }
  for (int f = 0; f < 11; ++f)
    if (so) so[f] = L.stat_off[f];
  if (total) *total = L.stat_total;
  return ACMI_OK;
}

// The GEMM operand loaders address with 32-bit element offsets (gemm_ops.hpp):
// every buffer a launch reads must span < 2^31 elements.
static bool spans32(long long rows, long long stride, long long per_row) {
  return rows <= 0 || (rows - 1) * stride + per_row < (1LL << 31);
}

static int forward_dispatch(const acmi_net_t* net, const uint8_t* obs, int64_t img_stride,
                            int B, const acmi_acts_t* acts, int want_value,
                            long long act_stride, acmi_stream_t stream,
                            const TailArgs* tail = nullptr) {
  Layout L;
  ACMI_REQUIRE(net && acts && obs && net->params, ACMI_ERR_ARG, "acmi_forward: null argument");
  ACMI_REQUIRE(make_layout(net->num_actions, net->conv3_filters, &L), ACMI_ERR_ARG,
               "acmi_forward: bad A=%d/C3=%d", net->num_actions, net->conv3_filters);
  ACMI_REQUIRE(B >= 0 && img_stride >= 84 * 84 * 4 && img_stride % 4 == 0, ACMI_ERR_ARG,
               "acmi_forward: bad B=%d / img_stride=%lld", B, (long long)img_stride);
  ACMI_REQUIRE(acts->a1 && acts->a2 && acts->a3 && acts->a4 && acts->logits &&
                   acts->ld_logits >= net->num_actions && (!want_value || acts->value),
               ACMI_ERR_ARG, "acmi_forward: bad activation buffers");
  ACMI_REQUIRE(masks_ok(acts), ACMI_ERR_ARG, "acmi_forward: ReLU masks m1..m3 must be all set or all NULL");
  ACMI_REQUIRE(act_stride >= 1, ACMI_ERR_ARG, "bad activation stride");
  ACMI_REQUIRE(spans32(B, img_stride, 84 * 84 * 4) && spans32(B, act_stride * 400 * 32, 400 * 32),
               ACMI_ERR_ARG, "acmi_forward: batch spans >= 2^31 elements (B=%d)", B);
  if (B == 0) return ACMI_OK;
  hipStream_t s = (hipStream_t)stream;
  if (L.C3 == 32)
    return forward_impl<32>(L, net->params, obs, img_stride, B, acts, want_value, act_stride, s, tail,
                            net->conv_prep);
  return forward_impl<64>(L, net->params, obs, img_stride, B, acts, want_value, act_stride, s, tail,
                          net->conv_prep);
}

int64_t acmi_conv_prep_bytes(int C3) {
  // the tower's conv weights, then conv2's input-gradient weights (convt2.hpp)
  // and fc4's weights (fc4roll.hpp)
  // and conv3's input-gradient weights (convt3.hpp)
  return C3 == 32   ? TowerPrep<32>::BYTES + CT2::BYTES + fc4_prep_bytes(49 * 32) + CT3Prep<32>::BYTES
         : C3 == 64 ? TowerPrep<64>::BYTES + CT2::BYTES + fc4_prep_bytes(49 * 64) + CT3Prep<64>::BYTES
                    : -1;
}

// two zeroed runs of 16-byte words in one launch
__global__ __launch_bounds__(256) void zero2_kernel(uint4* a, long long na, uint4* b, long long nb) {
  const uint4 z = make_uint4(0u, 0u, 0u, 0u);
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < na + nb; i += (long long)gridDim.x * 256) {
    if (i < na) a[i] = z;
    else b[i - na] = z;
  }
}

// acmi_conv_prepare's two dependent passes, each one launch over block ranges:
//   bounds: the tower's header (tower_stats_body, 64 blocks) and max |W2| of conv2's
//     input-gradient weights (convt2_wmax_body, kPrepWmaxBlocks), atomicMax into
//     the zeroed words;
//   split: the a3 bound from the final a2 bound (tower_stats3_body, four columns per
//     block), then the f16x2 fragments of the tower, of conv2's input gradient and
//     of fc4 (each scaled by a bound of the first pass)
constexpr int kPrepWmaxBlocks = 32;
struct PrepArgs {
  const float *w1, *b1, *w2, *b2, *w3, *b3, *w4;
  int C3, K4;
  char* tower;       // TowerPrep<C3>
  unsigned* hdr;     // its bounds header
  char* ct2;         // CT2 block
  char* fc4;         // fc4 fragments
  int nb3, nbt, nbc;  // split-pass block counts: stats3, tower, convt2 (fc4, then convt3 after)
  int nbf;            // fc4's
  char* ct3;          // conv3 input-gradient fragments (CT3Prep)
};
__global__ __launch_bounds__(256) void conv_prep_bounds_kernel(PrepArgs a) {
  const int b = blockIdx.x;
  if (b < 64) tower_stats_body(a.w1, a.b1, a.w2, a.b2, a.w3, 576 * a.C3, a.w4, a.K4 * 512, a.hdr, b);
  else convt2_wmax_body(a.w2, a.ct2, b - 64, kPrepWmaxBlocks);
}
__global__ __launch_bounds__(256) void conv_prep_split_kernel(PrepArgs a) {
  int b = blockIdx.x;
  if (b < a.nb3) {
    const int co = 4 * b + (threadIdx.x >> 6);
    if (co < a.C3) tower_stats3_body(a.w3, a.b3, a.C3, a.hdr, co);
  } else if ((b -= a.nb3) < a.nbt) {
    tower_prep_body(a.w1, a.w2, a.w3, a.C3, a.tower, a.hdr, b);
  } else if ((b -= a.nbt) < a.nbc) {
    convt2_prep_body(a.w2, a.ct2, b);
  } else if ((b -= a.nbc) < a.nbf) {
    fc4_prep_body(a.w4, a.K4, a.fc4, a.hdr, b);
  } else {
    b -= a.nbf;
    if (a.C3 == 32) convt3_prep_body<32>(a.w3, a.ct3, a.hdr + kTowMaxW3, b);
    else convt3_prep_body<64>(a.w3, a.ct3, a.hdr + kTowMaxW3, b);
  }
}

int acmi_conv_prepare(const acmi_net_t* net, void* prep, acmi_stream_t stream) {
  ACMI_REQUIRE(net_modes_ok(net), ACMI_ERR_ARG, "acmi_conv_prepare: bad acmi_net_t mode fields");
  const ModeScope mode_scope(net);
  Layout L;
  ACMI_REQUIRE(net && net->params && prep && make_layout(net->num_actions, net->conv3_filters, &L),
               ACMI_ERR_ARG, "acmi_conv_prepare: bad arguments");
  ACMI_REQUIRE((uintptr_t)prep % 16 == 0, ACMI_ERR_ARG, "acmi_conv_prepare: prep must be 16-byte aligned");
  const long long o2 = L.C3 == 32 ? TowerPrep<32>::BYTES : TowerPrep<64>::BYTES;
  const long long oh = L.C3 == 32 ? TowerPrep<32>::HDR : TowerPrep<64>::HDR;
  // the atomicMax targets -- the tower's bounds header and conv2 input gradient's
  // max |W2| words -- zeroed by one launch, then the tower's f16x2 fragments
  static_assert(TowerPrep<32>::HDR_BYTES % 16 == 0 && (CT2::BYTES - CT2::FRAG_BYTES) % 16 == 0 &&
                    TowerPrep<32>::HDR % 16 == 0 && TowerPrep<64>::HDR % 16 == 0 && CT2::FRAG_BYTES % 16 == 0,
                "16-byte runs");
  hipLaunchKernelGGL(zero2_kernel, dim3(64), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<uint4*>(static_cast<char*>(prep) + oh), TowerPrep<32>::HDR_BYTES / 16,
                     reinterpret_cast<uint4*>(static_cast<char*>(prep) + o2 + CT2::FRAG_BYTES),
                     (CT2::BYTES - CT2::FRAG_BYTES) / 16);
  const float* P = net->params;
  char* base = static_cast<char*>(prep);
  const int K4 = 49 * L.C3;
  const int nbf = K4 / 16 * 16 * 64 / 256;
  const int nb3p = (L.C3 == 32 ? CT3Prep<32>::KSTEPS : CT3Prep<64>::KSTEPS) * 2 * 64 / 256;
  PrepArgs a{P + L.off[0], P + L.off[1], P + L.off[2], P + L.off[3], P + L.off[4], P + L.off[5], P + L.off[6],
             L.C3, K4, base, reinterpret_cast<unsigned*>(base + oh), base + o2, base + o2 + CT2::BYTES,
             L.C3 / 4, (16 + 64 + 36 * (L.C3 / 32)) * 64 / 256 + 1, CT2::NKS * 4 * 64 / 256, nbf,
             base + o2 + CT2::BYTES + fc4_prep_bytes(K4)};
  hipLaunchKernelGGL(conv_prep_bounds_kernel, dim3(64 + kPrepWmaxBlocks), dim3(256), 0, (hipStream_t)stream, a);
  hipLaunchKernelGGL(conv_prep_split_kernel, dim3(a.nb3 + a.nbt + a.nbc + nbf + nb3p), dim3(256), 0,
                     (hipStream_t)stream, a);
  ACMI_LAUNCH_CHECK("acmi_conv_prepare");
  return ACMI_OK;
}

int acmi_forward(const acmi_net_t* net, const uint8_t* obs, int64_t img_stride, int B,
                 const acmi_acts_t* acts, int want_value, acmi_stream_t stream) {
  ACMI_REQUIRE(net_modes_ok(net), ACMI_ERR_ARG, "acmi_forward: bad acmi_net_t mode fields");
  const ModeScope mode_scope(net);
  return forward_dispatch(net, obs, img_stride, B, acts, want_value, 1, stream);
}

/* Rollout variant: batch row b is image (b*act_img_stride) of the activation
 * buffers (env-major [N][T] storage; pointers pre-offset by step t). */
int acmi_forward_strided(const acmi_net_t* net, const uint8_t* obs, int64_t img_stride, int B,
                         const acmi_acts_t* acts, int want_value, int64_t act_img_stride,
                         acmi_stream_t stream) {
  ACMI_REQUIRE(net_modes_ok(net), ACMI_ERR_ARG, "acmi_forward_strided: bad acmi_net_t mode fields");
  const ModeScope mode_scope(net);
  return forward_dispatch(net, obs, img_stride, B, acts, want_value, act_img_stride, stream);
}

int acmi_rollout_step(const acmi_net_t* net, const uint8_t* obs, int64_t img_stride, int B,
                      const acmi_acts_t* acts, int64_t act_img_stride, const acmi_rollout_io_t* io,
                      acmi_stream_t stream) {
  ACMI_REQUIRE(net_modes_ok(net), ACMI_ERR_ARG, "acmi_rollout_step: bad acmi_net_t mode fields");
  const ModeScope mode_scope(net);
  ACMI_REQUIRE(io && io->actions && io->bad_rows && io->obs_out && io->rewards && io->terminals &&
                   io->episode_rewards && io->ld >= 1 && io->out_stride % 16 == 0 &&
                   img_stride % 16 == 0 && io->row_offset >= 0 && net &&
                   net->num_actions < kMaxHeads,
               ACMI_ERR_ARG, "acmi_rollout_step: bad arguments");
  TailArgs ta{*io, obs, (long long)img_stride};
  return forward_dispatch(net, obs, img_stride, B, acts, 1, act_img_stride, stream, &ta);
}

int64_t acmi_forward_ws_floats(int B) {
  if (B <= 0) return 0;
  int nz, chunk;
  fc4_plan(B, 49 * 64, &nz, &chunk);
  int nz2, chunk2;
  fc4_plan(B, 49 * 32, &nz2, &chunk2);
  // + the split rollout step's pending env states (forward_impl)
  return (long long)std::max(nz, nz2) * (B + 1) * 512 +
         (B <= kSplitMaxB ? (long long)B * (long long)(sizeof(PendState) / 4) : 0);
}

int64_t acmi_backward_ws_floats(int B, int A, int C3) {
  Layout L;
  if (!make_layout(A, C3, &L) || B < 0) return -1;
  return std::max(bwd_prefix_floats(B), stats_prefix_floats(B, A)) + bwd_partial_floats(B, A, C3);
}

int acmi_backward(const acmi_net_t* net, const uint8_t* obs, int64_t img_stride, int B,
                  const acmi_acts_t* acts, const acmi_bwd_t* bwd, float* grads,
                  float* a_stats, float* ws, int64_t ws_floats, acmi_stream_t stream) {
  ACMI_REQUIRE(net_modes_ok(net), ACMI_ERR_ARG, "acmi_backward: bad acmi_net_t mode fields");
  const ModeScope mode_scope(net);
  Layout L;
  ACMI_REQUIRE(net && acts && bwd && grads && ws && obs, ACMI_ERR_ARG,
               "acmi_backward: null argument");
  ACMI_REQUIRE(masks_ok(acts), ACMI_ERR_ARG, "acmi_backward: ReLU masks m1..m3 must be all set or all NULL");
  ACMI_REQUIRE(make_layout(net->num_actions, net->conv3_filters, &L), ACMI_ERR_ARG,
               "acmi_backward: bad net");
  ACMI_REQUIRE(B > 0 && img_stride >= 84 * 84 * 4 && img_stride % 4 == 0, ACMI_ERR_ARG,
               "acmi_backward: bad B / img_stride");
  ACMI_REQUIRE(bwd->ldh >= net->num_actions + 1 && bwd->ldh % 4 == 0, ACMI_ERR_ARG,
               "acmi_backward: ldh must be >= A+1 and a multiple of 4 (zero padded)");
  ACMI_REQUIRE(spans32(B, img_stride, 84 * 84 * 4) && spans32(B, 400 * 32, 400 * 32), ACMI_ERR_ARG,
               "acmi_backward: batch spans >= 2^31 elements (B=%d)", B);
  const long long need = acmi_backward_ws_floats(B, net->num_actions, net->conv3_filters);
  ACMI_REQUIRE(ws_floats >= need, ACMI_ERR_WS, "acmi_backward: workspace of %lld floats < %lld",
               (long long)ws_floats, need);
  hipStream_t s = (hipStream_t)stream;
  if (L.C3 == 32)
    return backward_impl<32>(L, net->params, obs, img_stride, B, acts, bwd, grads, a_stats, ws,
                             ws_floats, s, static_cast<const char*>(net->conv_prep));
  return backward_impl<64>(L, net->params, obs, img_stride, B, acts, bwd, grads, a_stats, ws,
                           ws_floats, s, static_cast<const char*>(net->conv_prep));
}

int acmi_backward_stacked(const acmi_net_t* net, const uint8_t* obs, int64_t img_stride, int B,
                          const acmi_acts_t* acts, const acmi_bwd_t* bwd, float* grads, float* a_stats,
                          float* ws, int64_t ws_floats, const acmi_bwd_t* bwd_s, uint32_t seed,
                          uint32_t row_offset, uint32_t counter, float* ws_s, int64_t ws_s_floats,
                          acmi_stream_t stream) {
  ACMI_REQUIRE(net_modes_ok(net), ACMI_ERR_ARG, "acmi_backward_stacked: bad acmi_net_t mode fields");
  const ModeScope mode_scope(net);
  Layout L;
  ACMI_REQUIRE(net && acts && bwd && bwd_s && grads && a_stats && ws && ws_s && obs, ACMI_ERR_ARG,
               "acmi_backward_stacked: null argument");
  ACMI_REQUIRE(masks_ok(acts), ACMI_ERR_ARG, "acmi_backward_stacked: ReLU masks m1..m3 must be all set or all NULL");
  ACMI_REQUIRE(make_layout(net->num_actions, net->conv3_filters, &L), ACMI_ERR_ARG, "acmi_backward_stacked: bad net");
  ACMI_REQUIRE(B > 0 && img_stride >= 84 * 84 * 4 && img_stride % 4 == 0, ACMI_ERR_ARG,
               "acmi_backward_stacked: bad B / img_stride");
  ACMI_REQUIRE(bwd->ldh >= net->num_actions + 1 && bwd->ldh % 4 == 0, ACMI_ERR_ARG,
               "acmi_backward_stacked: ldh must be >= A+1 and a multiple of 4 (zero padded)");
  ACMI_REQUIRE(spans32(B, img_stride, 84 * 84 * 4) && spans32(B, 400 * 32, 400 * 32), ACMI_ERR_ARG,
               "acmi_backward_stacked: batch spans >= 2^31 elements (B=%d)", B);
  ACMI_REQUIRE(ws != ws_s && bwd->d1 != bwd_s->d1 && bwd->d2 != bwd_s->d2 && bwd->d3 != bwd_s->d3 &&
                   bwd->d4 != bwd_s->d4,
               ACMI_ERR_ARG, "acmi_backward_stacked: the two chains need their own workspaces and d1..d4");
  const long long need = acmi_backward_ws_floats(B, net->num_actions, net->conv3_filters);
  ACMI_REQUIRE(ws_floats >= need && ws_s_floats >= need, ACMI_ERR_WS,
               "acmi_backward_stacked: workspaces of %lld / %lld floats < %lld", (long long)ws_floats,
               (long long)ws_s_floats, need);
  hipStream_t s = (hipStream_t)stream;
  const char* prep = static_cast<const char*>(net->conv_prep);
  if (L.C3 == 32)
    return backward_stacked_impl<32>(L, net->params, obs, img_stride, B, acts, bwd, grads, a_stats, ws, ws_floats,
                                     bwd_s, seed, row_offset, counter, ws_s, ws_s_floats, s, prep);
  return backward_stacked_impl<64>(L, net->params, obs, img_stride, B, acts, bwd, grads, a_stats, ws, ws_floats,
                                   bwd_s, seed, row_offset, counter, ws_s, ws_s_floats, s, prep);
}

int acmi_kfac_output_stats_finish(const acmi_net_t* net, int B, const acmi_acts_t* acts, const acmi_bwd_t* bwd_s,
                                  float* g_stats, float* ws_s, int64_t ws_s_floats, acmi_stream_t stream) {
  ACMI_REQUIRE(net_modes_ok(net), ACMI_ERR_ARG, "acmi_kfac_output_stats_finish: bad acmi_net_t mode fields");
  const ModeScope mode_scope(net);
  Layout L;
  ACMI_REQUIRE(net && acts && bwd_s && g_stats && ws_s, ACMI_ERR_ARG, "acmi_kfac_output_stats_finish: null argument");
  ACMI_REQUIRE(make_layout(net->num_actions, net->conv3_filters, &L), ACMI_ERR_ARG, "bad net");
  ACMI_REQUIRE(B > 0 && spans32(B, 400 * 32, 400 * 32), ACMI_ERR_ARG, "bad B");
  const long long need = acmi_backward_ws_floats(B, net->num_actions, net->conv3_filters);
  ACMI_REQUIRE(ws_s_floats >= need, ACMI_ERR_WS, "acmi_kfac_output_stats_finish: workspace of %lld floats < %lld",
               (long long)ws_s_floats, need);
  hipStream_t s = (hipStream_t)stream;
  const char* prep = static_cast<const char*>(net->conv_prep);
  if (L.C3 == 32)
    return output_stats_impl<32>(L, net->params, B, acts, bwd_s, 0, 0, 0, g_stats, ws_s, ws_s_floats, s, prep, 2);
  return output_stats_impl<64>(L, net->params, B, acts, bwd_s, 0, 0, 0, g_stats, ws_s, ws_s_floats, s, prep, 2);
}

int acmi_stream_wait_backward_dx(acmi_stream_t stream) {
  hipEvent_t* ev = dx_done_event();
  ACMI_REQUIRE(ev && hipStreamWaitEvent((hipStream_t)stream, *ev, 0) == hipSuccess, ACMI_ERR_HIP,
               "acmi_stream_wait_backward_dx failed");
  return ACMI_OK;
}

int acmi_kfac_output_stats(const acmi_net_t* net, int B, const acmi_acts_t* acts,
                           const acmi_bwd_t* bwd, uint32_t seed, uint32_t row_offset,
                           uint32_t counter, float* g_stats, float* ws, int64_t ws_floats,
                           acmi_stream_t stream) {
  ACMI_REQUIRE(net_modes_ok(net), ACMI_ERR_ARG, "acmi_kfac_output_stats: bad acmi_net_t mode fields");
  const ModeScope mode_scope(net);
  Layout L;
  ACMI_REQUIRE(net && acts && bwd && g_stats && ws, ACMI_ERR_ARG,
               "acmi_kfac_output_stats: null argument");
  ACMI_REQUIRE(make_layout(net->num_actions, net->conv3_filters, &L), ACMI_ERR_ARG, "bad net");
  ACMI_REQUIRE(B > 0 && spans32(B, 400 * 32, 400 * 32), ACMI_ERR_ARG, "bad B");
  ACMI_REQUIRE(masks_ok(acts), ACMI_ERR_ARG, "acmi_kfac_output_stats: ReLU masks m1..m3 must be all set or all NULL");
  const long long need = acmi_backward_ws_floats(B, net->num_actions, net->conv3_filters);
  ACMI_REQUIRE(ws_floats >= need, ACMI_ERR_WS, "acmi_kfac_output_stats: workspace of %lld floats < %lld",
               (long long)ws_floats, need);
  hipStream_t s = (hipStream_t)stream;
  if (L.C3 == 32)
    return output_stats_impl<32>(L, net->params, B, acts, bwd, seed, row_offset, counter,
                                 g_stats, ws, ws_floats, s, static_cast<const char*>(net->conv_prep));
  return output_stats_impl<64>(L, net->params, B, acts, bwd, seed, row_offset, counter, g_stats,
                               ws, ws_floats, s, static_cast<const char*>(net->conv_prep));
}

int acmi_prof_enable(int site, int capacity) {
  ACMI_REQUIRE(site >= 0 && capacity >= 0 && capacity <= 65536, ACMI_ERR_ARG,
               "acmi_prof_enable: bad site/capacity");
  if (g_prof_ev) {
    for (int i = 0; i < 2 * g_prof_cap; ++i) (void)hipEventDestroy(g_prof_ev[i]);
    delete[] g_prof_ev;
    g_prof_ev = nullptr;
  }
  g_prof_site = 0;
  g_prof_cap = 0;
  g_prof_n = 0;
  if (site == 0 || capacity == 0) return ACMI_OK;
  g_prof_ev = new hipEvent_t[2 * capacity];
  for (int i = 0; i < 2 * capacity; ++i) {
    if (hipEventCreate(&g_prof_ev[i]) != hipSuccess) {
      set_error("acmi_prof_enable: hipEventCreate failed");
      return ACMI_ERR_HIP;
    }
  }
  g_prof_site = site;
  g_prof_cap = capacity;
  return ACMI_OK;
}

int acmi_prof_collect(double* total_ms, int* count) {
  ACMI_REQUIRE(total_ms && count, ACMI_ERR_ARG, "acmi_prof_collect: null argument");
  double t = 0.0;
  for (int i = 0; i < g_prof_n; ++i) {
    if (hipEventSynchronize(g_prof_ev[2 * i + 1]) != hipSuccess) {
      set_error("acmi_prof_collect: hipEventSynchronize failed");
      return ACMI_ERR_HIP;
    }
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, g_prof_ev[2 * i], g_prof_ev[2 * i + 1]);
    t += ms;
  }
  *total_ms = t;
  *count = g_prof_n;
  g_prof_n = 0;
  return ACMI_OK;
}

// Host-only check of the launch planners (no GPU): every sub-tile of the
// upper triangle of P^T P and every (P, dY) sub-tile is produced by sym_plan's
// groups, each column's sum by exactly one wave, for K = 64..max_k; and
// plan_rounds' chunks cover the rows exactly.  0 = ok, else the failing K.
int acmi_debug_convt2(const acmi_net_t* net, int mode, const float* d2a, const float* d2b, const uint32_t* m1,
                      float* d1, int B, float* gram_part, const uint32_t* d2max_a, const uint32_t* d2max_b,
                      uint32_t* d1max, acmi_stream_t stream) {
  ACMI_REQUIRE(net_modes_ok(net), ACMI_ERR_ARG, "acmi_debug_convt2: bad acmi_net_t mode fields");
  const ModeScope mode_scope(net);
  ACMI_REQUIRE(net && net->conv_prep && d2a && d2b && m1 && d1 && gram_part && d2max_a && d2max_b && d1max && B > 0,
               ACMI_ERR_ARG, "acmi_debug_convt2: bad arguments");
  const char* p2 = static_cast<const char*>(net->conv_prep) +
                   (net->conv3_filters == 32 ? TowerPrep<32>::BYTES : TowerPrep<64>::BYTES);
  hipStream_t s = (hipStream_t)stream;
  const float* act1 = reinterpret_cast<const float*>(m1);
  if (mode == 0) {
    hipLaunchKernelGGL((convt2_kernel<false, true>), dim3(convt2_store_blocks(B)), dim3(256), 0, s, p2, d2a, act1, d1,
                       B, nullptr, d2max_a, d1max, nullptr, nullptr);
    hipLaunchKernelGGL((convt2_kernel<true, true>), dim3(convt2_gram_blocks(B)), dim3(256), 0, s, p2, d2b, act1,
                       nullptr, B, gram_part, d2max_b, nullptr, nullptr, nullptr);
  } else {
    hipLaunchKernelGGL((convt2_kernel<true, true, true>), dim3(convt2_gram_blocks(B)), dim3(256), 0, s, p2, d2a,
                       act1, d1, B, gram_part, d2max_a, d1max, d2b, d2max_b);
  }
  ACMI_LAUNCH_CHECK("acmi_debug_convt2");
  return ACMI_OK;
}

int acmi_debug_ws_flushes(void) {
  const int n = g_ws_flushes;
  g_ws_flushes = 0;
  return n;
}

int acmi_selftest_plans(int max_k) {
  for (int K = 64; K <= max_k; K += 32) {
    SymPlan p;
    if (!sym_plan(K, 64, &p)) continue;  // shape falls back to the 128x128 tiles
    const int J = K + 64;
    std::vector<unsigned char> cov((size_t)K * J, 0);
    std::vector<int> cs(J, 0);
    for (int g = 0; g < p.ngroups; ++g)
      for (int w = 0; w < 4; ++w) {
        if (p.g[g].wa[w] < 0) continue;
        const int a = p.g[g].base[p.g[g].wa[w]], b = p.g[g].base[p.g[g].wb[w]];
        if (a < 0 || b < 0 || a >= K) return K;
        for (int i = a; i < a + 64 && i < K; ++i)
          for (int j = b; j < b + 64 && j < J; ++j) cov[(size_t)i * J + j] = 1;
        if (a == 0)
          for (int j = b; j < b + 64 && j < J; ++j) cs[j]++;
      }
    for (int i = 0; i < K; ++i)
      for (int j = i; j < J; ++j)
        if (!cov[(size_t)i * J + j]) return K;
    for (int j = 0; j < J; ++j)
      if (cs[j] < 1) return K;
  }
  // six-slab groups (symred6_kernel): every needed sub-tile exactly once, at
  // most 16 per group and 2 per wave, each column's sum by exactly one wave
  for (int K : {512, 576})
    for (int cp : {8, 32, 64}) {
      SymPlan6 p;
      if (!sym_plan6(K, cp, &p)) return -(K + cp);
      const int nb = K / 64;
      std::vector<int> cov((size_t)(nb + 1) * (nb + 1), 0), cs(nb + 1, 0);
      for (int g = 0; g < p.ngroups; ++g) {
        int n = 0;
        for (int w = 0; w < 8; ++w)
          for (int t = 0; t < 2; ++t) {
            const int ra = p.g[g].ra[w][t], cb = p.g[g].cb[w][t];
            if (ra < 0) {
              if (t == 0 && p.g[g].ra[w][1] >= 0) return -(K + cp);  // tile 1 without tile 0
              continue;
            }
            ++n;
            const int a = p.g[g].base[ra], b = p.g[g].base[cb];
            if (a < 0 || b < 0 || a % 64 || a >= K || b < a) return -(K + cp);
            cov[(size_t)(a / 64) * (nb + 1) + b / 64]++;
            if (a == 0) cs[b / 64]++;
            // a half-width (dY) tile in slot 0 needs slot 1 half as well (kernel variants)
            if (t == 1 && p.g[g].base[p.g[g].cb[w][0]] == K && b != K) return -(K + cp);
          }
        if (n > 16) return -(K + cp);
      }
      for (int a = 0; a < nb; ++a)
        for (int b = a; b <= nb; ++b)
          if (cov[(size_t)a * (nb + 1) + b] != 1) return -(K + cp);
      for (int b = 0; b <= nb; ++b)
        if (cs[b] != 1) return -(K + cp);
    }
  // greedy six-slab groups (fc4 and the other K): every needed sub-tile exactly once,
  // at most 16 per group, a half-width tile never in slot 0 under a full one, each
  // column slab's sum by exactly one (0, b) tile
  for (int K : {1568, 512, 576})
    for (int cp : {512, 64, 8}) {
      SymPlan6 p;
      if (!sym_plan6_greedy(K, cp, &p)) return -(K + cp + 1);
      const int J = K + cp, ns = (J + 63) / 64, nbp = (K + 63) / 64;
      std::vector<int> cov((size_t)ns * ns, 0), cs(ns, 0);
      for (int g = 0; g < p.ngroups; ++g) {
        int n = 0;
        for (int w = 0; w < 8; ++w) {
          bool half0 = false;
          for (int t = 0; t < 2; ++t) {
            const int ra = p.g[g].ra[w][t], cb = p.g[g].cb[w][t];
            if (ra < 0) {
              if (t == 0 && p.g[g].ra[w][1] >= 0) return -(K + cp + 1);
              continue;
            }
            ++n;
            const int a = p.g[g].base[ra], b = p.g[g].base[cb];
            const bool half = b + 32 >= J;
            if (t == 0) half0 = half;
            else if (half0 && !half) return -(K + cp + 1);
            if (a % 64 || b % 64 || a >= K || b < a || b >= J) return -(K + cp + 1);
            cov[(size_t)(a / 64) * ns + b / 64]++;
            if (a == 0) cs[b / 64]++;
          }
        }
        if (n > 16) return -(K + cp + 1);
      }
      for (int a = 0; a < nbp; ++a)
        for (int b = a; b < ns; ++b)
          if (cov[(size_t)a * ns + b] != 1) return -(K + cp + 1);
      for (int b = 0; b < ns; ++b)
        if (cs[b] != 1) return -(K + cp + 1);
    }
  for (long long rows : {1000LL, 4096000LL, 829440LL, 501760LL, 10240LL}) {
    for (int live : {1, 3, 11, 14, 90}) {
      int nc, ch;
      plan_rounds(rows, live, 1024, &nc, &ch);
      if (ch % 32 != 0 || (long long)nc * ch < rows || (long long)(nc - 1) * ch >= rows) return -1;
    }
  }
  // band plans (conv2, conv3 at C3 = 32 / 64): exact cover, column-sum owners,
  // and the fold tables reproduce the patch-row sums (host emulation in double)
  const int bshape[3][7] = {{20, 20, 32, 4, 4, 2, 64}, {9, 9, 64, 3, 3, 1, 32}, {9, 9, 64, 3, 3, 1, 64}};
  for (int i = 0; i < 3; ++i) {
    const int* b = bshape[i];
    const BandPlan* p = band_host_plan(b[0], b[1], b[2], b[3], b[4], b[5], b[6]);
    if (!p || band_plan_check(*p) != 0 || band_plan_emulate(*p) > 1e-12) return -(1000 + i);
    for (long long rows : {1LL, 37LL, 10240LL, 20480LL}) {
      int nc, ch;
      band_chunks(rows, (int)p->groups.size(), &nc, &ch);
      if (ch % 16 != 0 || (long long)nc * ch < rows || (long long)(nc - 1) * ch >= rows) return -(1010 + i);
    }
  }
  return 0;
}

int acmi_gemm_f32(const float* A, const float* B, float* C, int M, int N, int K,
                  acmi_stream_t stream) {
  ACMI_REQUIRE(A && B && C && M > 0 && N > 0 && K > 0 && K % 4 == 0 && N % 4 == 0,
               ACMI_ERR_ARG, "acmi_gemm_f32: need K%%4==0, N%%4==0");
  RowsAsK<DenseRows> opA{DenseRows{A, K, M, K}};
  MatI<true> opB{B, N, K, N};
  EpiStore epi{C, N};
  launch_gemm<128, 128, 32, 2, 2, false, false>(opA, opB, epi, M, N, K, 1, 0,
                                                (hipStream_t)stream);
  ACMI_LAUNCH_CHECK("acmi_gemm_f32");
  return ACMI_OK;
}

}  // extern "C"
