// Device pieces shared by the rollout kernels: the batched synthetic Atari
// stepper (multi_env.py:121-137 + wrappers.py:201-235 + wrappers.py:263-323)
// and categorical sampling (policies.py:86-87), used by the standalone kernels
// in rl.hip and by the fused rollout tail in net.hip.
#pragma once

#include "common.hpp"

namespace acmi {

constexpr int FRAME_WORDS = 84 * 84 / 4;
constexpr uint32_t RESET_TAG = 0xFFFFFFFFu;
constexpr uint32_t LEN_TAG = 0xFFFFFFFEu;
constexpr uint32_t REW_SALT = 0x85EBCA6Bu;
constexpr uint32_t REW_LO = 838861u;      // round(0.05 * 2^24)
constexpr uint32_t REW_HI = 15938355u;    // 2^24 - REW_LO

__device__ __forceinline__ uint32_t word_hash(uint32_t base, uint32_t g) {
  return mix32(base ^ (g * 0x9E3779B9u));
}
__device__ __forceinline__ int32_t episode_length(uint32_t seed, uint32_t e, uint32_t k) {
  return 50 + (int32_t)(key4(seed, e, k, LEN_TAG) % 451u);
}

// One env step for env n (global id e) by a whole 256-thread workgroup: reads
// the pre-step state, lazily auto-resets, writes the next 4-frame stack,
// reward, terminal and episode total.  Contains a __syncthreads (every thread
// of the block must call it).  The previous stack's words are loaded first,
// all kEnvWords of a thread at once (env_prefetch: they do not depend on the
// action, so the fused rollout tail issues them before its head arithmetic);
// a load per loop iteration would wait out one memory latency per iteration.
constexpr int kEnvThreads = 256;
constexpr int kEnvWords = (FRAME_WORDS + kEnvThreads - 1) / kEnvThreads;  // 7

struct EnvPre {  // an env's pre-step state and current stack words, loaded up front
  uint4 old[kEnvWords];
  int32_t k, t, L;
  float total;
  bool was_done;
};

__device__ __forceinline__ void env_prefetch(acmi_env_state_t st, int n, const uint8_t* obs_in, EnvPre& p) {
  const uint4* in = reinterpret_cast<const uint4*>(obs_in);
#pragma unroll
  for (int i = 0; i < kEnvWords; ++i) {
    const int g = threadIdx.x + kEnvThreads * i;
    p.old[i] = in[g < FRAME_WORDS ? g : 0];
  }
  p.was_done = st.done[n] != 0;
  p.k = st.episode[n];
  p.t = st.step[n];
  p.L = st.length[n];
  p.total = st.total[n];
}

// (the state of env n must have been read by every thread -- env_prefetch --
// before this is called: it begins with the barrier that orders those reads
// before thread 0's state writes)
__device__ __forceinline__ void env_step_block_pre(acmi_env_state_t st, int n, uint32_t e, uint32_t seed,
                                                   uint32_t action, const EnvPre& pre,
                                                   uint8_t* obs_out, float* rewards,
                                                   uint8_t* terminals, float* ep_rewards,
                                                   long long ld) {
  const bool was_done = pre.was_done;
  int32_t k = pre.k;
  int32_t t = pre.t;
  int32_t L = pre.L;
  float total = pre.total;
  __syncthreads();
  if (was_done) {  // _AutoResetWrapper: reset lazily at the next step
    k += 1;
    t = 0;
    L = episode_length(seed, e, (uint32_t)k);
    total = 0.f;
  }
  t += 1;
  const uint32_t a = action & 255u;
  const uint32_t base = key4(seed, e, (uint32_t)k, (uint32_t)t * 256u + a);
  const uint32_t rh = mix32(base ^ REW_SALT) >> 8;
  const float rew = rh < REW_LO ? -1.f : (rh >= REW_HI ? 1.f : 0.f);
  const bool term = t >= L;
  const uint32_t rbase = key4(seed, e, (uint32_t)k, RESET_TAG);
  uint4* out = reinterpret_cast<uint4*>(obs_out);
#pragma unroll
  for (int i = 0; i < kEnvWords; ++i) {
    const int g = threadIdx.x + kEnvThreads * i;
    if (g >= FRAME_WORDS) break;
    uint4 old = pre.old[i];
    if (was_done) {  // FrameStackWrapper.reset: the reset frame repeated 4x
      const uint32_t w = word_hash(rbase, (uint32_t)g);
      old.x = (w & 255u) * 0x01010101u;
      old.y = ((w >> 8) & 255u) * 0x01010101u;
      old.z = ((w >> 16) & 255u) * 0x01010101u;
      old.w = (w >> 24) * 0x01010101u;
    }
    const uint32_t f = word_hash(base, (uint32_t)g);
    // np.roll(stack, -1, axis=-1); zero-fill on terminal; last channel = frame
    uint4 o;
    o.x = (term ? 0u : (old.x >> 8)) | ((f & 255u) << 24);
    o.y = (term ? 0u : (old.y >> 8)) | (((f >> 8) & 255u) << 24);
    o.z = (term ? 0u : (old.z >> 8)) | (((f >> 16) & 255u) << 24);
    o.w = (term ? 0u : (old.w >> 8)) | ((f >> 24) << 24);
    out[g] = o;
  }
  if (threadIdx.x == 0) {
    total += rew;
    rewards[n * ld] = rew;
    terminals[n * ld] = term ? 1 : 0;
    ep_rewards[n * ld] = term ? total : __int_as_float(0x7fc00000);
    st.episode[n] = k;
    st.step[n] = t;
    st.length[n] = L;
    st.total[n] = term ? 0.f : total;
    st.done[n] = term ? 1 : 0;
  }
}

__device__ __forceinline__ void env_step_block(acmi_env_state_t st, int n, uint32_t e, uint32_t seed,
                                               uint32_t action, const uint8_t* obs_in,
                                               uint8_t* obs_out, float* rewards,
                                               uint8_t* terminals, float* ep_rewards,
                                               long long ld) {
  EnvPre pre;
  env_prefetch(st, n, obs_in, pre);
  env_step_block_pre(st, n, e, seed, action, pre, obs_out, rewards, terminals, ep_rewards, ld);
}

// Categorical draw over the A logits z[0..A) (inverse CDF of softmax in f32
// with u = u01(key4(seed, sid, ctr, row)) or the given u); -1 for a row with a
// non-finite logit (*bad_flag set).  mode: argmax.
__device__ __forceinline__ int sample_row(const float* z, int A, uint32_t seed, uint32_t sid,
                                          uint32_t ctr, uint32_t row, const float* u_given,
                                          int mode, bool* bad_flag) {
  float mx = -INFINITY;
  bool finite = true;
  int amax = 0;
  for (int a = 0; a < A; ++a) {
    const float v = z[a];
    finite = finite && isfinite(v);
    if (v > mx) { mx = v; amax = a; }
  }
  *bad_flag = !finite;
  if (!finite) return -1;
  if (mode) return amax;  // first maximal index, like argmax
  float se = 0.f;
  for (int a = 0; a < A; ++a) se += expf(z[a] - mx);
  const float u = u_given ? *u_given : u01(key4(seed, sid, ctr, row));
  const float target = u * se;
  float c = 0.f;
  int y = A - 1;
  for (int a = 0; a < A; ++a) {
    c += expf(z[a] - mx);
    if (target < c) { y = a; break; }
  }
  return y;
}

}  // namespace acmi
