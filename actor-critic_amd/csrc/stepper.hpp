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

// One env step for env n (global id e) by a whole workgroup: reads the
// pre-step state, lazily auto-resets, writes the next 4-frame stack, reward,
// terminal and episode total.  Contains a __syncthreads (every thread of the
// block must call it).
__device__ __forceinline__ void env_step_block(acmi_env_state_t st, int n, uint32_t e, uint32_t seed,
                                               uint32_t action, const uint8_t* obs_in,
                                               uint8_t* obs_out, float* rewards,
                                               uint8_t* terminals, float* ep_rewards,
                                               long long ld) {
  // every thread reads the (pre-step) state, then a barrier before thread 0
  // writes the new state
  const bool was_done = st.done[n] != 0;
  int32_t k = st.episode[n];
  int32_t t = st.step[n];
  int32_t L = st.length[n];
  float total = st.total[n];
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
  const uint4* in = reinterpret_cast<const uint4*>(obs_in);
  uint4* out = reinterpret_cast<uint4*>(obs_out);
  for (int g = threadIdx.x; g < FRAME_WORDS; g += blockDim.x) {
    uint4 old;
    if (was_done) {  // FrameStackWrapper.reset: the reset frame repeated 4x
      const uint32_t w = word_hash(rbase, (uint32_t)g);
      old.x = (w & 255u) * 0x01010101u;
      old.y = ((w >> 8) & 255u) * 0x01010101u;
      old.z = ((w >> 16) & 255u) * 0x01010101u;
      old.w = (w >> 24) * 0x01010101u;
    } else {
      old = in[g];
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
