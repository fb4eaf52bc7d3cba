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

// Mixed-game synthetic Atari-57 (BASELINE configs[4]; the reference's MultiEnv
// holds one game, multi_env.py:36-47).  Env n plays game st.game[n] (index into
// the Atari-57 list, wrappers.ATARI57); a null game array = every env the
// default game (Breakout's dynamics, no action masking).  A game fixes its
// dynamics salt (XORed into the seed: its own frames, rewards and lengths), its
// episode-length range, its +-1 reward rates and its legal-action count under
// the full 18-action set (actions past it act as NOOP, as in ALE).  Breakout's
// entry is the default game's dynamics.  Restated in oracle.game_params.
constexpr int kNumGames = 57;
constexpr int kGameBreakout = 12;
__constant__ uint8_t kGameActions[kNumGames] = {
    18, 10, 7, 9, 14, 4, 18, 18, 9, 18, 6, 18, 4, 18, 18, 9, 18, 6, 18, 9,
    18, 3, 18, 8, 18, 18, 18, 18, 18, 18, 14, 18, 9, 6, 8, 18, 6, 18, 6, 18,
    18, 18, 18, 3, 18, 6, 18, 5, 18, 10, 8, 6, 18, 9, 10, 18, 18};

struct GameParams {
  uint32_t salt, len_min, len_span, rew_lo, rew_hi, n_legal;
};

__device__ __forceinline__ GameParams game_params(int g) {  // g < 0: the default game
  GameParams p{0u, 50u, 451u, REW_LO, REW_HI, 256u};
  if (g < 0 || g == kGameBreakout) {
    if (g == kGameBreakout) p.n_legal = 4u;
    return p;
  }
  const uint32_t h = mix32(0x47414D45u ^ ((uint32_t)g * 0x9E3779B9u));
  const uint32_t h2 = mix32(h), h3 = mix32(h2);
  p.salt = h | 1u;
  p.len_min = 30u + h2 % 171u;          // 30 .. 200
  p.len_span = 100u + (h2 >> 8) % 1901u;  // episodes up to ~2100 steps
  p.rew_lo = (uint32_t)(((uint64_t)(h3 & 0xFFFFu) * 838861u) >> 16);  // P(-1) in [0, 0.05)
  p.rew_hi = 16777216u - 83886u - (uint32_t)(((uint64_t)(h3 >> 16) * (3355443u - 83886u)) >> 16);  // P(+1) in (0.005, 0.2]
  p.n_legal = kGameActions[g];
  return p;
}
__device__ __forceinline__ int env_game(acmi_env_state_t st, int n) { return st.game ? (int)st.game[n] : -1; }

__device__ __forceinline__ int32_t episode_length(uint32_t seed, uint32_t e, uint32_t k,
                                                  const GameParams& gp) {
  return (int32_t)(gp.len_min + key4(seed ^ gp.salt, e, k, LEN_TAG) % gp.len_span);
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
  int game;
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
  p.game = env_game(st, n);
}

// (the state of env n must have been read by every thread -- env_prefetch --
// before this is called: it begins with the barrier that orders those reads
// before thread 0's state writes)
// mirror (nullable): the new stack is also stored there, 16-byte word g at
// mirror[g] (the fused rollout tail hands it to the next step's conv tower in LDS)
__device__ __forceinline__ void env_step_block_pre(acmi_env_state_t st, int n, uint32_t e, uint32_t seed,
                                                   uint32_t action, const EnvPre& pre,
                                                   uint8_t* obs_out, float* rewards,
                                                   uint8_t* terminals, float* ep_rewards,
                                                   long long ld, uint4* mirror = nullptr) {
  const bool was_done = pre.was_done;
  int32_t k = pre.k;
  int32_t t = pre.t;
  int32_t L = pre.L;
  float total = pre.total;
  const GameParams gp = game_params(pre.game);
  __syncthreads();
  if (was_done) {  // _AutoResetWrapper: reset lazily at the next step
    k += 1;
    t = 0;
    L = episode_length(seed, e, (uint32_t)k, gp);
    total = 0.f;
  }
  t += 1;
  const uint32_t a = (action & 255u) < gp.n_legal ? (action & 255u) : 0u;  // illegal: NOOP
  const uint32_t gseed = seed ^ gp.salt;
  const uint32_t base = key4(gseed, e, (uint32_t)k, (uint32_t)t * 256u + a);
  const uint32_t rh = mix32(base ^ REW_SALT) >> 8;
  const float rew = rh < gp.rew_lo ? -1.f : (rh >= gp.rew_hi ? 1.f : 0.f);
  const bool term = t >= L;
  const uint32_t rbase = key4(gseed, e, (uint32_t)k, RESET_TAG);
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
    if (mirror) mirror[g] = o;
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

// The env step of one of several workgroups sharing env n (the split rollout
// step, towersplit.hpp): every one reads the pre-step state (nobody writes it
// during the launch), builds the new stack's 16-byte words [g0, g1) into `mirror`
// (its LDS image, word g at mirror[g]) and files words [o0, o1) into obs_out
// (the owners partition the stack); the writer also stores the reward, terminal
// and episode total and the post-step state into pend[0..5] with pend[5] = 1
// (committed into st by the next step's fc4 launch, env_commit_pending: a part
// that started late could otherwise read a state another part already advanced).
// The arithmetic is env_step_block_pre's, word for word.
struct PendState {  // pend[8] per env: episode, step, length, total (bits), done, flag
  int32_t k, t, L, total_bits, done, flag, pad0, pad1;
};
__device__ __forceinline__ void env_step_part(acmi_env_state_t st, int n, uint32_t e, uint32_t seed, uint32_t action,
                                              const uint8_t* obs_in, int g0, int g1, int o0, int o1,
                                              uint8_t* obs_out, uint8_t* obs_copy, uint4* mirror, bool writer,
                                              float* rewards, uint8_t* terminals, float* ep_rewards, long long ld,
                                              PendState* pend) {
  const bool was_done = st.done[n] != 0;
  int32_t k = st.episode[n];
  int32_t t = st.step[n];
  int32_t L = st.length[n];
  float total = st.total[n];
  const GameParams gp = game_params(env_game(st, n));
  if (was_done) {
    k += 1;
    t = 0;
    L = episode_length(seed, e, (uint32_t)k, gp);
    total = 0.f;
  }
  t += 1;
  const uint32_t a = (action & 255u) < gp.n_legal ? (action & 255u) : 0u;
  const uint32_t gseed = seed ^ gp.salt;
  const uint32_t base = key4(gseed, e, (uint32_t)k, (uint32_t)t * 256u + a);
  const uint32_t rh = mix32(base ^ REW_SALT) >> 8;
  const float rew = rh < gp.rew_lo ? -1.f : (rh >= gp.rew_hi ? 1.f : 0.f);
  const bool term = t >= L;
  const uint32_t rbase = key4(gseed, e, (uint32_t)k, RESET_TAG);
  const uint4* in = reinterpret_cast<const uint4*>(obs_in);
  uint4* out = reinterpret_cast<uint4*>(obs_out);
  constexpr int NW = (36 * 21 + kEnvThreads - 1) / kEnvThreads;  // a part's range: <= 36 rows of 21 words
  uint4 old[NW];
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const int g = g0 + (int)threadIdx.x + kEnvThreads * i;
    old[i] = in[g < g1 ? g : g0];
  }
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const int g = g0 + (int)threadIdx.x + kEnvThreads * i;
    if (g >= g1) break;
    uint4 ow = old[i];
    if (obs_copy && g >= o0 && g < o1) reinterpret_cast<uint4*>(obs_copy)[g] = ow;
    if (was_done) {
      const uint32_t w = word_hash(rbase, (uint32_t)g);
      ow.x = (w & 255u) * 0x01010101u;
      ow.y = ((w >> 8) & 255u) * 0x01010101u;
      ow.z = ((w >> 16) & 255u) * 0x01010101u;
      ow.w = (w >> 24) * 0x01010101u;
    }
    const uint32_t f = word_hash(base, (uint32_t)g);
    uint4 o;
    o.x = (term ? 0u : (ow.x >> 8)) | ((f & 255u) << 24);
    o.y = (term ? 0u : (ow.y >> 8)) | (((f >> 8) & 255u) << 24);
    o.z = (term ? 0u : (ow.z >> 8)) | (((f >> 16) & 255u) << 24);
    o.w = (term ? 0u : (ow.w >> 8)) | ((f >> 24) << 24);
    mirror[g] = o;
    if (g >= o0 && g < o1) out[g] = o;
  }
  if (writer && threadIdx.x == 0) {
    total += rew;
    rewards[n * ld] = rew;
    terminals[n * ld] = term ? 1 : 0;
    ep_rewards[n * ld] = term ? total : __int_as_float(0x7fc00000);
    PendState ps;
    ps.k = k;
    ps.t = t;
    ps.L = L;
    ps.total_bits = __float_as_int(term ? 0.f : total);
    ps.done = term ? 1 : 0;
    ps.flag = 1;
    ps.pad0 = ps.pad1 = 0;
    pend[n] = ps;
  }
}
// the pending post-step states of envs 0 .. B-1 into st (one thread per env)
__device__ __forceinline__ void env_commit_pending(acmi_env_state_t st, PendState* pend, int B) {
  for (int n = threadIdx.x; n < B; n += blockDim.x) {
    const PendState ps = pend[n];
    if (!ps.flag) continue;
    st.episode[n] = ps.k;
    st.step[n] = ps.t;
    st.length[n] = ps.L;
    st.total[n] = __int_as_float(ps.total_bits);
    st.done[n] = ps.done;
    pend[n].flag = 0;
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
