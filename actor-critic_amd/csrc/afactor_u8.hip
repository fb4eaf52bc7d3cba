// conv1 K-FAC input factor from the raw u8 observations, in exact integer
// arithmetic on the i8 matrix cores.
//
// The conv1 A factor is A = mean_r [p;1][p;1]^T over every conv1 location r,
// p = the 8x8x4 patch of u/255 (envs/atari/model.py:92-95, :227-229).  With
// x = u - 128 in [-128, 127] (one XOR 0x80 per byte):
//     sum_r u_a u_b = sum_r x_a x_b + 128 (Sx_a + Sx_b) + 128^2 R,
//     Sx_a = sum_r x_a,
// so the 256x256 Gram block is an i8 x i8 -> i32 product (v_mfma_i32_32x32x32_i8,
// 2x the bf16 rate, 16x the f32 MFMA rate).  Every partial is an exact integer
// (a 16384-row chunk is < 2^31), chunks are summed in int64, and only the final
// division by 255^2 R rounds — the factor is exact to f32 rounding, tighter than
// the fp32 reference computation.  Only the upper-triangular 128x128 tile pairs
// (0,0), (0,1), (1,1) are computed.
//
// Operand lane map (verified on gfx950, scripts/probes/mfma_i8_probe.hip):
// lane l holds A[row l&31][k = 16(l>>5) + j] and B[k = 16(l>>5) + j][col l&31],
// j = 0..15; D uses the standard 32x32 map.
#include <algorithm>

#include "common.hpp"
#include "symred3.hpp"  // split2, u8x8_to_f16, ds_tr16, cat8h, f16x2 scales (fused conv1 wgrad)

namespace acmi {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int AF_BK = 64;          // rows per stage (two 32-deep MFMA steps)
constexpr int AF_LINE = 80;        // bytes per LDS column line: 64 rows + 16 pad
constexpr int AF_TILE = 128 * AF_LINE;
constexpr int AF_CHUNK = 16384;    // max rows per block: |partial| < 2^31
constexpr int AF_SLOTS = 256 * 4;  // resident blocks (4 per CU by LDS)

// rows < r_end load their patch bytes; the others load this run of 0x80
// bytes, i.e. x = 0 after the XOR (selected on the address, see gemm_ops.hpp)
__device__ __attribute__((weak, aligned(16))) uint32_t kX0Run[4] = {0x80808080u, 0x80808080u,
                                                                    0x80808080u, 0x80808080u};

// chunks: at least ceil(rows / AF_CHUNK), grown so 3 tile pairs x chunks fill
// whole rounds of AF_SLOTS blocks; chunk length a multiple of AF_BK
static void af_plan(long long rows, int* nchunk, int* chunk) {
  const long long nc0 = std::max<long long>(1, (rows + AF_CHUNK - 1) / AF_CHUNK);
  const long long rounds = (3 * nc0 + AF_SLOTS - 1) / AF_SLOTS;
  const long long nc = std::max<long long>(nc0, rounds * AF_SLOTS / 3);
  long long ch = (rows + nc - 1) / nc;
  ch = (ch + AF_BK - 1) / AF_BK * AF_BK;
  *chunk = (int)std::max<long long>(ch, AF_BK);
  *nchunk = (int)((rows + *chunk - 1) / *chunk);
}
constexpr int AF_OBS_W = 84;

__global__ __launch_bounds__(256) void conv1_afactor_i8_kernel(const uint8_t* obs,
                                                               long long img_stride,
                                                               int rows, int chunk_rows,
                                                               int* part, int* colsum) {
  // 1-D grid, XCD-contiguous (gemm.hpp): logical block l = (chunk, pair), the
  // 3 tile pairs of a chunk adjacent, so they read the chunk's frames through
  // one L2
  const int total = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, base_l = total >> 3, rem = total & 7;
  const int l = xcd * base_l + min(xcd, rem) + (b >> 3);
  const int chunk = l / 3;
  const int pair = l - 3 * chunk;  // tile pairs (0,0) (0,1) (1,1)
  const int ta = pair == 2 ? 1 : 0;
  const int tb = pair == 0 ? 0 : 1;
  const bool diag = ta == tb;
  const int r_begin = chunk * chunk_rows;
  const int r_end = min(rows, r_begin + chunk_rows);
  __shared__ __attribute__((aligned(16))) uint8_t lds[2][2][AF_TILE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // staging map: 4 rows (4*q4 .. +3) x 8 columns (8*cg .. +7) per thread
  const int q4 = tid & 15;
  const int cg = tid >> 4;
  // column c = 128 t + 8 cg -> (kh, kw0): 8 bytes = pixels kw0, kw0+1, 4 channels each
  auto col_off = [&](int t) {
    const int c = 128 * t + 8 * cg;
    const int kh = c >> 5;
    const int kw0 = (c & 31) >> 2;
    return (kh * AF_OBS_W + kw0) * 4;
  };
  const int coffA = col_off(ta);
  const int coffB = col_off(tb);

  // raw patch bytes; the XOR (x = u ^ 0x80) is applied at commit, after the
  // MFMAs, so nothing waits on the loads at fetch time.  A thread's 4 rows
  // r .. r+3 (r % 4 == 0: chunks are multiples of 64 rows, every r_end a
  // multiple of 400) are 4 consecutive output columns of ONE output row, i.e.
  // the same patch 16 bytes further on: one row decode per stage, one validity
  // test (the rows are all valid or all past r_end), 32-bit offsets (the host
  // checks the frames span < 2^32 bytes).
  uint2 ra[4], rb[4];
  const uint8_t* x0 = reinterpret_cast<const uint8_t*>(kX0Run);
  const uint32_t istride = (uint32_t)img_stride;
  auto fetch = [&](int r0) {
    const int r = r0 + 4 * q4;
    const bool ok = r < r_end;
    const uint32_t rr = ok ? (uint32_t)r : (uint32_t)r_begin;
    const uint32_t img = rr / 400u;
    const uint32_t p = rr - img * 400u;
    const uint32_t oh = p / 20u;
    const uint32_t ow = p - oh * 20u;
    const uint32_t off = img * istride + (oh * 4 * AF_OBS_W + ow * 4) * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      ra[q] = *reinterpret_cast<const uint2*>(ok ? obs + (off + (uint32_t)(coffA + 16 * q)) : x0);
      if (!diag)
        rb[q] = *reinterpret_cast<const uint2*>(ok ? obs + (off + (uint32_t)(coffB + 16 * q)) : x0);
    }
  };
  // 4 rows x 4 bytes -> 4 column words of 4 consecutive rows (v_perm_b32)
  auto transpose4 = [](uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t* out) {
    const uint32_t p01l = __builtin_amdgcn_perm(w1, w0, 0x05010400u);
    const uint32_t p01h = __builtin_amdgcn_perm(w1, w0, 0x07030602u);
    const uint32_t p23l = __builtin_amdgcn_perm(w3, w2, 0x05010400u);
    const uint32_t p23h = __builtin_amdgcn_perm(w3, w2, 0x07030602u);
    out[0] = __builtin_amdgcn_perm(p23l, p01l, 0x05040100u);
    out[1] = __builtin_amdgcn_perm(p23l, p01l, 0x07060302u);
    out[2] = __builtin_amdgcn_perm(p23h, p01h, 0x05040100u);
    out[3] = __builtin_amdgcn_perm(p23h, p01h, 0x07060302u);
  };
  auto commit = [&](int buf) {
    constexpr uint32_t F = 0x80808080u;
    uint32_t cols[8];
    transpose4(ra[0].x ^ F, ra[1].x ^ F, ra[2].x ^ F, ra[3].x ^ F, cols);
    transpose4(ra[0].y ^ F, ra[1].y ^ F, ra[2].y ^ F, ra[3].y ^ F, cols + 4);
    uint8_t* dst = lds[buf][0];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      *reinterpret_cast<uint32_t*>(dst + (8 * cg + j) * AF_LINE + 4 * q4) = cols[j];
    if (!diag) {
      transpose4(rb[0].x ^ F, rb[1].x ^ F, rb[2].x ^ F, rb[3].x ^ F, cols);
      transpose4(rb[0].y ^ F, rb[1].y ^ F, rb[2].y ^ F, rb[3].y ^ F, cols + 4);
      uint8_t* dstb = lds[buf][1];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        *reinterpret_cast<uint32_t*>(dstb + (8 * cg + j) * AF_LINE + 4 * q4) = cols[j];
    }
  };

  v16i acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0;
  int csum = 0;

  const int nst = r_end > r_begin ? (r_end - r_begin + AF_BK - 1) / AF_BK : 0;
  if (nst > 0) {
    fetch(r_begin);
    commit(0);
  }
  __syncthreads();
  const int half = lane >> 5;
  for (int st = 0; st < nst; ++st) {
    const int cur = st & 1;
    fetch(r_begin + (st + 1) * AF_BK);  // past the chunk: the x = 0 run
    __builtin_amdgcn_sched_barrier(0);
    const uint8_t* As = lds[cur][0];
    const uint8_t* Bs = lds[cur][diag ? 0 : 1];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      v4i a[2], b[2];
#pragma unroll
      for (int tm = 0; tm < 2; ++tm)
        a[tm] = *reinterpret_cast<const v4i*>(As + (64 * wm + 32 * tm + (lane & 31)) * AF_LINE + 32 * s + 16 * half);
#pragma unroll
      for (int tn = 0; tn < 2; ++tn)
        b[tn] = *reinterpret_cast<const v4i*>(Bs + (64 * wn + 32 * tn + (lane & 31)) * AF_LINE + 32 * s + 16 * half);
#pragma unroll
      for (int tm = 0; tm < 2; ++tm)
#pragma unroll
        for (int tn = 0; tn < 2; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[tm], b[tn], acc[tm][tn], 0, 0, 0);
    }
    if (diag && tid < 128) {  // column sums of x over the staged rows
      const uint32_t* line = reinterpret_cast<const uint32_t*>(As + tid * AF_LINE);
#pragma unroll
      for (int w = 0; w < AF_BK / 4; ++w) csum = __builtin_amdgcn_sdot4((int)line[w], 0x01010101, csum, false);
    }
    __builtin_amdgcn_sched_barrier(0);
    commit(cur ^ 1);
    __syncthreads();
  }

  int* out = part + (long long)chunk * 65536;
#pragma unroll
  for (int tm = 0; tm < 2; ++tm)
#pragma unroll
    for (int tn = 0; tn < 2; ++tn) {
      const int col = 128 * tb + 64 * wn + 32 * tn + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = 128 * ta + 64 * wm + 32 * tm + (r & 3) + 8 * (r >> 2) + 4 * half;
        out[row * 256 + col] = acc[tm][tn][r];
      }
    }
  if (diag && tid < 128) colsum[(long long)chunk * 256 + 128 * ta + tid] = csum;
}

// One block per chunk for the whole upper triangle AND the conv1 weight gradient
// (ACMI_GEMM_X3 mode; the 3-block form above stages each row's patch bytes 4
// times over its tile pairs -- 512 bytes per row -- and is bound by that
// gather): all 256 patch columns staged once per 64-row stage (256 bytes per
// row), d1 rows staged beside them, so the u8 gather is shared by the A factor
// and the weight gradient [P;1]^T d1.  Same A partial layout, so
// conv1_afactor_finalize is shared; weight-gradient partials [chunk][257][32]
// (row 256: the bias gradient) reduced by finalize_wgrad_kernel.  Roles (an
// earlier form dealt the 36 A-factor tiles and the 8 weight-gradient tiles to
// all 8 waves, so every wave read the whole split d1 operand -- about 230 KB of
// LDS reads per stage, the column sums 8-way bank conflicted):
//  * waves 0-3 own the A factor on column-block quarters, 9 tiles each: wave 0
//    the upper triangle of blocks 0-3 but (3,3) (from 4 fragments), wave 1 that
//    of blocks 4-7 but (7,7), waves 2 / 3 blocks 0-3 x 4-5 / 6-7 plus (3,3) /
//    (7,7) (from 6 fragments): 20 fragment reads per 32 rows instead of 52;
//  * waves 4-7 own the weight gradient, 64 patch columns (two tiles) each, so
//    one read of the split d1 operand serves two tiles, and the column sums
//    (v_dot4 of the patch bytes they read anyway);
//  * the gather runs two stages ahead (two register sets).
// Weight-gradient arithmetic: f16x2 (f16x2.hpp) -- d1 scaled by the power of two
// of max |d1| (published by conv2's input-gradient epilogue, d1max) and split
// into f16 h, l at the commit; the patch bytes u enter as the f16 subnormals
// u * 2^-24 (exact; tower.hpp u8x8_to_f16); two MFMAs per k16 and tile, the
// partials unscaled by 2^24 / s when stored.  Integer A partials are exact.
__device__ __forceinline__ void af_transpose4(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3,
                                              uint32_t* out) {
  const uint32_t p01l = __builtin_amdgcn_perm(w1, w0, 0x05010400u);
  const uint32_t p01h = __builtin_amdgcn_perm(w1, w0, 0x07030602u);
  const uint32_t p23l = __builtin_amdgcn_perm(w3, w2, 0x05010400u);
  const uint32_t p23h = __builtin_amdgcn_perm(w3, w2, 0x07030602u);
  out[0] = __builtin_amdgcn_perm(p23l, p01l, 0x05040100u);
  out[1] = __builtin_amdgcn_perm(p23l, p01l, 0x07060302u);
  out[2] = __builtin_amdgcn_perm(p23h, p01h, 0x05040100u);
  out[3] = __builtin_amdgcn_perm(p23h, p01h, 0x07060302u);
}


struct AfRegs {  // one stage's gather: 4 rows x 8 patch bytes, one float4 of d1
  uint2 a[4];
  uint32_t f;  // the rows' XOR mask: 0x80 bytes (x = u - 128), 0 past the chunk
  StF4 d;
};

__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void conv1_afactor_roles_kernel(
    const uint8_t* obs, long long img_stride, int rows, int chunk_rows, int* part, int* colsum,
    const float* d1, float* wpart, const unsigned* d1max) {
  const int total = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, base_l = total >> 3, rem = total & 7;
  const int chunk = xcd * base_l + min(xcd, rem) + (b >> 3);
  const int r_begin = chunk * chunk_rows;
  const int r_end = min(rows, r_begin + chunk_rows);
  __shared__ __attribute__((aligned(16))) uint8_t lds[2][256 * AF_LINE];
  constexpr int DRA = 64;             // d1 image row bytes: 32 channels x f16
  constexpr int DPART = AF_BK * DRA;  // 4 KB per split part (h, l)
  __shared__ __attribute__((aligned(16))) char dimg[2][2 * DPART];
  const float sd = f16x2_scale_of_bits(d1max);  // (every lane: before the role branch)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // roles branch on SGPRs
  const int half = lane >> 5;
  // staging map (as above): 4 rows x 8 patch columns per thread; d1: one float4
  const int drow = tid >> 3, dcol = (tid & 7) * 4;
  const int q4 = tid & 15;
  const int c = 8 * (tid >> 4);
  const int coff = (((c >> 5) * AF_OBS_W) + ((c & 31) >> 2)) * 4;
  const uint32_t istride = (uint32_t)img_stride;

  // Buffer loads on 32-bit offsets: a row past r_end gets an offset past the
  // buffer's end, so the hardware returns zeros (its patch XOR mask is then 0:
  // x = 0; its d1 = 0).  The gather position advances AF_BK rows per fetch
  // (fetches run in row order), so the per-stage decode is a few adds.
  const uint32_t obs_nr = (uint32_t)(rows / 400) * istride;
  const uint32_t d1_nr = (uint32_t)rows * 128u;
  const __amdgpu_buffer_rsrc_t obs_rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(obs), (short)0, (int)obs_nr, 0x00020000);
  const __amdgpu_buffer_rsrc_t d1_rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(d1), (short)0, (int)d1_nr, 0x00020000);
  int fr = r_begin + 4 * q4;                                  // first of the thread's 4 rows
  uint32_t fp = (uint32_t)fr % 400u;                          // its output position
  uint32_t fimg = (uint32_t)fr / 400u * istride + (uint32_t)coff;  // image + column offset
  int fk = r_begin + drow;                                    // d1 row
  const uint32_t dcb = (uint32_t)dcol * 4u;
  auto fetch = [&](AfRegs& R) {
    const bool ok = fr < r_end;
    const uint32_t oh = (fp * 3277u) >> 16;  // fp / 20 (fp < 400)
    // ((4 oh) * 84 + 4 ow) * 4 with ow = fp - 20 oh
    const uint32_t off = ok ? fimg + 16u * fp + 1024u * oh : obs_nr;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      R.a[q] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(obs_rs, off + 16u * q, 0, 0));
    R.f = ok ? 0x80808080u : 0u;
    const uint32_t doff = fk < r_end ? (uint32_t)fk * 128u + dcb : d1_nr;
    R.d = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(d1_rs, doff, 0, 0));
    fr += AF_BK;
    fk += AF_BK;
    fp += AF_BK;
    const bool wrap = fp >= 400u;
    fp = wrap ? fp - 400u : fp;
    fimg = wrap ? fimg + istride : fimg;
  };
  double dsum[4] = {0.0, 0.0, 0.0, 0.0};  // bias gradient: ~8000 rows per thread column
  auto commit = [&](const AfRegs& R, int buf) {
    const uint32_t F = R.f;
    uint32_t cols[8];
    af_transpose4(R.a[0].x ^ F, R.a[1].x ^ F, R.a[2].x ^ F, R.a[3].x ^ F, cols);
    af_transpose4(R.a[0].y ^ F, R.a[1].y ^ F, R.a[2].y ^ F, R.a[3].y ^ F, cols + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) *reinterpret_cast<uint32_t*>(lds[buf] + (c + j) * AF_LINE + 4 * q4) = cols[j];
    dsum[0] += (double)R.d.x;
    dsum[1] += (double)R.d.y;
    dsum[2] += (double)R.d.z;
    dsum[3] += (double)R.d.w;
    uint2 h, l;
    split2(R.d.x, R.d.y, sd, h.x, l.x);
    split2(R.d.z, R.d.w, sd, h.y, l.y);
    char* ds = dimg[buf] + drow * DRA + 2 * dcol;
    *reinterpret_cast<uint2*>(ds) = h;
    *reinterpret_cast<uint2*>(ds + DPART) = l;
  };

  const int fb = wave == 1 ? 4 : 0;  // tri roles: first of the 4 column blocks
  const int gb = wave == 2 ? 4 : 6;  // rect roles: column blocks gb, gb + 1
  // d1 fragment offset in the [k][32] image (conv1_wgrad_x3_kernel's map)
  const int daoff = (8 * half + ((lane >> 2) & 3)) * DRA + 8 * (4 * ((lane >> 4) & 1) + (lane & 3));
  const int nst = r_end > r_begin ? (r_end - r_begin + AF_BK - 1) / AF_BK : 0;
  int* out = part + (long long)chunk * 65536;
  auto put = [&](const v16i& v, int ti, int tj) {
    const int col = 32 * tj + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = 32 * ti + (r & 3) + 8 * (r >> 2) + 4 * half;
      out[row * 256 + col] = v[r];
    }
  };

  // Each role runs the whole stage loop with its own accumulators (one loop
  // shared by the roles merges their register sets at every join and spills).
  // The branch is wave-uniform and every role executes the same barriers.
  auto run = [&](auto ROLEc) {
    constexpr int ROLE = decltype(ROLEc)::value;  // 0 tri, 1 rect, 2 weight gradient
    constexpr int NT = ROLE == 2 ? 2 : 9;
    v16i acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = 0;
    int csum[2] = {0, 0};  // weight-gradient role: its two patch columns' sums of x

    auto compute = [&](int cur) {
      const uint8_t* S = lds[cur] + (lane & 31) * AF_LINE + 16 * half;
      if constexpr (ROLE == 0) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          v4i f[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) f[i] = *reinterpret_cast<const v4i*>(S + (fb + i) * 32 * AF_LINE + 32 * s);
          int t = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = i; j < 4 - (i == 3); ++j, ++t)
              acc[t] = __builtin_amdgcn_mfma_i32_32x32x32_i8(f[i], f[j], acc[t], 0, 0, 0);
        }
      } else if constexpr (ROLE == 1) {
        // the diagonal tile (3,3) / (7,7): block db's fragment
        const int db = wave == 2 ? 3 : 7;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          v4i f[4], g[2];
#pragma unroll
          for (int i = 0; i < 4; ++i) f[i] = *reinterpret_cast<const v4i*>(S + i * 32 * AF_LINE + 32 * s);
#pragma unroll
          for (int j = 0; j < 2; ++j) g[j] = *reinterpret_cast<const v4i*>(S + (gb + j) * 32 * AF_LINE + 32 * s);
          const v4i dg = *reinterpret_cast<const v4i*>(S + db * 32 * AF_LINE + 32 * s);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[2 * i + j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(f[i], g[j], acc[2 * i + j], 0, 0, 0);
          acc[8] = __builtin_amdgcn_mfma_i32_32x32x32_i8(dg, dg, acc[8], 0, 0, 0);
        }
      } else {
        // weight gradient: C^T[channel][patch column] over this stage's 64 rows.
        // Software-pipelined: every LDS operand of the stage is read up front,
        // and the u8 -> f16 conversion of k-step ks + 1 (VALU) is interleaved
        // with the four MFMAs of k-step ks (one wave issues both in order).
        const char* dsb = dimg[cur];
        const uint8_t* pc = lds[cur] + (64 * (wave - 4) + (lane & 31)) * AF_LINE + 8 * half;
        constexpr int NK = AF_BK / 16;
        f16x8 a[NK][2];
        uint2 xb[NK][2];
#pragma unroll
        for (int ks = 0; ks < NK; ++ks) {
#pragma unroll
          for (int pt = 0; pt < 2; ++pt) {
            const char* ap = dsb + pt * DPART + 16 * ks * DRA + daoff;
            a[ks][pt] = cat8h(ds_tr16(ap), ds_tr16(ap + 4 * DRA));
          }
#pragma unroll
          for (int tt = 0; tt < 2; ++tt) xb[ks][tt] = *reinterpret_cast<const uint2*>(pc + tt * 32 * AF_LINE + 16 * ks);
        }
        auto convert = [&](const uint2& x, int tt) {
          csum[tt] = __builtin_amdgcn_sdot4((int)x.x, 0x01010101, csum[tt], false);
          csum[tt] = __builtin_amdgcn_sdot4((int)x.y, 0x01010101, csum[tt], false);
          return u8x8_to_f16(make_uint2(x.x ^ 0x80808080u, x.y ^ 0x80808080u));  // back to u
        };
        f32x16 w0 = __builtin_bit_cast(f32x16, acc[0]);
        f32x16 w1 = __builtin_bit_cast(f32x16, acc[1]);
        f16x8 b0 = convert(xb[0][0], 0), b1 = convert(xb[0][1], 1);
#pragma unroll
        for (int ks = 0; ks < NK; ++ks) {
          f16x8 n0 = b0, n1 = b1;
          if (ks + 1 < NK) {
            n0 = convert(xb[ks + 1][0], 0);
            n1 = convert(xb[ks + 1][1], 1);
          }
#pragma unroll
          for (int pt = 1; pt >= 0; --pt) {  // l, then h
            w0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[ks][pt], b0, w0, 0, 0, 0);
            w1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[ks][pt], b1, w1, 0, 0, 0);
          }
          if (ks + 1 < NK)
#pragma unroll
            for (int i = 0; i < 4; ++i) {  // one MFMA, then a share of the next conversion
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
            }
          b0 = n0;
          b1 = n1;
        }
        acc[0] = __builtin_bit_cast(v16i, w0);
        acc[1] = __builtin_bit_cast(v16i, w1);
      }
    };

    AfRegs R0, R1;
    fetch(R0);
    fetch(R1);
    commit(R0, 0);
    __syncthreads();
    // stage st computes buffer st & 1, gathers stage st + 2 into the register set
    // stage st just committed, and commits stage st + 1 from the other set
    auto stage = [&](int st, AfRegs& Rn, const AfRegs& Rc) {
      const int cur = st & 1;
      fetch(Rn);
      __builtin_amdgcn_sched_barrier(0);
      compute(cur);
      __builtin_amdgcn_sched_barrier(0);
      commit(Rc, cur ^ 1);
      __syncthreads();
    };
    // (the odd last stage after the loop: a conditional second stage inside it
    // would leave the first set's loads pending at the back edge, and the wait
    // at the loop head would drain every load each iteration)
    int st = 0;
    for (; st + 1 < nst; st += 2) {
      stage(st, R0, R1);
      stage(st + 1, R1, R0);
    }
    if (st < nst) stage(st, R0, R1);

    if constexpr (ROLE == 0) {
      int t = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = i; j < 4 - (i == 3); ++j, ++t) put(acc[t], fb + i, fb + j);
    } else if constexpr (ROLE == 1) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) put(acc[2 * i + j], i, gb + j);
      put(acc[8], wave == 2 ? 3 : 7, wave == 2 ? 3 : 7);
    } else {
      // column sums: the two row halves (lanes l, l + 32) of each patch column;
      // integer sums, any order
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const int v = csum[tt] + __shfl_xor(csum[tt], 32);
        if (half == 0) colsum[(long long)chunk * 256 + 64 * (wave - 4) + 32 * tt + lane] = v;
      }
      // acc[tt][r]: channel (r&3) + 8(r>>2) + 4(lane>>5), patch column i;
      // unscaled: the subnormal pixels' 2^-24 and d1's scale (exact)
      float* wout = wpart + (long long)chunk * 257 * 32;
      const float unscale = 16777216.0f / sd;
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const f32x16 w = __builtin_bit_cast(f32x16, acc[tt]) * unscale;
        const int i = 64 * (wave - 4) + 32 * tt + (lane & 31);
#pragma unroll
        for (int gq = 0; gq < 4; ++gq)
          *reinterpret_cast<float4*>(wout + i * 32 + 8 * gq + 4 * half) =
              make_float4(w[4 * gq], w[4 * gq + 1], w[4 * gq + 2], w[4 * gq + 3]);
      }
    }
  };
  if (wave < 2)
    run(std::integral_constant<int, 0>{});
  else if (wave < 4)
    run(std::integral_constant<int, 1>{});
  else
    run(std::integral_constant<int, 2>{});

  // bias gradient (row 256): the 64 row-threads of each channel group through LDS
  double* cs = reinterpret_cast<double*>(&lds[0][0]);  // free after the last stage's barrier
#pragma unroll
  for (int e = 0; e < 4; ++e) cs[drow * 32 + dcol + e] = dsum[e];
  __syncthreads();
  if (tid < 32) {
    double t = 0.0;
    for (int r = 0; r < AF_BK; ++r) t += cs[r * 32 + tid];
    wpart[(long long)chunk * 257 * 32 + 256 * 32 + tid] = (float)t;
  }
}

// chunks for the one-block-per-chunk kernel: the chunk count is a multiple of
// 256 slots, one block per CU per round (against 512: configs[2] 477-480 K ->
// 490-491 K env-steps/s, the default config unchanged -- the chunk partials'
// reduction and the fused weight gradient's finalize halve; 128 / 384 / 1024
// slower, profiles/r04_ab/af_slots.txt)
static void af_plan_tri(long long rows, int* nchunk, int* chunk) {
  const long long slots = 256;
  const long long nc0 = std::max<long long>(1, (rows + AF_CHUNK - 1) / AF_CHUNK);
  const long long rounds = (nc0 + slots - 1) / slots;
  const long long nc = std::max<long long>(nc0, rounds * slots);
  long long ch = (rows + nc - 1) / nc;
  ch = (ch + AF_BK - 1) / AF_BK * AF_BK;
  *chunk = (int)std::max<long long>(ch, AF_BK);
  *nchunk = (int)((rows + *chunk - 1) / *chunk);
}

// A (257 x 257, f32) from the exact integer partials, in two passes:
//  1. conv1_afactor_reduce: int64 sums over the chunks -- blocks of 64 consecutive
//     elements x 4 chunk groups (every chunk's partial row read coalesced, 8 loads
//     in flight per thread, 4x the waves of one thread per element); elements of
//     the 32x32 tiles below the diagonal (never written) are skipped; the last 4
//     blocks sum the column sums.  Integer sums: the order is immaterial.
//  2. conv1_afactor_finalize: A = (sum u u^T) / (255^2 R) with u = x + 128,
//     mirrored into both halves.
__global__ __launch_bounds__(256) void conv1_afactor_reduce(const int* part, const int* colsum,
                                                            int nchunk, long long* sums) {
  __shared__ long long red[4][64];
  const int t = threadIdx.x, e0 = blockIdx.x * 64, el = t & 63, g = t >> 6;
  const bool cs = e0 >= 65536;  // column-sum blocks
  const int e = (cs ? e0 - 65536 : e0) + el;
  const int row = e >> 8, col = e & 255;
  long long acc = 0;
  if (cs ? e < 256 : (row >> 5) <= (col >> 5)) {
    const int* src = cs ? colsum + e : part + e;
    const long long stride = cs ? 256 : 65536;
    for (int c0 = g; c0 < nchunk; c0 += 32) {
      int v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int c = c0 + 4 * u;
        v[u] = src[(long long)(c < nchunk ? c : 0) * stride];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += (c0 + 4 * u < nchunk) ? v[u] : 0;
    }
  }
  red[g][el] = acc;
  __syncthreads();
  if (g == 0) sums[(cs ? 65536 : 0) + e] = red[0][el] + red[1][el] + red[2][el] + red[3][el];
}

__global__ void conv1_afactor_finalize(const long long* sums, int rows, float* astat) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= 257 * 257) return;
  const int lo = idx / 257, hi = idx - lo * 257;
  if (lo > hi) return;
  const long long R = rows;
  const long long* sx = sums + 65536;
  double v;
  if (hi == 256 && lo == 256) {
    v = 1.0;
  } else if (hi == 256) {
    v = (double)(sx[lo] + 128 * R) / (255.0 * (double)R);
  } else {
    const long long uu = sums[lo * 256 + hi] + 128 * (sx[lo] + sx[hi]) + 16384 * R;
    v = (double)uu / (65025.0 * (double)R);
  }
  astat[lo * 257 + hi] = (float)v;
  astat[hi * 257 + lo] = (float)v;
}

// partials + column sums (ints), then the int64 sums (8-byte aligned, 2 ints of slack)
long long conv1_afactor_ws_ints(long long rows) {
  int nchunk, chunk, nt, ct;
  af_plan(rows, &nchunk, &chunk);
  af_plan_tri(rows, &nt, &ct);
  return (long long)std::max(nchunk, nt) * (65536 + 256) + 2 * (65536 + 256) + 2 +
         (long long)nt * 257 * 32 + 4;  // + the fused weight-gradient partials (floats)
}

// chunks of the one-block-per-chunk (fused) kernel, for the weight-gradient finalize
int conv1_afactor_fused_chunks(long long rows) {
  int nt, ct;
  af_plan_tri(rows, &nt, &ct);
  return nt;
}

int conv1_afactor_u8(const uint8_t* obs, long long img_stride, int B, float* astat, int* ws,
                     long long ws_ints, hipStream_t s, const float* d1, float** wpart_out, const unsigned* d1max) {
  const long long rows = 400LL * B;
  const bool tri = g_gemm_mode == ACMI_GEMM_X3;
  ACMI_REQUIRE(tri == (d1 != nullptr) && (!d1 || d1max), ACMI_ERR_ARG,
               "conv1 A factor: the x3 mode fuses the weight gradient (d1 and its published max needed)");
  int nchunk, chunk;
  if (tri)
    af_plan_tri(rows, &nchunk, &chunk);
  else
    af_plan(rows, &nchunk, &chunk);
  ACMI_REQUIRE(conv1_afactor_ws_ints(rows) <= ws_ints, ACMI_ERR_WS,
               "conv1 A-factor workspace too small");
  ACMI_REQUIRE(img_stride % 8 == 0, ACMI_ERR_ARG, "conv1 A factor needs 8-byte aligned images");
  ACMI_REQUIRE(img_stride > 0 && (long long)B * img_stride < (1LL << 32), ACMI_ERR_ARG,
               "conv1 A factor: frames must span < 2^32 bytes");
  int* part = ws;
  int* colsum = ws + (long long)nchunk * 65536;
  long long* sums = reinterpret_cast<long long*>(
      ((uintptr_t)(colsum + (long long)nchunk * 256) + 7) & ~(uintptr_t)7);
  // fused weight-gradient partials after the int64 sums (16-byte aligned)
  float* wpart = reinterpret_cast<float*>(((uintptr_t)(sums + 65536 + 256) + 15) & ~(uintptr_t)15);
  if (wpart_out) *wpart_out = d1 ? wpart : nullptr;
  if (tri) {
    // buffer-resource offsets: frames and d1 within 2^32 bytes (152K frames)
    ACMI_REQUIRE((long long)B * img_stride <= (1LL << 32) - 64 && rows * 128 < (1LL << 32), ACMI_ERR_ARG,
                 "conv1 A factor: batch too large for 32-bit buffer offsets (B=%d)", B);
    hipLaunchKernelGGL(conv1_afactor_roles_kernel, dim3(nchunk), dim3(512), 0, s, obs, img_stride,
                       (int)rows, chunk, part, colsum, d1, wpart, d1max);
  } else
    hipLaunchKernelGGL(conv1_afactor_i8_kernel, dim3(3 * nchunk), dim3(256), 0, s, obs, img_stride,
                       (int)rows, chunk, part, colsum);
  hipLaunchKernelGGL(conv1_afactor_reduce, dim3(65536 / 64 + 4), dim3(256), 0, s, part, colsum, nchunk,
                     sums);
  hipLaunchKernelGGL(conv1_afactor_finalize, dim3(cdiv(257 * 257, 256)), dim3(256), 0, s, sums,
                     (int)rows, astat);
  ACMI_LAUNCH_CHECK("conv1_afactor_u8");
  return ACMI_OK;
}

}  // namespace acmi
