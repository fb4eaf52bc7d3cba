// K-FAC on gfx950: running factors (EMA with zero-debias), pi-adjusted
// damped inverses in fp64 (batched block Gauss-Jordan), fp64 one-sided
// Jacobi eigenvalues, natural-gradient preconditioning with the trust-region
// coefficient computed on the device, and the momentum update.
//
// Reference: kfac_utils.py:38-53 (schedule + apply), a2c_acktr.py:233-247
// (hyper-parameters), third-party tensorflow/kfac (un-vendored, unpinned:
// conventions restated in DESIGN.md §K-FAC and oracle/oracle.py).
#include <math.h>

#include <algorithm>
#include <vector>

#include "gemm.hpp"

namespace acmi {

struct Layout;
bool get_layout(int A, int C3, Layout* L);

// mirror of net.hip's Layout (kept in sync through acmi_kfac_layout)
struct KLayout {
  long long din[6], dout[6], stat_off[11], stat_total;
  long long poff[12];  // param offsets
  long long nparams;
  long long inv_off[12];  // Ainv_l at [2l], Ginv_l at [2l+1]
  long long inv_ld[12];   // row stride of each inverse block (n rounded up to 4)
  long long inv_total;
};

static bool klayout(int A, int C3, KLayout* K) {
  int64_t din[6], dout[6], so[11], tot, off[12];
  if (acmi_kfac_layout(A, C3, din, dout, so, &tot) != ACMI_OK) return false;
  if (acmi_param_offsets(A, C3, off) != ACMI_OK) return false;
  for (int l = 0; l < 6; ++l) {
    K->din[l] = din[l];
    K->dout[l] = dout[l];
  }
  for (int f = 0; f < 11; ++f) K->stat_off[f] = so[f];
  K->stat_total = tot;
  for (int i = 0; i < 12; ++i) K->poff[i] = off[i];
  K->nparams = acmi_param_count(A, C3);
  // inverse blocks are n x ld, ld = n rounded up to 4 (zero padding columns):
  // the preconditioning GEMMs then read every row as aligned float4 runs
  long long o = 0;
  for (int m = 0; m < 12; ++m) {
    const long long n = (m & 1) ? K->dout[m / 2] : K->din[m / 2];
    K->inv_off[m] = o;
    K->inv_ld[m] = (n + 3) / 4 * 4;
    o += n * K->inv_ld[m];
  }
  K->inv_total = o;
  return true;
}

static const int CONV_LOCATIONS[6] = {400, 81, 49, 1, 1, 1};

// ---------------------------------------------------------------------------
// EMA
// ---------------------------------------------------------------------------
__global__ void ema_kernel(float* biased, float* fac, const float* st, long long n, float decay,
                           float debias, float sscale) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const float b = decay * biased[i] + (1.f - decay) * (st[i] * sscale);
    biased[i] = b;
    fac[i] = b * debias;
  }
}

// ---------------------------------------------------------------------------
// damped inverse: traces -> damped fp64 copies -> block Gauss-Jordan
// ---------------------------------------------------------------------------
constexpr int GJB = 32;  // pivot block
constexpr int MAXM = 12;

struct MatSet {
  int count;
  int n[MAXM];        // logical size
  int np[MAXM];       // padded to GJB
  long long m_off[MAXM];    // np x np doubles in ws: the matrix before even steps
  long long m1_off[MAXM];   // np x np doubles: before odd steps (the sweep ping-pongs)
  long long pi_off[MAXM];   // 2 x GJB x GJB doubles: the pivot inverse of even / odd steps
  int id[MAXM];       // original matrix index (for active subsets)
  int tile0[MAXM + 1];  // gj_step_kernel: first tile block of each matrix (prefix sums)
};

// traces of the 11 factors (normalised by dimension) -> tr[f]
struct TraceSet {
  const float* fac;
  long long off[11];
  int dim[11];
};
__global__ void traces_kernel(TraceSet t, double* tr) {
  const int f = blockIdx.x;
  const int n = t.dim[f];
  const float* m = t.fac + t.off[f];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += (double)m[(long long)i * n + i];
  __shared__ double red[4];
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) tr[f] = (red[0] + red[1] + red[2] + red[3]) / (double)n;
}

// damped matrix m = 2l + (isG): source factor, damping from pi
struct DampSet {
  const float* fac;
  long long src_off[12];
  int n[12];
  int np[12];
  long long m_off[12];
  int afac[12];   // trace index of the layer's A factor
  int gfac[12];   // trace index of the layer's G factor
  float lam[12];  // normalised damping lambda_l
};
__global__ void damp_kernel(DampSet d, const double* tr, double* ws) {
  const int m = blockIdx.y;
  const int n = d.n[m], np = d.np[m];
  const long long tot = (long long)np * np;
  const double ta = tr[d.afac[m]], tg = tr[d.gfac[m]];
  double pi = (ta > 0.0 && tg > 0.0) ? sqrt(ta / tg) : 1.0;
  const double sl = sqrt((double)d.lam[m]);
  const double add = (m & 1) ? sl / pi : sl * pi;
  const float* src = d.fac + d.src_off[m];
  double* dst = ws + d.m_off[m];
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < tot;
       e += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(e / np), c = (int)(e - (long long)r * np);
    double v;
    if (r < n && c < n) {
      // symmetrise the f32 factor exactly
      v = 0.5 * ((double)src[(long long)r * n + c] + (double)src[(long long)c * n + r]);
      if (r == c) v += add;
    } else {
      v = (r == c) ? 1.0 : 0.0;  // identity padding: block-diag(M, I)
    }
    dst[e] = v;
  }
}

// Gauss-Jordan (sweep) inverse of the GJB x GJB pivot block in LDS, all 256
// threads: per sweep every thread reads the pivot row / column entries of its
// four elements from one LDS image and writes the four updated elements to the
// other (ping-pong: one barrier per sweep).  1/pivot from v_rcp_f64 and two
// Newton steps (within an ulp of the IEEE quotient, a third of the division
// sequence's latency).  The 32 one-pivot sweeps were 12 us of the former 22 us panel
// launch with the division and two barriers per sweep; pairs of pivots per
// sweep (below) halve the chain.  (One wave doing all 32 x 32 elements without
// barriers -- 16 per lane -- measured slower: 2.52 vs 1.69 ms per inverse; the
// longer per-lane LDS chains cost more than the barriers.)
__device__ __forceinline__ double recip_f64(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = fma(-d, r, 1.0);
  r = fma(r, e, r);
  e = fma(-d, r, 1.0);
  return fma(r, e, r);
}
#ifndef ACMI_GJ_PAIRS
#define ACMI_GJ_PAIRS 1
#endif
__device__ void pivot_inverse(double (*P)[GJB + 1], double (*Q)[GJB + 1]) {
  const int tid = threadIdx.x;
  const int c = tid & (GJB - 1), r0 = tid >> 5;  // rows r0, r0+8, r0+16, r0+24
#if ACMI_GJ_PAIRS
  // Two pivots per sweep (16 sweeps, 16 barriers): pivot pair K = {t, t+1} with
  // its 2 x 2 inverse D (closed form, 1/det by recip_f64):
  //   M_KK <- D,  M_Kj <- D M_Kj,  M_iK <- -M_iK D,  M_ij <- M_ij - M_iK D M_Kj
  // -- the composition of the two one-pivot sweeps, with half their dependent
  // LDS round trips, reciprocals and barriers.  The 2 x 2 diagonal blocks of the
  // damped SPD factors and of their Schur complements are SPD (det > 0).
  static_assert(GJB % 4 == 0, "an even number of pair sweeps ends in P");
  for (int t = 0; t < GJB; t += 4) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      double (*src)[GJB + 1] = h ? Q : P;
      double (*dst)[GJB + 1] = h ? P : Q;
      const int k0 = t + 2 * h;
      // every LDS read of the sweep first (the writes go to the other image, but
      // interleaved with them the reads could not be hoisted: one LDS round trip
      // per row), then the arithmetic, then the four writes
      const double a = src[k0][k0], b = src[k0][k0 + 1], e = src[k0 + 1][k0], d = src[k0 + 1][k0 + 1];
      const double s0 = src[k0][c], s1 = src[k0 + 1][c];
      double m0[4], m1[4], mc[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = r0 + 8 * q;
        m0[q] = src[r][k0];
        m1[q] = src[r][k0 + 1];
        mc[q] = src[r][c];
      }
      const double idet = recip_f64(fma(a, d, -(b * e)));
      const double D00 = d * idet, D01 = -b * idet, D10 = -e * idet, D11 = a * idet;
      const double u0 = fma(D00, s0, D01 * s1), u1 = fma(D10, s0, D11 * s1);  // (D M_Kc)
      const int ck = c - k0;
      const double dc0 = ck == 0 ? D00 : D01, dc1 = ck == 0 ? D10 : D11;  // column c of D (c in K)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = r0 + 8 * q;
        double v;
        if (r == k0 || r == k0 + 1) {
          const double w = r == k0 ? u0 : u1;
          v = (ck == 0 || ck == 1) ? (r == k0 ? dc0 : dc1) : w;
        } else {
          v = (ck == 0 || ck == 1) ? -fma(m0[q], dc0, m1[q] * dc1) : mc[q] - fma(m0[q], u0, m1[q] * u1);
        }
        dst[r][c] = v;
      }
      __syncthreads();
    }
  }
#else
  static_assert(GJB % 2 == 0, "an even number of sweeps ends in P");
  for (int t = 0; t < GJB; t += 2) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      double (*src)[GJB + 1] = h ? Q : P;
      double (*dst)[GJB + 1] = h ? P : Q;
      const int tt = t + h;
      const double ipiv = recip_f64(src[tt][tt]);
      const double ptc = src[tt][c];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = r0 + 8 * q;
        const double prt = src[r][tt];
        const double prc = src[r][c];
        double v;
        if (r == tt) v = c == tt ? ipiv : ptc * ipiv;
        else v = c == tt ? -prt * ipiv : prc - prt * ptc * ipiv;
        dst[r][c] = v;
      }
      __syncthreads();
    }
  }
#endif
}

// Symmetric sweep: the damped factors are symmetric, and the sweep operator
//   M_kk <- -P^-1,  M_kj <- P^-1 M_kj,  M_ik <- M_ik P^-1,  M_ij <- M_ij - M_ik P^-1 M_kj
// keeps every intermediate matrix symmetric (sweeping all pivots leaves -M^-1),
// so gj_step_kernel computes the 64x64 tiles on and above the diagonal only
// (half the work and traffic of the plain Gauss-Jordan update) and everything
// reads element (r, c) from the upper triangle (gj_sym).
__device__ __forceinline__ double gj_sym(const double* M, int np, int r, int c) {
  return r <= c ? M[(long long)r * np + c] : M[(long long)c * np + r];
}

// One kernel per pivot step k (pivot block rows / columns kb = 32k .. kb + 31),
// reading the matrix M_k and writing M_{k+1} (two buffers, ping-pong), with
// the pivot inverse Pinv_k already computed -- by the previous step's kernel:
//   blocks (m, 0): the NEXT pivot block of matrix m -- its 32 x 32 entries of
//     M_{k+1} (the same sums, in the same order, as the tile block that stores
//     them) and their 32-sweep inverse into Pinv_{k+1}, concurrently with
//   blocks (m, 1 + t): upper-triangle 64 x 64 tile t of M_{k+1}: Rrow' =
//     Pinv_k M_k[kb.., j] for the tile's columns (thread (column, 8 pivot rows)),
//     the old pivot columns Ccol = M_k[i][kb..] of its rows, and 4 x 4 outputs
//     per thread.
// So a step is one launch whose critical path is a tile update or one pivot
// inverse, not both in sequence: the sweep's 32 dependent barriers (12 us) used
// to sit in a separate panel launch before every update (50 + 50 launches for the
// 1568-wide factor, 1.69 ms per inverse).  Blocks (m, 0) come first in dispatch
// order (grid x = matrix, y = 0 the pivot block).
__device__ __forceinline__ const double* gj_in(const MatSet& s, int mi, int step, double* ws) {
  return ws + ((step & 1) ? s.m1_off[mi] : s.m_off[mi]);
}
__device__ __forceinline__ double* gj_out(const MatSet& s, int mi, int step, double* ws) {
  return ws + ((step & 1) ? s.m_off[mi] : s.m1_off[mi]);
}

// Pinv_0 of every matrix (blocks: matrices)
__global__ __launch_bounds__(256) void gj_first_kernel(MatSet s, double* ws) {
  const int mi = blockIdx.x;
  const int np = s.np[mi];
  const double* M = ws + s.m_off[mi];
  __shared__ double P[GJB][GJB + 1];
  __shared__ double Q[GJB][GJB + 1];
  for (int e = threadIdx.x; e < GJB * GJB; e += 256) P[e / GJB][e % GJB] = M[(long long)(e / GJB) * np + e % GJB];
  __syncthreads();
  pivot_inverse(P, Q);
  double* PI = ws + s.pi_off[mi];
  for (int e = threadIdx.x; e < GJB * GJB; e += 256) PI[e] = P[e / GJB][e % GJB];
}

// LDS of gj_step_kernel (doubles): the tile blocks' Pv [32][33] | Cs [64][33] |
// Rs [32][65]; the pivot block's four [32][33] arrays over the same words
constexpr int kGjLds = GJB * (GJB + 1) + 64 * (GJB + 1) + GJB * (64 + 1);
typedef double GjRow[GJB + 1];

// The step's products on the fp64 matrix cores (v_mfma_f64_16x16x4f64): a 16 x 16
// block of A[.][0..31] B[0..31][.] as eight k-steps of 4 in k order.  Lane l feeds
// A[l & 15][4s + (l >> 4)] and B[4s + (l >> 4)][l & 15]; result reg r is element
// (row (l >> 4) + 4r, column l & 15).  The tile blocks and the next-pivot block
// form every element of Rrow' and of the update with this same chain, so the
// pivot block's copy of M_{k+1}'s next pivot block is bit-identical to the one
// the tile block stores.
typedef double f64x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ int gj_lrow(int r) { return ((threadIdx.x & 63) >> 4) + 4 * r; }  // result row
__device__ __forceinline__ int gj_lcol() { return threadIdx.x & 15; }                          // result column
template <int NB, class FA, class FB>
__device__ __forceinline__ void gj_mfma32(f64x4 (&acc)[NB], FA a, FB b) {
  const int l = threadIdx.x & 63, ar = l & 15, ak = l >> 4;
#pragma unroll
  for (int u = 0; u < NB; ++u) acc[u] = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s = 0; s < GJB / 4; ++s)
#pragma unroll
    for (int u = 0; u < NB; ++u)
      acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a(u, ar, 4 * s + ak), b(u, 4 * s + ak, ar), acc[u], 0, 0, 0);
}

// block (m, 0): Pinv_{k+1} from M_k and Pinv_k
__device__ void gj_next_pivot(const MatSet& s, double* ws, int step, int mi, double* lds) {
  const int np = s.np[mi];
  const int kb = step * GJB, nb = kb + GJB;
  if (nb >= np) return;
  const double* M = gj_in(s, mi, step, ws);
  const double* PIk = ws + s.pi_off[mi] + (step & 1) * GJB * GJB;
  double* PIn = ws + s.pi_off[mi] + ((step + 1) & 1) * GJB * GJB;
  GjRow* Pv = reinterpret_cast<GjRow*>(lds);  // Pinv_k; later the sweep's Q
  GjRow* Mr = Pv + GJB;  // M_k[kb + q][nb + c]: pivot rows over the next block's columns; later P
  GjRow* Cn = Mr + GJB;  // M_k[nb + r][kb + t]: the next block's rows over the pivot columns
  GjRow* Rn = Cn + GJB;  // Rrow' over the next block's columns
  GjRow* P = Mr;
  GjRow* Q = Pv;
  const int c = threadIdx.x & (GJB - 1), r0 = threadIdx.x >> 5;
  // wave w: the 16 x 16 block (rows 16 (w >> 1), columns 16 (w & 1)) of Rn and P
  const int w = threadIdx.x >> 6, br = 16 * (w >> 1), bc = 16 * (w & 1);
  double oldv[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = r0 + 8 * u;
    Pv[r][c] = PIk[r * GJB + c];
    Mr[r][c] = gj_sym(M, np, kb + r, nb + c);
    Cn[c][r] = M[(long long)(kb + r) * np + nb + c];  // (the upper element of (nb + c, kb + r))
    oldv[u] = M[(long long)(nb + br + gj_lrow(u)) * np + nb + bc + gj_lcol()];
  }
  __syncthreads();
  {  // the tile blocks' Rrow' = Pinv_k M_k[kb.., nb..]
    f64x4 acc[1];
    gj_mfma32(acc, [&](int, int i, int k) { return Pv[br + i][k]; }, [&](int, int k, int j) { return Mr[k][bc + j]; });
#pragma unroll
    for (int r = 0; r < 4; ++r) Rn[br + gj_lrow(r)][bc + gj_lcol()] = acc[0][r];
  }
  __syncthreads();
  {  // the tile blocks' update: P = M_k[nb.., nb..] - Ccol Rrow'
    f64x4 acc[1];
    gj_mfma32(acc, [&](int, int i, int k) { return Cn[br + i][k]; }, [&](int, int k, int j) { return Rn[k][bc + j]; });
#pragma unroll
    for (int r = 0; r < 4; ++r) P[br + gj_lrow(r)][bc + gj_lcol()] = oldv[r] - acc[0][r];
  }
  __syncthreads();
  pivot_inverse(P, Q);
#pragma unroll
  for (int u = 0; u < 4; ++u) PIn[(r0 + 8 * u) * GJB + c] = P[r0 + 8 * u][c];
}

// grid: the active matrices' pivot blocks, then every matrix's upper-triangle
// 64x64 tiles (tile0 prefix sums)
__global__ __launch_bounds__(256) void gj_step_kernel(MatSet s, double* ws, int step) {
  __shared__ double lds[kGjLds];
  if ((int)blockIdx.x < s.count) {
    gj_next_pivot(s, ws, step, blockIdx.x, lds);
    return;
  }
  const int b = blockIdx.x - s.count;
  int mi = 0;
  while (mi + 1 < s.count && b >= s.tile0[mi + 1]) ++mi;
  const int np = s.np[mi];
  const int nt = (np + 63) / 64;
  int ti = 0, rem = b - s.tile0[mi];  // tile (ti, tj), ti <= tj, row-major over the upper triangle
  while (ti < nt && rem >= nt - ti) rem -= nt - ti, ++ti;
  if (ti >= nt) return;
  const int i0 = ti * 64, j0 = (ti + rem) * 64;
  const int kb = step * GJB;
  const double* M = gj_in(s, mi, step, ws);
  double* Mo = gj_out(s, mi, step, ws);
  const double* PIk = ws + s.pi_off[mi] + (step & 1) * GJB * GJB;
  // every load issued up front, then the LDS stores: the old values of the
  // non-pivot outputs, Pinv_k, the old pivot columns of the rows (Cs) and the
  // pivot rows over the tile's columns (Rs) -- 36 independent loads per thread in
  // one round trip (loads behind conditions or interleaved with their LDS stores
  // each waited for the whole queue: ~20 round trips per step)
  // (the upper-triangle element of (row, pivot column) / (pivot row, column) is a
  // row segment of M on one side of the pivot and a column segment on the other:
  // consecutive threads walk whichever index is contiguous in memory)
  auto sym_idx = [&](int r, int c) -> long long {  // gj_sym's element, clamped into the matrix
    const int a = min(min(r, c), np - 1), b = min(max(r, c), np - 1);
    return (long long)a * np + b;
  };
  // (no selects on the loaded values: a value of a padding row / column or of the
  // pivot block is loaded from a clamped address and never used -- the outputs
  // out of range are not stored, the pivot rows / columns take Rrow' / Pinv, and
  // the Rrow' sums of the pivot and padding columns are not formed -- so the
  // compiler cannot turn a select into a branch that waits for its load)
  // wave w: output quadrant (rows 32 (w >> 1), columns 32 (w & 1)) as 2 x 2
  // blocks of 16 x 16 (block u: rows + 16 (u >> 1), columns + 16 (u & 1))
  const int w = threadIdx.x >> 6, qr = 32 * (w >> 1), qc = 32 * (w & 1);
  auto out_i = [&](int u, int r) { return i0 + qr + 16 * (u >> 1) + gj_lrow(r); };
  auto out_j = [&](int u) { return j0 + qc + 16 * (u & 1) + gj_lcol(); };
  double old[4][4];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      old[u][r] = M[(long long)min(out_i(u, r), np - 1) * np + min(out_j(u), np - 1)];
  const bool rows_below = i0 >= kb + GJB, cols_left = j0 + 64 <= kb;
  double pv[GJB * GJB / 256], cv[64 * GJB / 256], rv[64 * GJB / 256];
#pragma unroll
  for (int u = 0; u < GJB * GJB / 256; ++u) pv[u] = PIk[threadIdx.x + 256 * u];
#pragma unroll
  for (int u = 0; u < 64 * GJB / 256; ++u) {
    const int e = threadIdx.x + 256 * u;
    const int r = rows_below ? e % 64 : e / GJB, t = rows_below ? e / 64 : e % GJB;
    cv[u] = M[sym_idx(i0 + r, kb + t)];
    const int q = cols_left ? e % GJB : e / 64, c = cols_left ? e / GJB : e % 64;
    rv[u] = M[sym_idx(kb + q, j0 + c)];  // pivot rows
  }
  GjRow* Pv = reinterpret_cast<GjRow*>(lds);
  GjRow* Cs = Pv + GJB;                                         // [64]
  double (*Rs)[64 + 1] = reinterpret_cast<double (*)[64 + 1]>(Cs + 64);  // [GJB]
#pragma unroll
  for (int u = 0; u < GJB * GJB / 256; ++u) {
    const int e = threadIdx.x + 256 * u;
    Pv[e / GJB][e % GJB] = pv[u];
  }
#pragma unroll
  for (int u = 0; u < 64 * GJB / 256; ++u) {
    const int e = threadIdx.x + 256 * u;
    const int r = rows_below ? e % 64 : e / GJB, t = rows_below ? e / 64 : e % GJB;
    Cs[r][t] = cv[u];
    const int q = cols_left ? e % GJB : e / 64, c = cols_left ? e / GJB : e % 64;
    Rs[q][c] = rv[u];
  }
  __syncthreads();
  {  // Rrow' = Pinv_k M_k[kb.., j] in place of the pivot rows: wave w, columns 16 w ..
    f64x4 acc[2];  // row blocks 0, 16
    gj_mfma32(acc, [&](int u, int i, int k) { return Pv[16 * u + i][k]; },
              [&](int, int k, int j) { return Rs[k][16 * w + j]; });
    const int cj = 16 * w + gj_lcol(), j = j0 + cj;
    const bool jcol = j < np && !(j >= kb && j < kb + GJB);
    double v[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = 16 * u + gj_lrow(r);
        // pivot columns: Rrow' = Pinv; padding columns: never used
        v[u][r] = jcol ? acc[u][r] : (j < np ? Pv[t][j - kb] : 0.0);
      }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) Rs[16 * u + gj_lrow(r)][cj] = v[u][r];
  }
  __syncthreads();
  f64x4 acc[4];  // Ccol Rrow' over the wave's quadrant
  gj_mfma32(acc, [&](int u, int i, int k) { return Cs[qr + 16 * (u >> 1) + i][k]; },
            [&](int u, int k, int j) { return Rs[k][qc + 16 * (u & 1) + j]; });
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int jj = out_j(u);
    if (jj >= np) continue;
    const bool jpiv = jj >= kb && jj < kb + GJB;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = out_i(u, r);
      if (i >= np) continue;
      const bool ipiv = i >= kb && i < kb + GJB;
      double v;
      if (ipiv) {  // pivot rows: Pinv M_kj; the pivot block -Pinv
        const double rr = Rs[i - kb][jj - j0];
        v = jpiv ? -rr : rr;
      } else {     // pivot columns: M_ik Pinv; the rest M_ij - M_ik Pinv M_kj
        v = jpiv ? acc[u][r] : old[u][r] - acc[u][r];
      }
      Mo[(long long)i * np + jj] = v;
    }
  }
}

struct OutSet {
  const double* ws;
  long long m_off[12];
  int n[12];
  int np[12];
  int ld[12];
  long long dst_off[12];
};
__global__ void gj_store_kernel(OutSet o, float* inv) {
  const int m = blockIdx.y;
  const int n = o.n[m], np = o.np[m], ld = o.ld[m];
  const double* M = o.ws + o.m_off[m];
  float* dst = inv + o.dst_off[m];
  const long long tot = (long long)n * ld;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < tot;
       e += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(e / ld), c = (int)(e - (long long)r * ld);
    dst[e] = c < n ? (float)(-gj_sym(M, np, r, c)) : 0.f;  // the sweep leaves -M^-1
  }
}

// ---------------------------------------------------------------------------
// eigenvalues: fp64 one-sided (Hestenes) Jacobi, round-robin pairs, one wave
// per column pair, one launch per round; singular values == eigenvalues of
// the SPD factors.
// ---------------------------------------------------------------------------
struct EigSet {
  int count;
  int n[11];
  int ne[11];  // n rounded up to even
  long long u_off[11];
};

__global__ void eig_load_kernel(const float* fac, EigSet s, TraceSet t, double* ws) {
  const int m = blockIdx.y;
  const int n = s.n[m];
  const float* src = fac + t.off[m];
  double* U = ws + s.u_off[m];
  const long long tot = (long long)n * n;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < tot;
       e += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(e / n), c = (int)(e - (long long)r * n);
    // column-major U (column c contiguous) of the symmetrised factor
    U[(long long)c * n + r] = 0.5 * ((double)src[(long long)r * n + c] + (double)src[(long long)c * n + r]);
  }
}

// grid.x = pair index (waves of 64 in blocks of 256), grid.y = matrix
__global__ __launch_bounds__(256) void eig_round_kernel(EigSet s, double* ws, int round,
                                                        int* rotated, double tol) {
  const int m = blockIdx.y;
  const int n = s.n[m], ne = s.ne[m];
  const int npairs = ne / 2;
  const int pair = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pair >= npairs || ne < 2) return;
  const int lane = threadIdx.x & 63;
  const int rr = round % (ne - 1);
  int p, q;
  if (pair == 0) {
    p = rr;
    q = ne - 1;
  } else {
    p = (rr + pair) % (ne - 1);
    q = (rr - pair + (ne - 1)) % (ne - 1);
  }
  if (p >= n || q >= n) return;
  double* U = ws + s.u_off[m];
  double* up = U + (long long)p * n;
  double* uq = U + (long long)q * n;
  double a = 0.0, b = 0.0, g = 0.0;
  for (int i = lane; i < n; i += 64) {
    const double x = up[i], y = uq[i];
    a += x * x;
    b += y * y;
    g += x * y;
  }
  a = wave_sum_d(a);
  b = wave_sum_d(b);
  g = wave_sum_d(g);
  if (fabs(g) <= tol * sqrt(a * b) || g == 0.0) return;
  const double zeta = (b - a) / (2.0 * g);
  const double t = (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
  const double c = 1.0 / sqrt(1.0 + t * t);
  const double sn = c * t;
  for (int i = lane; i < n; i += 64) {
    const double x = up[i], y = uq[i];
    up[i] = c * x - sn * y;
    uq[i] = sn * x + c * y;
  }
  if (lane == 0) atomicOr(rotated, 1);
}

// eigenvalue = column norm; sorted ascending by rank
__global__ void eig_store_kernel(EigSet s, const double* ws, long long* out_off, double* out,
                                 double* tmp) {
  const int m = blockIdx.x;
  const int n = s.n[m];
  const double* U = ws + s.u_off[m];
  double* nr = tmp + out_off[m];
  for (int c = threadIdx.x; c < n; c += blockDim.x) {
    double acc = 0.0;
    for (int i = 0; i < n; ++i) acc += U[(long long)c * n + i] * U[(long long)c * n + i];
    nr[c] = sqrt(acc);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < n; c += blockDim.x) {
    const double v = nr[c];
    int rank = 0;
    for (int d = 0; d < n; ++d) {
      const double w = nr[d];
      rank += (w < v) || (w == v && d < c);
    }
    out[out_off[m] + rank] = v;
  }
}

// ---------------------------------------------------------------------------
// natural-gradient step
// ---------------------------------------------------------------------------
constexpr int KRED = 512;
__global__ void kdot_partial_kernel(const float* x, const float* y, long long n, float* part) {
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

__global__ void kcoeff_kernel(const float* part, int nb, float lr, float c, float* coeff,
                              float* coeff_out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) s += part[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float sq = (red[0] + red[1] + red[2] + red[3]) * lr * lr;
    // min(1, sqrt(c / sq)); sq <= 0 or NaN -> 1 (fminf drops the NaN)
    const float v = fminf(1.f, sqrtf(c / sq));
    coeff[0] = v;
    coeff[1] = sq;
    if (coeff_out) coeff_out[0] = v;
  }
}

// y[i][j] = sum_k A[i][k] g[k][j] for the narrow (dout % 4 != 0) first
// products of the K-FAC step: block (i, j), one wave over k (fixed order:
// lane-strided partial sums, then the butterfly)
__global__ __launch_bounds__(64) void kfac_narrow_kernel(const float* a, int lda, const float* g, int dout, int n,
                                                       float* y, int ldy) {
  const int i = blockIdx.x, j = blockIdx.y;
  const float* ar = a + (long long)i * lda;
  float s = 0.f;
  for (int k = threadIdx.x; k < n; k += 64) s += ar[k] * g[(long long)k * dout + j];
  s = wave_sum(s);
  if (threadIdx.x == 0) y[(long long)i * ldy + j] = s;
}

__global__ void kapply_kernel(float* p, float* v, const float* d, long long n, float lr,
                              float mom, const float* coeff) {
  const float cf = coeff[0];
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const float nv = mom * v[i] + cf * d[i];
    v[i] = nv;
    p[i] -= lr * nv;
  }
}

// ---------------------------------------------------------------------------
// factor statistics as upper triangles (the data-parallel all-reduce): factor f
// (n x n row-major at stat_off[f], symmetric) <-> n(n+1)/2 floats, row r's
// columns r .. n-1; the selected factors back to back.  Block (row r, factor).
// ---------------------------------------------------------------------------
struct PackSet {
  int count;
  long long src_off[11];  // full factor in the stats area
  long long dst_off[11];  // packed triangle
  int n[11];
};

static bool pack_set(const KLayout& K, int which, PackSet* p, long long* total) {
  if (which < 1 || which > 3) return false;
  p->count = 0;
  long long o = 0;
  for (int f = 0; f < 11; ++f) {
    if (!((f < 5 ? 1 : 2) & which)) continue;
    const int n = (int)(f < 5 ? K.din[f] : K.dout[f - 5]);
    const int k = p->count++;
    p->src_off[k] = K.stat_off[f];
    p->dst_off[k] = o;
    p->n[k] = n;
    o += (long long)n * (n + 1) / 2;
  }
  *total = o;
  return true;
}

template <bool PACK>
__global__ __launch_bounds__(256) void kfac_pack_kernel(PackSet p, const float* src, float* dst) {
  const int k = blockIdx.y, r = blockIdx.x, n = p.n[k];
  if (r >= n) return;
  const long long tri = p.dst_off[k] + (long long)r * n - (long long)r * (r - 1) / 2 - r;  // + c
  const long long full = p.src_off[k];
  for (int c = r + threadIdx.x; c < n; c += 256) {
    if constexpr (PACK) {
      dst[tri + c] = src[full + (long long)r * n + c];
    } else {  // both halves: the factor comes back exactly symmetric
      const float v = src[tri + c];
      dst[full + (long long)r * n + c] = v;
      dst[full + (long long)c * n + r] = v;
    }
  }
}

}  // namespace acmi

using namespace acmi;

extern "C" {

int acmi_kfac_ema(float* biased, float* factors, const float* stats, int64_t n, float decay,
                  float debias, float stats_scale, acmi_stream_t stream) {
  ACMI_REQUIRE(biased && factors && stats && n > 0, ACMI_ERR_ARG, "acmi_kfac_ema: bad args");
  hipLaunchKernelGGL(ema_kernel, dim3(std::min<long long>(cdiv(n, 256), 2048)), dim3(256), 0,
                     (hipStream_t)stream, biased, factors, stats, (long long)n, decay, debias,
                     stats_scale);
  ACMI_LAUNCH_CHECK("acmi_kfac_ema");
  return ACMI_OK;
}

int64_t acmi_kfac_packed_floats(int A, int C3, int which) {
  KLayout K;
  PackSet p;
  long long tot;
  if (!klayout(A, C3, &K) || !pack_set(K, which, &p, &tot)) return -1;
  return tot;
}

static int kfac_pack_launch(int A, int C3, int which, const float* src, float* dst, hipStream_t st, bool pack) {
  KLayout K;
  PackSet p;
  long long tot;
  ACMI_REQUIRE(src && dst && klayout(A, C3, &K) && pack_set(K, which, &p, &tot), ACMI_ERR_ARG,
               "acmi_kfac_pack/unpack: bad arguments");
  int maxn = 0;
  for (int k = 0; k < p.count; ++k) maxn = std::max(maxn, p.n[k]);
  if (pack)
    hipLaunchKernelGGL(kfac_pack_kernel<true>, dim3(maxn, p.count), dim3(256), 0, st, p, src, dst);
  else
    hipLaunchKernelGGL(kfac_pack_kernel<false>, dim3(maxn, p.count), dim3(256), 0, st, p, src, dst);
  ACMI_LAUNCH_CHECK("acmi_kfac_pack");
  return ACMI_OK;
}

int acmi_kfac_pack(int A, int C3, int which, const float* stats, float* packed, acmi_stream_t stream) {
  return kfac_pack_launch(A, C3, which, stats, packed, (hipStream_t)stream, true);
}

int acmi_kfac_unpack(int A, int C3, int which, const float* packed, float* stats, acmi_stream_t stream) {
  return kfac_pack_launch(A, C3, which, packed, stats, (hipStream_t)stream, false);
}

int acmi_kfac_inverse_layout(int A, int C3, int64_t* offsets, int64_t* lds) {
  KLayout K;
  ACMI_REQUIRE(offsets && lds && klayout(A, C3, &K), ACMI_ERR_ARG,
               "acmi_kfac_inverse_layout: bad arguments");
  for (int m = 0; m < 12; ++m) {
    offsets[m] = K.inv_off[m];
    lds[m] = K.inv_ld[m];
  }
  return ACMI_OK;
}

int64_t acmi_kfac_inverse_floats(int A, int C3) {
  KLayout K;
  if (!klayout(A, C3, &K)) return -1;
  return K.inv_total;
}

static void inverse_plan(const KLayout& K, MatSet* s, long long* total) {
  long long o = 16;  // traces
  s->count = 12;
  for (int m = 0; m < 12; ++m) {
    const int l = m / 2;
    const int n = (int)((m & 1) ? K.dout[l] : K.din[l]);
    const int np = (n + GJB - 1) / GJB * GJB;
    s->n[m] = n;
    s->np[m] = np;
    s->id[m] = m;
    s->m_off[m] = o;
    o += (long long)np * np;
    s->m1_off[m] = o;
    o += (long long)np * np;
    s->pi_off[m] = o;
    o += 2LL * GJB * GJB;
  }
  *total = o;
}

int64_t acmi_kfac_inverse_ws_doubles(int A, int C3) {
  KLayout K;
  if (!klayout(A, C3, &K)) return -1;
  MatSet s;
  long long tot;
  inverse_plan(K, &s, &tot);
  return tot;
}

static TraceSet trace_set(const KLayout& K, const float* fac) {
  TraceSet t;
  t.fac = fac;
  for (int f = 0; f < 11; ++f) {
    t.off[f] = K.stat_off[f];
    t.dim[f] = (int)(f < 5 ? K.din[f] : K.dout[f - 5]);
  }
  return t;
}

int acmi_kfac_inverse(int A, int C3, const float* factors, float damping, int conv_normalize,
                      float* inv, double* ws, acmi_stream_t stream) {
  KLayout K;
  ACMI_REQUIRE(factors && inv && ws && klayout(A, C3, &K), ACMI_ERR_ARG,
               "acmi_kfac_inverse: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  MatSet s;
  long long tot;
  inverse_plan(K, &s, &tot);
  double* tr = ws;
  hipLaunchKernelGGL(traces_kernel, dim3(11), dim3(256), 0, st, trace_set(K, factors), tr);
  DampSet d;
  d.fac = factors;
  int maxnp = 0;
  for (int m = 0; m < 12; ++m) {
    const int l = m / 2;
    const int af = l < 5 ? l : 4;  // fc_policy / fc_baseline share A_4
    d.src_off[m] = (m & 1) ? K.stat_off[5 + l] : K.stat_off[af];
    d.n[m] = s.n[m];
    d.np[m] = s.np[m];
    d.m_off[m] = s.m_off[m];
    d.afac[m] = af;
    d.gfac[m] = 5 + l;
    d.lam[m] = conv_normalize ? damping / (float)CONV_LOCATIONS[l] : damping;
    maxnp = std::max(maxnp, s.np[m]);
  }
  hipLaunchKernelGGL(damp_kernel, dim3(256, 12), dim3(256), 0, st, d, tr, ws);
  const int maxsteps = maxnp / GJB;
  hipLaunchKernelGGL(gj_first_kernel, dim3(12), dim3(256), 0, st, s, ws);
  for (int step = 0; step < maxsteps; ++step) {
    MatSet a;
    a.count = 0;
    for (int m = 0; m < 12; ++m) {
      if (s.np[m] / GJB > step) {
        const int k = a.count++;
        a.n[k] = s.n[m];
        a.np[k] = s.np[m];
        a.m_off[k] = s.m_off[m];
        a.m1_off[k] = s.m1_off[m];
        a.pi_off[k] = s.pi_off[m];
        a.id[k] = m;
      }
    }
    int tiles = 0;
    for (int k = 0; k < a.count; ++k) {
      const int nt = cdiv(a.np[k], 64);
      a.tile0[k] = tiles;
      tiles += nt * (nt + 1) / 2;
    }
    a.tile0[a.count] = tiles;
    hipLaunchKernelGGL(gj_step_kernel, dim3(a.count + tiles), dim3(256), 0, st, a, ws, step);
  }
  OutSet o;
  o.ws = ws;
  for (int m = 0; m < 12; ++m) {
    o.m_off[m] = ((s.np[m] / GJB) & 1) ? s.m1_off[m] : s.m_off[m];  // after the last step
    o.n[m] = s.n[m];
    o.np[m] = s.np[m];
    o.ld[m] = (int)K.inv_ld[m];
    o.dst_off[m] = K.inv_off[m];
  }
  hipLaunchKernelGGL(gj_store_kernel, dim3(256, 12), dim3(256), 0, st, o, inv);
  ACMI_LAUNCH_CHECK("acmi_kfac_inverse");
  return ACMI_OK;
}

static void eig_plan(const KLayout& K, EigSet* s, long long* total) {
  long long o = 64;  // flag + scratch for eigenvalue staging offsets
  s->count = 11;
  for (int f = 0; f < 11; ++f) {
    const int n = (int)(f < 5 ? K.din[f] : K.dout[f - 5]);
    s->n[f] = n;
    s->ne[f] = (n + 1) / 2 * 2;
    s->u_off[f] = o;
    o += (long long)n * n;
  }
  // staging for column norms (same size as the output)
  long long e = 0;
  for (int f = 0; f < 11; ++f) e += s->n[f];
  *total = o + e + 16;
}

int64_t acmi_kfac_eig_ws_doubles(int A, int C3) {
  KLayout K;
  if (!klayout(A, C3, &K)) return -1;
  EigSet s;
  long long tot;
  eig_plan(K, &s, &tot);
  return tot;
}

// NOTE: synchronises `stream` once per sweep to test convergence (diagnostic
// path, not used inside the training step).
int acmi_kfac_eigvals(int A, int C3, const float* factors, double* eigvals, double* ws,
                      acmi_stream_t stream) {
  KLayout K;
  ACMI_REQUIRE(factors && eigvals && ws && klayout(A, C3, &K), ACMI_ERR_ARG,
               "acmi_kfac_eigvals: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  EigSet s;
  long long tot;
  eig_plan(K, &s, &tot);
  TraceSet t = trace_set(K, factors);
  hipLaunchKernelGGL(eig_load_kernel, dim3(256, 11), dim3(256), 0, st, factors, s, t, ws);
  int* flag = reinterpret_cast<int*>(ws);  // ws[0..1] doubles reused as an int flag
  int maxne = 0, maxpairs = 0;
  for (int f = 0; f < 11; ++f) {
    maxne = std::max(maxne, s.ne[f]);
    maxpairs = std::max(maxpairs, s.ne[f] / 2);
  }
  const int rounds = std::max(1, maxne - 1);
  for (int sweep = 0; sweep < 40; ++sweep) {
    if (hipMemsetAsync(flag, 0, sizeof(int), st) != hipSuccess) {
      set_error("acmi_kfac_eigvals: memset failed");
      return ACMI_ERR_HIP;
    }
    for (int r = 0; r < rounds; ++r)
      hipLaunchKernelGGL(eig_round_kernel, dim3(cdiv(maxpairs, 4), 11), dim3(256), 0, st, s, ws,
                         r, flag, 1e-15);
    int h = 0;
    if (hipMemcpyAsync(&h, flag, sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {
      set_error("acmi_kfac_eigvals: sync failed");
      return ACMI_ERR_HIP;
    }
    if (!h) break;
  }
  // output offsets (device copy not needed: passed by value through a small buffer)
  long long offs[11];
  long long o = 0;
  for (int f = 0; f < 11; ++f) {
    offs[f] = o;
    o += s.n[f];
  }
  long long* doffs = reinterpret_cast<long long*>(ws + 8);  // 11 int64 fit in ws[8..19)
  // ws[8..19) lies inside the 64-double header reserved by eig_plan
  if (hipMemcpyAsync(doffs, offs, sizeof(offs), hipMemcpyHostToDevice, st) != hipSuccess) {
    set_error("acmi_kfac_eigvals: memcpy failed");
    return ACMI_ERR_HIP;
  }
  double* staging = ws + tot - 16 - o;
  hipLaunchKernelGGL(eig_store_kernel, dim3(11), dim3(256), 0, st, s, ws, doffs, eigvals,
                     staging);
  ACMI_LAUNCH_CHECK("acmi_kfac_eigvals");
  if (hipStreamSynchronize(st) != hipSuccess) {
    set_error("acmi_kfac_eigvals: final sync failed");
    return ACMI_ERR_HIP;
  }
  return ACMI_OK;
}

// per-layer t1 = Ainv g blocks (rows padded to ldg, offsets rounded to 4 floats)
static long long kfac_t1_floats(const KLayout& K, long long* off = nullptr) {
  long long o = 0;
  for (int l = 0; l < 6; ++l) {
    if (off) off[l] = o;
    o += (K.din[l] * K.inv_ld[2 * l + 1] + 3) / 4 * 4;
  }
  return o;
}

int64_t acmi_kfac_step_ws_floats(int A, int C3) {
  KLayout K;
  if (!klayout(A, C3, &K)) return -1;
  return kfac_t1_floats(K) + KRED + 16;
}

int acmi_kfac_step(int A, int C3, float* params, float* velocity, const float* grads,
                   const float* inv, float lr, float momentum, float norm_constraint,
                   float* precon, float* ws, float* coeff_out, acmi_stream_t stream) {
  KLayout K;
  ACMI_REQUIRE(params && velocity && grads && inv && precon && ws && klayout(A, C3, &K),
               ACMI_ERR_ARG, "acmi_kfac_step: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  long long t1off[6];
  const long long t1n = kfac_t1_floats(K, t1off);
  float* part = ws + t1n;
  float* coeff = part + KRED;
  // Delta_l = Ainv_l g_l Ginv_l for the six layers as two grouped launches (all
  // first products, then all second products) instead of twelve dependent ones;
  // t1_l = Ainv_l g_l (Ainv symmetric: A(k, i) = Ainv[k][i]), rows padded to ldg.
  // The value head (dout = 1, unaligned rows of g) has its own first launch.
  GemmGroup<MatI<true>, MatI<true>, EpiStore> g1;
  GemmGroup<MatTK<true>, MatI<true>, EpiStore> g2;
  g1.n = g2.n = 0;
  for (int l = 0; l < 6; ++l) {
    const int din = (int)K.din[l], dout = (int)K.dout[l];
    const int lda = (int)K.inv_ld[2 * l], ldg = (int)K.inv_ld[2 * l + 1];
    const float* ainv = inv + K.inv_off[2 * l];
    const float* ginv = inv + K.inv_off[2 * l + 1];
    const float* g = grads + K.poff[2 * l];  // [W; b] contiguous, din x dout
    float* t1 = ws + t1off[l];
    if (dout % 4 == 0) {
      const int q = g1.n++;
      g1.a[q] = MatI<true>{ainv, lda, din, din};
      g1.b[q] = MatI<true>{g, dout, din, dout};
      g1.e[q] = EpiStore{t1, ldg};
      g1.I[q] = din, g1.J[q] = dout, g1.K[q] = din;
    } else {
      // (a GEMM launch of 128 x 32 tiles for these few columns was 19.6 us at
      // dout = 1: one wave per output instead)
      hipLaunchKernelGGL(kfac_narrow_kernel, dim3(din, dout), dim3(64), 0, s, ainv, lda, g, dout, din, t1, ldg);
    }
    const int q = g2.n++;
    g2.a[q] = MatTK<true>{t1, ldg, dout, din};
    g2.b[q] = MatI<true>{ginv, ldg, dout, dout};
    g2.e[q] = EpiStore{precon + K.poff[2 * l], dout};
    g2.I[q] = din, g2.J[q] = dout, g2.K[q] = dout;
  }
  // 64x64 tiles: fc4 (1569 x 512) alone is 200 blocks; the other layers ride along
  launch_gemm_group<64, 64, 32, 1, 1>(g1, s);
  launch_gemm_group<64, 64, 32, 1, 1>(g2, s);
  const long long n = K.nparams;
  hipLaunchKernelGGL(kdot_partial_kernel, dim3(KRED), dim3(256), 0, s, grads, precon, n, part);
  hipLaunchKernelGGL(kcoeff_kernel, dim3(1), dim3(256), 0, s, part, KRED, lr, norm_constraint,
                     coeff, coeff_out);
  hipLaunchKernelGGL(kapply_kernel, dim3(std::min<long long>(cdiv(n, 256), 2048)), dim3(256), 0,
                     s, params, velocity, precon, n, lr, momentum, coeff);
  ACMI_LAUNCH_CHECK("acmi_kfac_step");
  return ACMI_OK;
}

}  // extern "C"
