// Operand loaders of the f32-MFMA GEMM engine (gemm.hpp).
//
// An operand supplies float4 runs of its logical matrix: KCONTIG operands give
// 4 consecutive k for one i (row-major [i][k] data), the others 4 consecutive
// i for one k.  Addressing is split into a row part (the non-contiguous index)
// and a column part (the contiguous one):
//   R row(int r) const;   C col(int c) const;
//   St stage(R, C, bool in) const;   float4 finish(St)  (free function)
// stage() issues the loads of one float4 run and computes its masks without
// touching the loaded data; finish() applies the masks when the run is written
// to LDS.  The K loop issues next-tile stage()s before the MFMAs of the
// current tile and finish()es them after, so the loads are in flight across
// the MFMAs (a mask applied at load time makes the compiler wait right there).
// The thread->element map of gemm_kernel keeps one of the two fixed for a
// thread across all K-tiles (KCONTIG: the row; otherwise the column), so the
// kernel hoists that part out of the K loop and the integer div/mod of the
// implicit im2col is paid once per thread instead of once per element.
// Every load is zero outside the operand's bounds.
#pragma once

#include <type_traits>

#include "common.hpp"

namespace acmi {

__device__ __forceinline__ float4 f4zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }

// exact u8 / 255.0f (one rounding), verified exhaustively for 0..255
__device__ __forceinline__ float u8norm(uint32_t u) {
  const float x = (float)u;
  const float inv = 1.0f / 255.0f;
  const float q = x * inv;
  const float r = __builtin_fmaf(-q, 255.0f, x);
  return __builtin_fmaf(r, inv, q);
}

// Element offsets are 32-bit unsigned: every operand the engine reads holds
// < 2^31 elements (checked on the host, acmi_*), so address arithmetic is
// one 32-bit decode plus one 64-bit scaled add per load.
struct OffOk {
  uint32_t off;
  bool ok;
};

// Operands and epilogues that depend on the block's third grid coordinate (a
// stride phase, a split-K chunk) hold it in a member `z`, which the GEMM kernels
// set per tile (set_z); they never read blockIdx.z themselves.
template <class T, class = void>
struct has_z : std::false_type {};
template <class T>
struct has_z<T, std::void_t<decltype(std::declval<T&>().z)>> : std::true_type {};
template <class T>
__device__ __forceinline__ void set_z(T& t, int z) {
  if constexpr (has_z<T>::value) t.z = z;
}

// Loads are never guarded by branches and their results never pass through
// a mask: an element outside the operand loads from a 16-byte zero run (or the
// homogeneous run (1,0,0,0)) instead, selected on the ADDRESS.  A load under a
// runtime condition makes hipcc branch around it and wait vmcnt(0) per element
// (cdna_hip_programming.md §5 'Three .s-level traps' (c)); a select or multiply
// on the loaded value drags that wait in front of the MFMAs.  With address
// masking the loaded registers go straight to ds_write after the MFMAs.
// The runs are a weak, writable global: were their contents known to the
// compiler, LLVM would fold `load(c ? p : zero)` into `c ? load(p) : 0` and be
// back at the branch.  Nothing writes them.
__device__ __attribute__((weak, aligned(16))) float kMaskRuns[8] = {0.f, 0.f, 0.f, 0.f,
                                                                   1.f, 0.f, 0.f, 0.f};
__device__ __forceinline__ const float* zero_run() { return kMaskRuns; }
__device__ __forceinline__ const float* homog_run() { return kMaskRuns + 4; }

using StF4 = float4;
struct StU8 {  // four u8 pixels
  uint32_t u;
};
__device__ __forceinline__ StF4 stage_f4(const float* p, bool ok) {
  return *reinterpret_cast<const float4*>(ok ? p : zero_run());
}
__device__ __forceinline__ float4 finish(const float4& s) { return s; }
// a run of up to 4 scalars p[0..n) (n may be < 4 at an unaligned tail)
__device__ __forceinline__ StF4 stage_tail(const float* p, bool ok, int n) {
  const float* z = zero_run();
  return make_float4(*(ok ? p : z), *(ok && n > 1 ? p + 1 : z), *(ok && n > 2 ? p + 2 : z),
                     *(ok && n > 3 ? p + 3 : z));
}
// u8 pixels enter the MFMAs as their integer values 0..255 (exact in f32,
// v_cvt_f32_ubyte0..3); the 1/255 of the reference's normalisation is applied
// once per output by the consumer (EpiAct::scale for conv1, the conv1 weight
// gradient's wscale in finalize_wgrad_kernel).
__device__ __forceinline__ float4 finish(const StU8& s) {
  const uint32_t u = s.u;
  return make_float4((float)(u & 255u), (float)((u >> 8) & 255u), (float)((u >> 16) & 255u),
                     (float)(u >> 24));
}

// ---------------------------------------------------------------------------
// Row sources (logical matrices [rows][cols]); c is the first of 4 columns.
// ---------------------------------------------------------------------------

// Patches of NHWC images for a VALID conv; row r = (img, oh, ow), column
// c = (kh, kw, ch) with ch fastest (== HWIO flatten == TF extract_image_patches
// order).  T = uint8_t yields raw 0..255 values (see finish(StU8)).
template <typename T, int H, int W, int C, int KH, int KW, int S>
struct ConvRows {
  static constexpr int OH = (H - KH) / S + 1;
  static constexpr int OW = (W - KW) / S + 1;
  static constexpr int L = OH * OW;
  static constexpr int COLS = KH * KW * C;
  static_assert(C % 4 == 0, "channel runs must hold float4");
  using R = OffOk;
  using Cp = OffOk;
  using elem_t = T;
  const T* x;
  uint32_t img_stride;  // elements of T between images
  int rows;             // images * L

  // row/col decode clamped indices instead of branching (see StF4); unsigned
  // division by the constant extents is a multiply-high and a shift
  __device__ __forceinline__ R row(int r0) const {
    const bool ok = r0 < rows;
    const uint32_t r = ok ? (uint32_t)r0 : 0u;
    const uint32_t img = r / L;
    const uint32_t p = r - img * L;
    const uint32_t oh = p / OW;
    const uint32_t ow = p - oh * OW;
    return R{img * img_stride + (oh * (S * W) + ow * S) * C, ok};
  }
  __device__ __forceinline__ Cp col(int c0) const {
    const bool ok = c0 < COLS;
    const uint32_t c = ok ? (uint32_t)c0 : 0u;
    const uint32_t kh = c / (KW * C);
    const uint32_t rem = c - kh * (KW * C);
    const uint32_t kw = rem / C;
    const uint32_t ch = rem - kw * C;
    return Cp{(kh * W + kw) * C + ch, ok};
  }
  // Row iterator for loops that walk rows r0, r0 + STEP, ... (symred3): the
  // (oh, ow) decode is carried along with adds and selects instead of the two
  // constant divisions and three multiplies of row() per row (quarter-rate
  // v_mul_hi/lo_u32 on the VALU that the staging shares with the MFMAs).
  struct It {
    uint32_t off;
    int oh, ow, r;
  };
  __device__ __forceinline__ It iter(int r0) const {
    const uint32_t r = r0 < rows ? (uint32_t)r0 : 0u;
    const uint32_t img = r / L;
    const uint32_t p = r - img * L;
    const uint32_t oh = p / OW;
    const uint32_t ow = p - oh * OW;
    return It{img * img_stride + (oh * (S * W) + ow * S) * C, (int)oh, (int)ow, r0};
  }
  template <int STEP>
  __device__ __forceinline__ void advance(It& it) const {
    static_assert(STEP < L, "one image boundary per step at most");
    constexpr int DR = STEP / OW, DC = STEP % OW;
    constexpr uint32_t ROW = S * W * C, COL = S * C;
    it.r += STEP;
    it.ow += DC;
    it.oh += DR;
    it.off += DR * ROW + DC * COL;
    const bool w1 = it.ow >= OW;
    it.ow -= w1 ? OW : 0;
    it.oh += w1 ? 1 : 0;
    it.off += w1 ? ROW - OW * COL : 0u;
    const bool w2 = it.oh >= OH;
    it.oh -= w2 ? OH : 0;
    it.off += w2 ? img_stride - OH * ROW : 0u;
  }
  __device__ __forceinline__ R row_of(const It& it) const { return R{it.off, it.r < rows}; }

  using St = typename std::conditional<sizeof(T) == 1, StU8, StF4>::type;
  __device__ __forceinline__ St stage(const R& r, const Cp& c, bool in) const {
    const bool ok = in && r.ok && c.ok;
    const T* src = x + (r.off + c.off);
    if constexpr (sizeof(T) == 1)
      return StU8{*reinterpret_cast<const uint32_t*>(
          ok ? static_cast<const void*>(src) : static_cast<const void*>(zero_run()))};
    else
      return stage_f4(src, ok);
  }
};

// Dense row-major [rows][cols] with leading dimension ld (ld % 4 == 0).
struct DenseRows {
  using R = OffOk;
  using Cp = OffOk;
  using elem_t = float;
  const float* x;
  int ld;
  int rows;
  int cols;  // multiple of 4, or rows zero-padded to ld
  __device__ __forceinline__ R row(int r) const {
    return R{(uint32_t)r * (uint32_t)ld, r < rows};
  }
  __device__ __forceinline__ Cp col(int c) const { return Cp{(uint32_t)c, c < cols}; }
  struct It {
    uint32_t off;
    int r;
  };
  __device__ __forceinline__ It iter(int r0) const {
    return It{(uint32_t)(r0 < rows ? r0 : 0) * (uint32_t)ld, r0};
  }
  template <int STEP>
  __device__ __forceinline__ void advance(It& it) const {
    it.r += STEP;
    it.off += (uint32_t)(STEP * ld);
  }
  __device__ __forceinline__ R row_of(const It& it) const { return R{it.off, it.r < rows}; }
  using St = StF4;
  __device__ __forceinline__ St stage(const R& r, const Cp& c, bool in) const {
    const bool ok = in && r.ok && c.ok;
    return stage_f4(x + (r.off + c.off), ok);
  }
};

// Gradient of a VALID conv w.r.t. its input, one stride phase (ph, pw) per
// blockIdx.z: row r = (img, ih', iw') -> input pixel (S*ih'+ph, S*iw'+pw);
// column c = (kh', kw', co) -> tap (ph+S*kh', pw+S*kw'), output pixel
// (ih'-kh', iw'-kw').  Only taps that hit the phase are enumerated, so the
// stride-2 conv2 gradient does no zero work except at the borders.
template <int IH, int IW, int KH, int KW, int S, int COUT>
struct ConvTRows {
  static constexpr int OH = (IH - KH) / S + 1;
  static constexpr int OW = (IW - KW) / S + 1;
  static_assert(IH % S == 0 && IW % S == 0 && KH % S == 0 && KW % S == 0,
                "phase decomposition needs divisible extents");
  static constexpr int PH = IH / S;  // phase grid extent
  static constexpr int PW = IW / S;
  static constexpr int KHP = KH / S;  // taps per phase
  static constexpr int KWP = KW / S;
  static constexpr int COLS = KHP * KWP * COUT;
  static constexpr int L = PH * PW;  // rows per image per phase
  static_assert(COUT % 4 == 0, "");
  struct R {
    uint32_t off;
    int ihp, iwp;
    bool ok;
  };
  struct Cp {
    int off;
    int khp, kwp;
    bool ok;
  };
  const float* dy;  // [img][OH][OW][COUT]
  int rows;         // images * L

  __device__ __forceinline__ R row(int r0) const {
    const bool ok = r0 < rows;
    const uint32_t r = ok ? (uint32_t)r0 : 0u;
    const uint32_t img = r / L;
    const uint32_t p = r - img * L;
    const uint32_t ihp = p / PW;
    const uint32_t iwp = p - ihp * PW;
    return R{(img * (OH * OW) + ihp * OW + iwp) * COUT, (int)ihp, (int)iwp, ok};
  }
  __device__ __forceinline__ Cp col(int c0) const {
    const bool ok = c0 < COLS;
    const int c = ok ? c0 : 0;
    const int khp = c / (KWP * COUT);
    const int rem = c - khp * (KWP * COUT);
    const int kwp = rem / COUT;
    const int co = rem - kwp * COUT;
    return Cp{co - (khp * OW + kwp) * COUT, khp, kwp, ok};
  }
  using St = StF4;
  __device__ __forceinline__ St stage(const R& r, const Cp& c, bool in) const {
    const int oh = r.ihp - c.khp;
    const int ow = r.iwp - c.kwp;
    const bool ok = in & r.ok & c.ok & (oh >= 0) & (ow >= 0) & (oh < OH) & (ow < OW);
    return stage_f4(dy + (uint32_t)(r.off + c.off), ok);
  }
};

// ---------------------------------------------------------------------------
// Operands
// ---------------------------------------------------------------------------

// A row source as an operand: KC = true -> A(k, i) = src row i, column k
// (forward-style); KC = false -> A(k, i) = src row k, column i (reduction).
template <class Src, bool KC>
struct RowsOp {
  static constexpr bool KCONTIG = KC;
  using R = typename Src::R;
  using C = typename Src::Cp;
  Src src;
  __device__ __forceinline__ R row(int r) const { return src.row(r); }
  __device__ __forceinline__ C col(int c) const { return src.col(c); }
  using St = typename Src::St;
  __device__ __forceinline__ St stage(const R& r, const C& c, bool in) const {
    return src.stage(r, c, in);
  }
};
template <class Src>
using RowsAsK = RowsOp<Src, true>;
template <class Src>
using RowsAsI = RowsOp<Src, false>;

// B(k, j) over row k of [P | dY]:  j < kp -> P(k, j) (kp = 0 skips P),
// kp <= j < kp + cout_pad -> dY(k, j-kp), zero beyond.  The homogeneous
// coordinate needs no column: its row is the kernel's column sums and its
// column equals that row's P part by symmetry.  dY rows must be zero-padded from cout up to
// cout_pad <= ldy (the loss kernel writes its padding; conv/fc couts are
// multiples of 4), so every dY run is one unmasked float4.
template <class Src>
struct CatRowsI {
  static constexpr bool KCONTIG = false;
  struct R {
    typename Src::R p;
    uint32_t dyoff;
    bool ok;
  };
  struct C {
    typename Src::Cp p;
    int seg;  // 0 patch, 1 dY, 3 zero
    int jj;
  };
  Src src;
  int kp;
  const float* dy;
  int ldy;
  int cout;
  int cout_pad;  // multiple of 4
  int rows;
  __device__ __forceinline__ R row(int r) const {
    const bool ok = r < rows;
    return R{src.row(ok ? r : 0), ok ? (uint32_t)r * (uint32_t)ldy : 0u, ok};
  }
  __device__ __forceinline__ C col(int j) const {
    C c;
    c.p = src.col(j < kp ? j : 0);
    c.jj = j - kp;
    c.seg = j < kp ? 0 : (c.jj < cout_pad ? 1 : 3);
    return c;
  }
  // Row iterator over the P source and the dY rows together (symred3)
  struct It {
    typename Src::It p;
    uint32_t dyoff;
    int r;
  };
  __device__ __forceinline__ It iter(int r0) const {
    return It{src.iter(r0 < rows ? r0 : 0), (r0 < rows ? (uint32_t)r0 : 0u) * (uint32_t)ldy, r0};
  }
  template <int STEP>
  __device__ __forceinline__ void advance(It& it) const {
    src.template advance<STEP>(it.p);
    it.dyoff += (uint32_t)(STEP * ldy);
    it.r += STEP;
  }
  // A thread's column run resolved once: its segment's base pointer (P column
  // offset or dY column folded in) and validity, so a staged run costs one
  // 32-bit select of the row offset, one 64-bit add and the zero-run select.
  struct CB {
    const float* base;
    bool isp;
    bool ok;
  };
  __device__ __forceinline__ CB col_base(int j) const {
    const C c = col(j);
    if constexpr (std::is_same<typename Src::elem_t, float>::value) {
      if (c.seg == 0) return CB{src.x + c.p.off, true, c.p.ok};
    }
    return CB{dy + (c.seg == 1 ? c.jj : 0), false, c.seg == 1};
  }
  __device__ __forceinline__ StF4 stage_it(const It& it, const CB& cb, bool in) const {
    const bool ok = in && cb.ok && it.r < rows;
    const uint32_t roff = cb.isp ? it.p.off : it.dyoff;
    return *reinterpret_cast<const float4*>(ok ? cb.base + roff : zero_run());
  }
  // One float4 load per element: P and dY are both float rows, so the
  // column's segment (fixed per thread) just selects the address.
  using St = StF4;
  __device__ __forceinline__ St stage(const R& r, const C& c, bool in) const {
    // u8 patch sources only appear with kp == 0 (plain conv1 weight gradient)
    constexpr bool FP = std::is_same<typename Src::elem_t, float>::value;
    const bool rin = in && r.ok;
    const float* a = (c.seg == 1 && rin) ? dy + (r.dyoff + (uint32_t)c.jj) : zero_run();
    if constexpr (FP) a = (c.seg == 0 && rin && r.p.ok && c.p.ok) ? src.x + (r.p.off + c.p.off) : a;
    return *reinterpret_cast<const float4*>(a);
  }
};

// B(k, j) = M[k][j], row-major with leading dimension ld (dims K x N).
template <bool ALIGNED>
struct MatI {
  static constexpr bool KCONTIG = false;
  using R = OffOk;
  using C = int;
  const float* m;
  int ld;
  int K;
  int N;
  __device__ __forceinline__ R row(int k) const { return R{(uint32_t)k * (uint32_t)ld, k < K}; }
  __device__ __forceinline__ C col(int j) const { return j; }
  using St = StF4;
  __device__ __forceinline__ St stage(const R& r, const C& j, bool in) const {
    const bool ok = in && r.ok && j < N;
    const float* p = m + (r.off + (uint32_t)j);
    if constexpr (ALIGNED) {  // N % 4 == 0
      return stage_f4(p, ok);
    } else {
      return stage_tail(p, ok, N - j);
    }
  }
};

// B(k, j) = M[j][k]  (transposed access; k contiguous; dims K x N; ld%4==0,
// K%4==0 when ALIGNED, else per-element masking)
template <bool ALIGNED>
struct MatTK {
  static constexpr bool KCONTIG = true;
  using R = OffOk;
  using C = int;
  const float* m;
  int ld;
  int K;
  int N;
  __device__ __forceinline__ R row(int j) const { return R{(uint32_t)j * (uint32_t)ld, j < N}; }
  __device__ __forceinline__ C col(int k) const { return k; }
  using St = StF4;
  __device__ __forceinline__ St stage(const R& r, const C& k, bool in) const {
    const bool ok = in && r.ok && k < K;
    const float* p = m + (r.off + (uint32_t)k);
    if constexpr (ALIGNED) {  // K % 4 == 0
      return stage_f4(p, ok);
    } else {
      return stage_tail(p, ok, K - k);
    }
  }
};
using MatTKu = MatTK<false>;

// Conv weight as the A operand of the (transposed) input gradient, all S*S
// stride phases stacked: A(k = (kh',kw',co), i = (ph,pw,ci)) =
// W[ph+S*kh'][pw+S*kw'][ci][co].  Every phase of an input super-pixel
// (ih', iw') gathers the same dY neighbourhood (ConvTRows), so the phases are
// just more rows of one GEMM: S*S*CIN of them (128 for conv2) instead of CIN.
// The tap offset separates into an i part and a k part.
template <int KH, int KW, int S, int CIN, int COUT>
struct ConvTWeights {
  static constexpr bool KCONTIG = true;
  static constexpr int KHP = KH / S;
  static constexpr int KWP = KW / S;
  static constexpr int K = KHP * KWP * COUT;
  static constexpr int N = S * S * CIN;
  using R = OffOk;
  using C = OffOk;
  const float* w;  // HWIO
  __device__ __forceinline__ R row(int j) const {
    const int ph = j / (S * CIN);
    const int rem = j - ph * (S * CIN);
    const int pw = rem / CIN;
    const int ci = rem - pw * CIN;
    return R{(uint32_t)(((ph * KW + pw) * CIN + ci) * COUT), j < N};
  }
  __device__ __forceinline__ C col(int k) const {
    if (k >= K) return C{0, false};
    const int khp = k / (KWP * COUT);
    const int rem = k - khp * (KWP * COUT);
    const int kwp = rem / COUT;
    const int co = rem - kwp * COUT;
    return C{(uint32_t)(S * (khp * KW + kwp) * CIN * COUT + co), true};
  }
  using St = StF4;
  __device__ __forceinline__ St stage(const R& r, const C& c, bool in) const {
    const bool ok = in && r.ok && c.ok;
    return stage_f4(w + (r.off + c.off), ok);
  }
};

}  // namespace acmi
